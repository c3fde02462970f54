"""The CPU oracle (oracle/gz_oracle.c) against the reference's own outputs.

Pins the restatement before anything is checked against it: every stage of
the `--c` Butteraugli pass, the reference-vs-reference activity mask, the
per-block greedy zeroing orders and the libstdc++ std::sort tie order are
compared bit-for-bit with fixtures generated from oracle/_ref (the reference
compiled from /root/reference) by tests/golden/make_fixtures.py.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle_lib import COEFF_DTYPE, ZERO_VARIANTS, Fixture, Stages, fixture_cases, lib, ROOT

CASES = fixture_cases()


def bits_equal(a, b):
    a = np.asarray(a).ravel()
    b = np.asarray(b).ravel()
    assert a.shape == b.shape
    if a.dtype == np.float32:
        return np.array_equal(a.view(np.uint32), b.view(np.uint32))
    return np.array_equal(a, b)


@pytest.mark.parametrize("case", CASES)
def test_oracle_compare_stages_bit_exact(case):
    L = lib()
    F = Fixture(case)
    w, h, n = F.w, F.h, F.w * F.h
    rgb = F.rgb()
    ref = np.zeros(3 * n, np.float32)
    L.gzo_srgb_to_linear_planes(w, h, rgb, ref)
    L.gzo_opsin_dynamics(w, h, ref)
    assert bits_equal(ref, F.f32("ref_xyb.f32"))
    coeffs = F.i16("cand_coeffs.i16")
    srgb = np.zeros(3 * n, np.uint8)
    L.gzo_coeffs_to_srgb(w, h, coeffs, srgb)
    assert bits_equal(srgb, np.fromfile(F.path("cand_srgb.u8"), np.uint8))
    cand = np.zeros(3 * n, np.float32)
    L.gzo_srgb_to_linear_planes(w, h, srgb, cand)
    assert bits_equal(cand, F.f32("cand_linear.f32"))
    L.gzo_opsin_dynamics(w, h, cand)
    assert bits_equal(cand, F.f32("cand_xyb.f32"))
    rn = F.rw * F.rh
    sizes = dict(mhic0=3 * n, mhic1=3 * n, edge=3 * rn, block_dc=3 * rn, block_ac=3 * rn,
                 block_ac_lf=3 * rn, mask=3 * n, mask_dc=3 * n, combined=rn)
    arrs = {k: np.zeros(v, np.float32) for k, v in sizes.items()}
    st = Stages(**{k: a.ctypes.data for k, a in arrs.items()})
    dm = np.zeros(n, np.float32)
    assert L.gzo_diffmap(w, h, ref.copy(), cand.copy(), dm, ctypes.addressof(st)) == 1
    for k in sizes:
        assert bits_equal(arrs[k], F.f32(k + ".f32")), k
    assert bits_equal(dm, F.f32("distmap.f32"))
    d = L.gzo_compare(w, h, rgb, coeffs, dm)
    assert np.float32(d) == np.float32(F.meta["distance"])


@pytest.mark.parametrize("variant", ZERO_VARIANTS)
@pytest.mark.parametrize("case", CASES)
def test_oracle_block_zeroing_bit_exact(case, variant):
    """Zeroing orders for every (lookahead, comp_mask, new_zeroing_model)
    variant the reference was run with (processor.cc:376-487)."""
    L = lib()
    F = Fixture(case)
    w, h, n = F.w, F.h, F.w * F.h
    rgb = F.rgb()
    ref = np.zeros(3 * n, np.float32)
    L.gzo_srgb_to_linear_planes(w, h, rgb, ref)
    L.gzo_opsin_dynamics(w, h, ref)
    m = np.zeros(3 * n, np.float32)
    mdc = np.zeros(3 * n, np.float32)
    L.gzo_mask(w, h, ref, ref, m, mdc)
    assert bits_equal(m, F.f32("ref_mask.f32"))
    out = np.zeros(F.nb * 192, COEFF_DTYPE)
    la, mask, new_model = variant
    L.gzo_block_zeroing_orders(w, h, rgb, m, F.i16("cand_coeffs.i16"), F.i16("orig_coeffs.i16"),
                               ctypes.c_float(F.target), la, mask, new_model, out.ctypes.data)
    z = F.zero_order(None if variant == (3, 7, 1) else variant).ravel()
    assert np.array_equal(out["idx"], z["idx"])
    assert bits_equal(out["block_err"], z["block_err"])


SORT_HARNESS = r"""
#include <algorithm>
#include <cstdio>
#include <random>
#include <utility>
#include <vector>
extern "C" void gzo_sort_pairs(int* idx, float* key, int n);
int main() {
  std::mt19937 rng(12345);
  for (int t = 0; t < 4000; ++t) {
    int n = rng() % 200;
    int levels = 1 + rng() % (t % 3 == 0 ? 3 : 40);  // many ties in a third of the cases
    std::vector<std::pair<int, float>> v(n);
    std::vector<int> idx(n);
    std::vector<float> key(n);
    for (int i = 0; i < n; ++i) {
      v[i] = {i, static_cast<float>(rng() % levels) * 0.25f};
      idx[i] = v[i].first;
      key[i] = v[i].second;
    }
    if (t % 7 == 0) std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.second > b.second; });
    for (int i = 0; i < n; ++i) { idx[i] = v[i].first; key[i] = v[i].second; }
    std::sort(v.begin(), v.end(), [](const std::pair<int, float>& a, const std::pair<int, float>& b) {
      return a.second < b.second; });
    gzo_sort_pairs(idx.data(), key.data(), n);
    for (int i = 0; i < n; ++i)
      if (idx[i] != v[i].first) { std::printf("MISMATCH t=%d n=%d i=%d\n", t, n, i); return 1; }
  }
  std::printf("OK\n");
  return 0;
}
"""


def test_oracle_sort_matches_libstdcxx(tmp_path):
    lib()  # builds the oracle
    src = tmp_path / "sort_check.cc"
    src.write_text(SORT_HARNESS)
    exe = tmp_path / "sort_check"
    odir = os.path.join(ROOT, "oracle", "_build")
    subprocess.run(["g++", "-O2", "-std=c++17", str(src), "-o", str(exe), "-L", odir, "-lgz_oracle",
                    "-Wl,-rpath," + odir], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True)
    assert res.returncode == 0 and res.stdout.strip() == "OK", res.stdout
