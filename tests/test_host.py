"""Host-side checks that need no GPU.

- the C-ABI library loads and exports every symbol include/guetzli_hip.h
  declares (no compute calls);
- the product's initial encoder (EncodeRGBToJpeg: RGB->YUV16 + integer FDCT,
  q=1) reproduces the reference's coefficients;
- the product's host search loop, quantizer and JPEG writer, driven by the
  CPU oracle as comparator (tests/native/host_oracle_e2e.cc), reproduce the
  reference's output bytes end to end;
- the direct multithreaded JPEG writer equals the serial reference-shaped one;
- the synthetic frame generator is deterministic;
- without a GPU the compute entry points fail loudly (no CPU fallback).
"""
import hashlib
import json
import os
import re
import subprocess

import numpy as np
import pytest

from oracle_lib import GOLDEN, Fixture, fixture_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "guetzli_hip.h")).read()
    return sorted(set(re.findall(r"\b(gz_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(gz):
    L = gz.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    assert sorted(gz.EXPORTED_SYMBOLS) == syms
    for s in syms:
        assert hasattr(L, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", gz.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    for s in syms:
        assert s in exported, s


def test_quality_to_target(gz):
    # guetzli/quality.cc:46-57
    assert gz.butteraugli_score_for_quality(95) == pytest.approx(0.971769, abs=0)
    assert gz.butteraugli_score_for_quality(90) == pytest.approx(1.473608, abs=0)
    assert gz.butteraugli_score_for_quality(84) == pytest.approx(1.945456, abs=0)
    assert gz.butteraugli_score_for_quality(50) == pytest.approx(2.810761, abs=0)


@pytest.mark.parametrize("case", fixture_cases())
def test_rgb_to_coeffs_matches_reference(gz, case):
    F = Fixture(case)
    c = gz.rgb_to_coeffs(F.rgb(), F.w, F.h)
    assert np.array_equal(c, F.i16("orig_coeffs.i16"))


@pytest.mark.parametrize("case", fixture_cases())
def test_block_error_adjustment_weights_match_reference(gz, case):
    """ComputeBlockErrorAdjustmentWeights (butteraugli_comparator.cc:169-233)
    of the reference's own distance map, both directions, radius 1..4: the
    committed weights_d<dir>_r<r>.f32 dumps, bit for bit."""
    F = Fixture(case)
    dm = F.f32("distmap.f32")
    for direction in (-1, 1):
        for rb in range(1, 5):
            exp = F.f32("weights_d%+d_r%d.f32" % (direction, rb))
            got = gz.block_error_adjustment_weights(F.w, F.h, F.target, direction, rb, dm)
            assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (direction, rb)


def _e2e_cases():
    cases = []
    for name, e in sorted(MANIFEST["e2e"].items()):
        if e["w"] * e["h"] <= 100 * 100 or name.startswith("bees_q"):
            cases.append(name)
    return cases


def _e2e_params_cases():
    return [("e2e_params", n) for n, e in sorted(MANIFEST.get("e2e_params", {}).items())
            if e["w"] * e["h"] <= 100 * 100]


def _e2e_edge_cases():
    return [("e2e_edge", n) for n in sorted(MANIFEST.get("e2e_edge", {}))]


@pytest.mark.parametrize("section,name", [("e2e", n) for n in _e2e_cases()] + _e2e_params_cases()
                         + _e2e_edge_cases())
def test_host_loop_with_oracle_comparator_bit_exact(host_e2e_bin, section, name, tmp_path):
    """Product host loop + CPU-oracle comparator == the reference's bytes,
    including the Params variants (old zeroing model, lookahead 1 / 2) and
    the edge paths (images under 32 px, quality below 84, force_420 on
    content without chroma)."""
    e = MANIFEST[section][name]
    out = tmp_path / "out.jpg"
    res = subprocess.run([host_e2e_bin, os.path.join(GOLDEN, e["input"]), str(e["w"]), str(e["h"]),
                          str(e["quality"]), str(out)] +
                         ["%s=%d" % kv for kv in sorted(e.get("params", {}).items())],
                         capture_output=True, text=True, timeout=600)
    if e.get("fail"):
        # guetzli::Process returns false (processor.cc:939-945)
        assert res.returncode == 3 and "2.0" in res.stderr, res.stderr
        return
    assert res.returncode == 0, res.stderr
    info = json.loads(res.stdout)
    assert info["iters"] == e["iters"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == e["sha256"]


@pytest.mark.parametrize("w,h,seed,scale", [(640, 360, 3, 1), (333, 197, 5, 7), (64, 8, 1, 2),
                                            (1920, 1080, 0, 3)])
def test_direct_writer_matches_serial_writer(gz, writer_check_bin, tmp_path, w, h, seed, scale):
    """The multithreaded CoeffImage encoder is byte-identical to
    SaveToJpegData + WriteJpeg (reference jpeg_data_writer.cc path)."""
    rgb = tmp_path / "in.rgb"
    rgb.write_bytes(gz.synthetic_frame(seed, w, h).tobytes())
    for threads in ("1", "3"):
        env = dict(os.environ, GZ_HOST_THREADS=threads)
        res = subprocess.run([writer_check_bin, str(rgb), str(w), str(h), str(scale)], env=env,
                             capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stdout + res.stderr
        assert json.loads(res.stdout)["equal"] == 1


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_lazy_sort_matches_libstdcxx_sort(lazy_sort_check_bin, seed):
    """The prefix-on-demand sort of the search loop's change order reproduces
    std::sort's permutation, ties included."""
    res = subprocess.run([lazy_sort_check_bin, str(seed)], capture_output=True, text=True,
                         timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    assert json.loads(res.stdout)["bad"] == 0


def test_host_pool_concurrent_and_nested(pool_check_bin):
    res = subprocess.run([pool_check_bin], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and res.stdout.startswith("ok"), res.stdout + res.stderr


def test_synthetic_frames_deterministic(gz):
    for name, e in MANIFEST.get("synthetic", {}).items():
        if e["w"] * e["h"] > 640 * 360:
            continue
        f = gz.synthetic_frame(e["seed"], e["w"], e["h"])
        if e.get("mode") == "gray":  # (make_synthetic_fixtures.py case_rgb)
            f = np.ascontiguousarray(f[:, :, 1:2].repeat(3, axis=2))
        assert f.shape == (e["h"], e["w"], 3)
        assert hashlib.sha256(f.tobytes()).hexdigest() == e["input_sha256"], name
        assert f.min() >= 16 and f.max() <= 240


def test_bad_arguments_fail_loudly(gz):
    with pytest.raises(gz.GuetzliError):
        gz.rgb_to_coeffs(np.zeros(10, np.uint8), 4, 4)
    with pytest.raises(gz.GuetzliError):
        gz.process(np.zeros(3 * 64 * 64, np.uint8), 64, 64, gz.Params(butteraugli_target=3.0))


def test_no_cpu_fallback_without_gpu(gz, gpu_available):
    if gpu_available:
        pytest.skip("a GPU is present")
    rgb = np.zeros(3 * 64 * 64, np.uint8)
    with pytest.raises(gz.GuetzliError) as e:
        gz.ButteraugliComparator(64, 64, rgb, 1.0)
    assert e.value.status == 2
    with pytest.raises(gz.GuetzliError) as e:
        gz.process(rgb, 64, 64, gz.Params.for_quality(95))
    assert e.value.status == 2


@pytest.mark.parametrize("name", sorted(n for n, e in MANIFEST.get("e2e_edge", {}).items()
                                        if e.get("fail") or e["w"] < 32 or e["h"] < 32))
def test_process_edge_paths_without_device(gz, name):
    """The two edge paths of guetzli::Process that need no Butteraugli,
    through the product's C ABI: images under 32 px in either dimension get
    the q=1 encode as their output (processor.cc:1170-1181 -> :971-977), and
    quality below 84 is refused (:939-945) -- with or without a device."""
    e = MANIFEST["e2e_edge"][name]
    rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    p = gz.Params.for_quality(e["quality"])
    if e.get("fail"):
        with pytest.raises(gz.GuetzliError) as err:
            gz.process(rgb, e["w"], e["h"], p)
        assert err.value.status == 1
        return
    data, st = gz.process(rgb, e["w"], e["h"], p, return_stats=True)
    assert st.iterations == e["iters"] == 0
    assert hashlib.sha256(data).hexdigest() == e["sha256"]


@pytest.mark.parametrize("decades", ["1", "3", "32"])
def test_speculative_tail_batches_bit_exact(host_e2e_bin, decades, tmp_path):
    """The back end's tail runs in speculative batches (codes of several
    decades built at once, changes past the break undone); the batch size
    must not change a byte or an iteration."""
    e = MANIFEST["e2e"]["bees_q95"]
    out = tmp_path / "out.jpg"
    res = subprocess.run([host_e2e_bin, os.path.join(GOLDEN, e["input"]), str(e["w"]), str(e["h"]),
                          str(e["quality"]), str(out)], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, GZ_SPEC_DECADES=decades))
    assert res.returncode == 0, res.stderr
    assert json.loads(res.stdout)["iters"] == e["iters"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == e["sha256"]


def test_staged_allgather_buffer_handling(collectives_check_bin):
    """host/rccl_collectives.h: the native RCCL gz_collectives' staging
    (grow-only device / pinned buffers, zero-byte exchanges, rank order,
    the variable-size gather on top, every buffer freed) over a host-memory
    transport with three ranks as threads."""
    res = subprocess.run([collectives_check_bin], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0 and res.stdout.startswith("ok"), res.stdout + res.stderr
