"""GPU parity: the HIP path (through the C ABI) against the reference.

Bit-exact against fixtures produced by the reference itself (oracle/_ref):
every stage of one Butteraugli pass, the block-corner activity mask, the
per-block greedy zeroing orders, and end-to-end JPEG bytes (sha256) of
`guetzli --c` on bees.png and synthetic frames.  Larger frames are checked
against the CPU oracle at sizes it finishes in seconds.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_lib import COEFF_DTYPE, GOLDEN, ZERO_VARIANTS, Fixture, fixture_cases, lib as oracle

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
STAGES = ["cand_linear", "cand_xyb", "mhic0", "mhic1", "edge", "block_dc", "block_ac",
          "block_ac_lf", "mask", "mask_dc", "combined", "distmap"]
FIXTURE_FILE = {"block_dc": "block_dc.f32", "block_ac": "block_ac.f32",
                "block_ac_lf": "block_ac_lf.f32", "distmap": "distmap.f32"}


def bits_equal(a, b):
    a = np.asarray(a, dtype=np.float32).ravel()
    b = np.asarray(b, dtype=np.float32).ravel()
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def mismatch(a, b):
    a = np.asarray(a, dtype=np.float32).ravel()
    b = np.asarray(b, dtype=np.float32).ravel()
    bad = a.view(np.uint32) != b.view(np.uint32)
    return "%d/%d differ, max |d| %.3g" % (bad.sum(), bad.size,
                                          np.max(np.abs(a.astype(np.float64) - b)) if bad.any() else 0)


@pytest.fixture(scope="module", autouse=True)
def need_gpu(gz):
    if gz.device_count() == 0:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")


@pytest.mark.parametrize("case", fixture_cases())
def test_compare_stages_bit_exact(gz, case):
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    st = cmp.compare_stages(F.i16("cand_coeffs.i16"))
    bad = []
    for name in STAGES:
        ref = F.f32(FIXTURE_FILE.get(name, name + ".f32"))
        if not bits_equal(st[name], ref):
            bad.append("%s: %s" % (name, mismatch(st[name], ref)))
    assert not bad, "; ".join(bad)
    assert np.float32(st["distance"]) == np.float32(F.meta["distance"])
    # per-block maxima of the distance map (ComputeBlockErrorAdjustmentWeights input)
    dm = F.f32("distmap.f32").reshape(F.h, F.w)
    bm = np.zeros(F.nb, np.float32)
    for by in range(F.bh):
        for bx in range(F.bw):
            bm[by * F.bw + bx] = max(0.0, dm[8 * by:8 * by + 8, 8 * bx:8 * bx + 8].max())
    assert bits_equal(cmp.block_max(), bm)


PROD_STAGES = ["mhic0", "mhic1", "edge", "block_dc", "block_ac", "distmap"]


@pytest.mark.parametrize("case", fixture_cases())
def test_production_stages_bit_exact(gz, case):
    """The planes of the search's own kernel variants (k_block_diff2 with the
    corner edge term fused in, k_combine_channels with the low-frequency term
    and the subsampled B mask, the LUT epilogue of the vertical blur) against
    the reference's stage dumps -- not the stand-alone dump kernels that
    compare_stages switches to."""
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    st = cmp.compare_stages_production(F.i16("cand_coeffs.i16"))
    bad = []
    for name in PROD_STAGES:
        ref = F.f32(FIXTURE_FILE.get(name, name + ".f32"))
        if not bits_equal(st[name], ref):
            bad.append("%s: %s" % (name, mismatch(st[name], ref)))
    assert not bad, "; ".join(bad)
    assert np.float32(st["distance"]) == np.float32(F.meta["distance"])
    # the search's plain (graph-launched) pass and distmap() agree with it
    assert np.float32(cmp.compare(F.i16("cand_coeffs.i16"))) == np.float32(F.meta["distance"])
    assert bits_equal(cmp.distmap(), st["distmap"])


def test_production_stages_reject_dump_only_planes(gz):
    """Planes only the dump kernels produce are refused, not silently zero."""
    F = Fixture(fixture_cases()[0])
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    n = F.w * F.h
    arr = np.zeros(3 * n, np.float32)
    st = gz._Stages(mask=arr.ctypes.data)
    rc = gz.lib().gz_comparator_compare_stages_production(cmp._h, gz._ptr(F.i16("cand_coeffs.i16")),
                                                           gz.ctypes.byref(st), None)
    assert rc != 0 and "only mhic0" in gz.lib().gz_last_error().decode()


def test_420_chroma_planes_wrap_to_pixel_bytes(gz):
    """k_coeffs_to_srgb8's 4:2:0 input: the factor-2 chroma planes are 16-bit
    state that wraps (the inverse upsampler can drive a pixel below 0 or past
    4095), and ToPixels keeps the low byte of (p + 8 - (x & 1)) >> 4
    (output_image.cc:83, a uint8_t cast).  Planes drawn over all 65536 values
    (both wrap directions, both x parities) must give the candidate the
    oracle forms from the same bytes -- compared as whole distance maps."""
    import ctypes
    L = oracle()
    L.gzo_ycbcr_to_rgb.argtypes = [ctypes.c_void_p]
    L.gzo_ycbcr_to_rgb.restype = None
    w, h = 96, 64
    rng = np.random.default_rng(42)
    rgb = gz.synthetic_frame(3, w, h)
    bw, bh = w // 8, h // 8
    y = np.zeros((bh * bw, 64), np.int16)
    y[:, 0] = rng.integers(-600, 600, size=bh * bw)
    y[:, 1:10] = rng.integers(-40, 40, size=(bh * bw, 9))
    planes = rng.integers(0, 65536, size=(2, h, w)).astype(np.uint16)
    # make sure the wrap edges are present: just below 0, around 4095/4096
    planes[0, 0, :8] = [0xFFF0, 0xFFF7, 0xFFF8, 0xFFFF, 4087, 4088, 4095, 4104]
    planes[1, 1, :8] = [4104, 4095, 4088, 4087, 0xFFFF, 0xFFF8, 0xFFF7, 0xFFF0]
    xs = np.arange(w)[None, :]
    byte = ((planes.astype(np.int64) + 8 - (xs & 1)) >> 4) & 0xff
    assert (byte[0, 0, :8] == [255, 255, 0, 0, 255, 255, 0, 0]).all()  # 4095 -> 255, 4096 -> 0 (wrapped)
    ypix = np.zeros((h, w), np.uint8)
    for b in range(bh * bw):
        out = np.zeros(64, np.uint8)
        L.gzo_block_idct(y[b], out)
        by, bx = divmod(b, bw)
        ypix[8 * by:8 * by + 8, 8 * bx:8 * bx + 8] = out.reshape(8, 8)
    exp = np.stack([ypix, byte[0], byte[1]], axis=-1).astype(np.uint8).copy()
    for p in range(w * h):
        L.gzo_ycbcr_to_rgb(exp.ctypes.data + 3 * p)
    cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
    d420 = cmp.compare_420(y, planes[0], planes[1])
    bm420 = cmp.block_max()
    dm420 = cmp.distmap()
    dr = ctypes.c_float()
    assert gz.lib().gz_comparator_compare_rgb(cmp._h, gz._ptr(exp.reshape(-1)), ctypes.byref(dr)) == 0
    assert np.float32(d420) == np.float32(dr.value)
    assert bits_equal(bm420, cmp.block_max())
    assert bits_equal(dm420, cmp.distmap()), mismatch(dm420, cmp.distmap())
    # a saturating byte (what a packed saturating store would give) is a
    # different candidate: the test can tell the two semantics apart
    sat = np.clip((planes.astype(np.int64) + 8 - (xs & 1)) >> 4, 0, 255)
    assert (sat != byte).mean() > 0.5


@pytest.mark.parametrize("case", fixture_cases())
def test_block_mask_scale_bit_exact(gz, case):
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    scale = cmp.start_block_comparisons()
    m = F.planes("ref_mask.f32")
    exp = np.stack([m[:, 8 * (b // F.bw), 8 * (b % F.bw)] for b in range(F.nb)])
    assert bits_equal(scale, exp)


@pytest.mark.parametrize("variant", ZERO_VARIANTS)
@pytest.mark.parametrize("case", fixture_cases())
def test_block_zeroing_orders_bit_exact(gz, case, variant):
    """Device zeroing orders == the reference's for every committed
    (lookahead, comp_mask, new_zeroing_model) variant; the candidate passes
    all components (the unsearched ones keep their values in the pixels)."""
    F = Fixture(case)
    la, mask, new_model = variant
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    out = cmp.block_zeroing_orders(F.i16("cand_coeffs.i16"), F.i16("orig_coeffs.i16"), F.target,
                                   comp_mask=mask, lookahead=la, new_zeroing_model=bool(new_model))
    z = F.zero_order(None if variant == (3, 7, 1) else variant)
    assert np.array_equal(out["idx"], z["idx"]), "idx differ in %d blocks" % (
        (out["idx"] != z["idx"]).any(axis=1).sum())
    assert bits_equal(out["block_err"], z["block_err"]), mismatch(out["block_err"], z["block_err"])


@pytest.mark.parametrize("case", fixture_cases())
def test_compare_blocks_bit_exact(gz, case):
    """SwitchBlock + CompareBlock (butteraugli_comparator.cc:85-163) through
    gz_comparator_compare_blocks: every block with its current coefficients
    and with one random non-zero coefficient zeroed equals the oracle's
    double bit for bit (edge blocks included)."""
    F = Fixture(case)
    L = oracle()
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    cur = F.i16("cand_coeffs.i16").reshape(3, F.nb, 64)
    mask = F.f32("ref_mask.f32")
    rgb = np.ascontiguousarray(F.rgb(), dtype=np.uint8).ravel()
    rng = np.random.default_rng(17)
    blocks, cands = [], []
    for b in range(F.nb):
        blk = np.ascontiguousarray(cur[:, b, :]).copy()
        blocks.append(b)
        cands.append(blk.copy())
        nz = np.flatnonzero(blk.reshape(-1))
        if nz.size:
            blk.reshape(-1)[rng.choice(nz)] = 0
            blocks.append(b)
            cands.append(blk)
    cands = np.stack(cands).astype(np.int16)
    err = cmp.compare_blocks(np.array(blocks), cands)
    ref = np.array([L.gzo_compare_block(F.w, F.h, rgb, mask, b, np.ascontiguousarray(c).ravel())
                    for b, c in zip(blocks, cands)], np.float64)
    bad = np.flatnonzero(err.view(np.uint64) != ref.view(np.uint64))
    assert bad.size == 0, "%d/%d differ, e.g. block %d: %r vs %r" % (
        bad.size, err.size, blocks[bad[0]], err[bad[0]], ref[bad[0]])


@pytest.mark.parametrize("case", fixture_cases())
def test_comparator_distmap_bit_exact(gz, case):
    """Comparator::distmap() after a Compare == the reference's map."""
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    d = cmp.compare(F.i16("cand_coeffs.i16"))
    assert np.float32(d) == np.float32(F.meta["distance"])
    ref = F.f32("distmap.f32")
    assert bits_equal(cmp.distmap(), ref), mismatch(cmp.distmap(), ref)


@pytest.mark.parametrize("case", fixture_cases())
def test_device_fdct_matches_reference(gz, case):
    """EncodeRGBToJpeg's q=1 coefficients computed by the device kernel equal
    the reference's (fixture orig_coeffs)."""
    F = Fixture(case)
    cmp = gz.ButteraugliComparator(F.w, F.h, F.rgb(), F.target)
    assert np.array_equal(cmp.original_coeffs(), F.i16("orig_coeffs.i16"))


@pytest.mark.parametrize("w,h,seed", [(1920, 1080, 0), (333, 197, 8), (64, 8, 3)])
def test_device_fdct_matches_host_encoder(gz, w, h, seed):
    """Device FDCT == the host restatement on ragged and full-HD frames."""
    rgb = gz.synthetic_frame(seed, w, h)
    cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
    assert np.array_equal(cmp.original_coeffs(), gz.rgb_to_coeffs(rgb, w, h))


def _quantized(gz, rgb, w, h, quant):
    c = gz.rgb_to_coeffs(rgb, w, h).reshape(3, -1, 64).astype(np.int32)
    qq = quant[:, None, :]
    r = np.fmod(c, qq)
    return (c + np.where(2 * r > qq, qq - r, np.where(-2 * r > qq, -qq - r, -r))).astype(np.int16)


@pytest.mark.parametrize("w,h,seed", [(333, 197, 2), (1920, 1080, 0), (64, 8, 5), (97, 41, 9)])
def test_device_jpeg_writer_matches_host_writer(gz, w, h, seed):
    """Device entropy coding (k_jpeg_stage/bits/emit + host tables) ==
    SaveToJpegData + WriteJpeg on the host, byte for byte: random quant
    tables (incl. 16-bit ones), then with all chroma cleared (1 component)."""
    rng = np.random.default_rng(seed)
    rgb = gz.synthetic_frame(seed, w, h)
    cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
    for trial in range(4):
        hi = (8, 40, 300, 2000)[trial]
        quant = rng.integers(1, hi, size=(3, 64)).astype(np.int32)
        co = _quantized(gz, rgb, w, h, quant)
        if trial == 3:
            co[1:] = 0
        dev = cmp.write_jpeg(co.reshape(-1), quant)
        host = gz.write_jpeg_host(co.reshape(-1), quant, w, h)
        assert dev == host, "trial %d: %d vs %d bytes" % (trial, len(dev), len(host))


def _occupy_lib():
    """tests/native/occupy.hip (built by __graft_entry__.build / conftest)."""
    import ctypes
    L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build",
                                 "libgz_occupy.so"))
    L.occupy_start.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.occupy_start.restype = ctypes.c_void_p
    L.occupy_held.argtypes = [ctypes.c_void_p]
    L.occupy_release.argtypes = [ctypes.c_void_p]
    return L


_OCCUPY_RUN = r"""
import concurrent.futures, ctypes, json, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import guetzli_amd as gz
spare_xcd = int(sys.argv[3])
ncoders = int(sys.argv[4]) if len(sys.argv) > 4 else 3
L = ctypes.CDLL(sys.argv[2])
L.occupy_start.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
L.occupy_start.restype = ctypes.c_void_p
L.occupy_held.argtypes = [ctypes.c_void_p]
L.occupy_release.argtypes = [ctypes.c_void_p]
w, h = 1920, 1080
rng = np.random.default_rng(31 + spare_xcd)
rgb = gz.synthetic_frame(4, w, h)
quant = rng.integers(1, 40, size=(3, 64)).astype(np.int32)
c = gz.rgb_to_coeffs(rgb, w, h).reshape(3, -1, 64).astype(np.int32)
qq = quant[:, None, :]
r = np.fmod(c, qq)
co = (c + np.where(2 * r > qq, qq - r, np.where(-2 * r > qq, -qq - r, -r))).astype(np.int16).reshape(-1)
host = gz.write_jpeg_host(co, quant, w, h)
cmps = [gz.ButteraugliComparator(w, h, rgb, 1.0) for _ in range(ncoders)]
warm = all(cm.write_jpeg(co, quant) == host for cm in cmps)
occ = L.occupy_start(0, spare_xcd, 20000)
assert occ, "occupy_start failed"
released = False
try:
    time.sleep(0.2)
    held = L.occupy_held(occ)
    with concurrent.futures.ThreadPoolExecutor(max_workers=ncoders) as ex:
        futs = [ex.submit(cm.write_jpeg, co, quant) for cm in cmps]
        done, pending = concurrent.futures.wait(futs, timeout=12.0)
        still_held = L.occupy_held(occ)
        assert L.occupy_release(occ) == 0
        released = True
        outs = [f.result(timeout=60) for f in futs]
finally:
    if not released:
        L.occupy_release(occ)
print(json.dumps({"warm": warm, "held": held, "still_held": still_held, "pending": len(pending),
                  "same": [o == host for o in outs]}))
"""


@pytest.mark.parametrize("spare_xcd,queues,coders", [(0, 16, 3), (5, 16, 3)])
def test_coder_forward_progress_under_occupancy(spare_xcd, queues, coders):
    """k_jpeg_code never waits without bound on a workgroup that has not been
    dispatched (jpeg_kernels.inc: look-back fallback + seam counters).
    Another stream's kernel holds every CU but those of one XCD (one
    workgroup with all 160 KiB of LDS per CU); three engines code a 1080p
    candidate at once while it holds: every coder finishes while the CUs are
    still held (only then is the holding kernel released), with the host
    writer's bytes.  In a process of its own with 16 hardware queues: with
    the default 4, a coder's stream may share the holding kernel's queue and
    then waits behind it in queue order (the runtime's stream-to-queue
    assignment, not the coder) -- round 5 saw exactly that.  At the
    shipped default of 4 queues the holding kernel itself could not be
    placed on a queue of its own (round 6: with two coders it never started
    while they ran, `held` 0), so forward progress there is argued from the
    kernel's bounded waits, not tested."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(here, "..", "guetzli-cuda-opencl_amd", "python")
    lib = os.path.join(here, "_build", "libgz_occupy.so")
    res = subprocess.run([sys.executable, "-c", _OCCUPY_RUN, pkg, lib, str(spare_xcd), str(coders)],
                         env=dict(os.environ, GPU_MAX_HW_QUEUES=str(queues)), capture_output=True, text=True,
                         timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["warm"], out
    assert out["held"] >= 160, "the holding kernel held only %d CUs" % out["held"]
    assert out["pending"] == 0, "%d coders did not finish while the CUs were held" % out["pending"]
    assert out["still_held"] >= 160, "the holding kernel let go early: %r" % out
    assert all(out["same"]), out


def _jpeg_sha(gz, rgb, w, h, q):
    data, stats = gz.process(rgb, w, h, gz.Params.for_quality(q), return_stats=True)
    # back-end candidates that cannot win are not coded; the size bound they
    # are judged by is the coder's exact bit count for every coded one
    detail = gz.last_process_detail()
    assert detail.get("scan_bound_mismatches", 0) == 0, detail
    return hashlib.sha256(data).hexdigest(), stats


@pytest.mark.parametrize("name", sorted(MANIFEST["e2e"]))
def test_process_reference_known_answers(gz, name):
    e = MANIFEST["e2e"][name]
    rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    sha, stats = _jpeg_sha(gz, rgb, e["w"], e["h"], e["quality"])
    assert stats.iterations == e["iters"]
    assert sha == e["sha256"]
    if name == "bees_q90":
        # (the reference's log of this search: 19 of its 21 back-end
        # candidates score far above the best output so far)
        assert gz.last_process_detail().get("scans_skipped", 0) >= 10


@pytest.mark.parametrize("name", sorted(MANIFEST.get("synthetic", {})))
def test_process_synthetic_known_answers(gz, name):
    e = MANIFEST["synthetic"][name]
    rgb = gz.synthetic_frame(e["seed"], e["w"], e["h"])
    if e.get("mode") == "gray":  # (tests/golden/make_synthetic_fixtures.py case_rgb)
        rgb = np.ascontiguousarray(rgb[:, :, 1:2].repeat(3, axis=2))
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == e["input_sha256"]
    sha, stats = _jpeg_sha(gz, rgb, e["w"], e["h"], e["quality"])
    assert stats.iterations == e["iters"]
    assert sha == e["sha256"]


@pytest.mark.parametrize("w,h,seed", [(256, 256, 7), (333, 197, 8)])
def test_compare_matches_oracle_on_synthetic(gz, w, h, seed):
    """Full-pass distance map vs the CPU oracle on frames it finishes in ~1 s."""
    L = oracle()
    rgb = gz.synthetic_frame(seed, w, h)
    coeffs = gz.rgb_to_coeffs(rgb, w, h)
    rng = np.random.default_rng(seed)
    q = rng.integers(1, 12, size=(3, 64))
    nb = ((w + 7) // 8) * ((h + 7) // 8)
    c = coeffs.reshape(3, nb, 64).astype(np.int32)
    qq = q[:, None, :]
    r = np.fmod(c, qq)
    delta = np.where(2 * r > qq, qq - r, np.where(-2 * r > qq, -qq - r, -r))
    cand = (c + delta).astype(np.int16).ravel()
    cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
    st = cmp.compare_stages(cand)
    dm = np.zeros(w * h, np.float32)
    d = L.gzo_compare(w, h, rgb.ravel(), cand, dm)
    assert bits_equal(st["distmap"], dm), mismatch(st["distmap"], dm)
    assert np.float32(st["distance"]) == np.float32(d)
    # the production (fused) variants: every distance-map pixel
    pr = cmp.compare_stages_production(cand)
    assert bits_equal(pr["distmap"], dm), mismatch(pr["distmap"], dm)
    for k in ("edge", "block_dc", "block_ac"):
        assert bits_equal(pr[k], st[k]), "%s: %s" % (k, mismatch(pr[k], st[k]))


@pytest.mark.parametrize("w,h,seed", [(256, 256, 7), (333, 197, 8), (517, 389, 4), (700, 301, 5),
                                      (519, 250, 6), (518, 45, 2)])
def test_compare_fast_path_matches_oracle(gz, w, h, seed):
    """The Compare pass as the search runs it (graph-launched, no stage dumps,
    the B activity mask evaluated only where CombineChannels samples it):
    distance and per-block maxima equal the CPU oracle's.  Sizes cover both
    parities of the (w-5)x(h-5) crop, a last 128-column blur group of one
    column (519) and rows / columns past the blurred grid."""
    L = oracle()
    rgb = gz.synthetic_frame(seed, w, h)
    coeffs = gz.rgb_to_coeffs(rgb, w, h)
    rng = np.random.default_rng(seed)
    q = rng.integers(1, 12, size=(3, 64))
    nb = ((w + 7) // 8) * ((h + 7) // 8)
    c = coeffs.reshape(3, nb, 64).astype(np.int32)
    qq = q[:, None, :]
    r = np.fmod(c, qq)
    cand = (c + np.where(2 * r > qq, qq - r, np.where(-2 * r > qq, -qq - r, -r))).astype(np.int16).ravel()
    cmp = gz.ButteraugliComparator(w, h, rgb, 1.0)
    d = cmp.compare(cand)
    d2 = cmp.compare(cand)  # graph replay
    dm = np.zeros(w * h, np.float32)
    dref = L.gzo_compare(w, h, rgb.ravel(), cand, dm)
    assert np.float32(d) == np.float32(dref) and np.float32(d2) == np.float32(dref)
    bw, bh = (w + 7) // 8, (h + 7) // 8
    dm = dm.reshape(h, w)
    bm = np.array([max(0.0, dm[8 * by:8 * by + 8, 8 * bx:8 * bx + 8].max())
                   for by in range(bh) for bx in range(bw)], np.float32)
    assert bits_equal(cmp.block_max(), bm)


def _known_answer_jobs(gz):
    """Distinct inputs with the reference's known answers: synthetic 1080p
    q95 seeds 0..7 (BASELINE configs[1]/[3] frames) and bees at q95/q90/q84."""
    jobs = []
    for s in range(8):
        e = MANIFEST["synthetic"]["synth_1920x1080_s%d_q95" % s]
        jobs.append(("synth_s%d" % s, gz.synthetic_frame(s, 1920, 1080), 1920, 1080, 95, e))
    for name in ("bees_q95", "bees_q90", "bees_q84"):
        e = MANIFEST["e2e"][name]
        rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
        jobs.append((name, rgb, e["w"], e["h"], e["quality"], e))
    return jobs


@pytest.mark.parametrize("threads", [8, 11])
def test_concurrent_encodes_known_answers(gz, threads):
    """configs[3]'s per-GPU shape: several encodes in flight on one GPU at
    once (one host thread + engine + stream each, sharing the engine pool,
    the host worker pool and the device entropy coder), inputs in HBM
    (gz_process_rgb_device, as bench.py) and in host memory: every output is
    byte-identical to the reference's, twice over (the second round reuses
    pooled engines)."""
    import concurrent.futures
    import ctypes
    jobs = _known_answer_jobs(gz)[:threads]
    # device copies of the inputs through the HIP runtime the library itself
    # uses (already loaded with it: same soname)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    dev = []
    for j in jobs:
        a = np.ascontiguousarray(j[1]).reshape(-1)
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), a.nbytes) == 0
        assert hip.hipMemcpy(p, a.ctypes.data, a.nbytes, 1) == 0  # hipMemcpyHostToDevice
        dev.append(p)

    def run(i):
        name, rgb, w, h, q, e = jobs[i]
        p = gz.Params.for_quality(q)
        if i % 2 == 0:
            data, st = gz.process_device(dev[i].value, w, h, p, return_stats=True)
        else:
            data, st = gz.process(rgb, w, h, p, return_stats=True)
        return name, hashlib.sha256(data).hexdigest(), st.iterations

    try:
        with concurrent.futures.ThreadPoolExecutor(max_workers=threads) as ex:
            for _ in range(2):
                for name, sha, iters in ex.map(run, range(len(jobs))):
                    e = jobs[[j[0] for j in jobs].index(name)][5]
                    assert (sha, iters) == (e["sha256"], e["iters"]), name
    finally:
        for p in dev:
            hip.hipFree(p)


def test_engine_pool_trim(gz):
    """Encodes leave their engines pooled; trim releases them (LRU, byte
    accounting) and the next encode re-creates one with the same bytes."""
    e = MANIFEST["e2e"]["bees_q95"]
    rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    gz.process(rgb, e["w"], e["h"], gz.Params.for_quality(95))
    assert gz.engine_pool_idle_bytes() > 0
    freed = gz.engine_pool_trim(0)
    assert freed > 0 and gz.engine_pool_idle_bytes() == 0
    data = gz.process(rgb, e["w"], e["h"], gz.Params.for_quality(95))
    assert hashlib.sha256(data).hexdigest() == e["sha256"]
    assert gz.engine_pool_idle_bytes() > 0


@pytest.mark.parametrize("name", sorted(MANIFEST.get("e2e_params", {})))
def test_process_params_variants_known_answers(gz, name):
    """Params::new_zeroing_model = false and zeroing_greedy_lookahead 1 / 2
    (processor.cc:400-405, :416) end to end: the reference's bytes."""
    e = MANIFEST["e2e_params"][name]
    rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    p = gz.Params.for_quality(e["quality"])
    p.zeroing_greedy_lookahead = e["params"].get("lookahead", 3)
    p.new_zeroing_model = bool(e["params"].get("new_model", 1))
    data, st = gz.process(rgb, e["w"], e["h"], p, return_stats=True)
    assert st.iterations == e["iters"]
    assert hashlib.sha256(data).hexdigest() == e["sha256"]


@pytest.mark.parametrize("kind", ["bees", "synthetic", "gray"])
def test_device_coded_original_output_matches_host_writer(gz, kind, monkeypatch):
    """The reference writes the original image first (processor.cc:965-967,
    kept when no candidate scores better).  For RGB input the library codes
    it on the device with the original's own headers; the hook compares
    those bytes with the host writer's (the gray case, whose chroma
    SaveToJpegData would drop, takes the host writer itself)."""
    monkeypatch.setenv("GZ_CHECK_ORIGINAL_OUTPUT", "1")
    if kind == "bees":
        e = MANIFEST["e2e"]["bees_q90"]
        rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
        w, h = e["w"], e["h"]
    elif kind == "synthetic":
        w, h = 333, 197
        rgb = gz.synthetic_frame(11, w, h)
    else:
        w, h = 96, 64
        g = gz.synthetic_frame(12, w, h).reshape(h, w, 3)[:, :, :1]
        rgb = np.ascontiguousarray(np.repeat(g, 3, axis=2)).reshape(-1)
    data = gz.process(rgb, w, h, gz.Params.for_quality(95))
    assert data[:2] == b"\xff\xd8"


@pytest.mark.parametrize("name", sorted(MANIFEST.get("e2e_edge", {})))
def test_process_edge_known_answers(gz, name):
    """The reference's edge paths on the device path: images under 32 px
    (no comparator), quality below 84 (refused), force_420 / try_420 on
    content whose chroma is all zero (the one-component continuation with
    the downsampling quantization generator, processor.cc:986-1016)."""
    e = MANIFEST["e2e_edge"][name]
    rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
    p = gz.Params.for_quality(e["quality"])
    p.force_420 = bool(e.get("params", {}).get("force_420", 0))
    p.try_420 = bool(e.get("params", {}).get("try_420", 0))
    if e.get("fail"):
        with pytest.raises(gz.GuetzliError) as err:
            gz.process(rgb, e["w"], e["h"], p)
        assert err.value.status == 1
        return
    data, st = gz.process(rgb, e["w"], e["h"], p, return_stats=True)
    assert st.iterations == e["iters"]
    assert hashlib.sha256(data).hexdigest() == e["sha256"]


_ENV_ENCODE = r"""
import hashlib, json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import guetzli_amd as gz
e = json.loads(sys.argv[2])
rgb = gz.synthetic_frame(e["seed"], e["w"], e["h"])
data, stats = gz.process(rgb, e["w"], e["h"], gz.Params.for_quality(e["quality"]), return_stats=True)
d = gz.last_process_detail()
print(json.dumps({"sha": hashlib.sha256(data).hexdigest(), "iters": stats.iterations,
                  "undone": d.get("backend_spec_undone", 0), "codes": d.get("backend_entropy_codes", 0),
                  "detail": {k: v for k, v in d.items() if k.startswith("backend_") and not k.endswith("_s")}}))
"""

# the counter each knob must move (the forced path really ran)
_VARIANT_EVIDENCE = {"GZ_TAIL_WINDOW": ("backend_tail_windows", "backend_tail_exact"),
                     "GZ_SELECT_OPEN": ("backend_select_open",),
                     "GZ_SEL_OVERFLOW": ("backend_tail_exact_nobulk",)}


@pytest.mark.parametrize("env", [{"GZ_REPLAY_DIV": "1000000"}, {"GZ_SPEC_DECADES": "1"},
                                 {"GZ_SPEC_DECADES": "32", "GZ_SPIN_US": "0"},
                                 {"GZ_TAIL_WINDOW": "16"}, {"GZ_SELECT_OPEN": "1"},
                                 {"GZ_SEL_OVERFLOW": "1"}])
def test_backend_variants_keep_known_answer(env):
    """Back-end variants that must not change the bytes (each in its own
    process: the knobs are read once).  GZ_REPLAY_DIV=1e6: every journal
    counts as long, so each sync after the device bulk prefix replays a
    journal over a partial host copy (that used to fail the
    encode); GZ_SPEC_DECADES: the speculative tail's batch fixed at one
    rebuild (the one-at-a-time loop) or 32; GZ_TAIL_WINDOW=16: the device
    selection's tail window runs out early, the tail continues in
    std::sort's exact order from there; GZ_SELECT_OPEN=1: every bulk prefix
    reported open (as when its last key is shared by several blocks), so
    the prefix is taken from std::sort's exact order on the host;
    GZ_SEL_OVERFLOW=1: every selection's window overflows, so the tail has no
    window at all -- including iterations without a bulk prefix, whose empty
    window used to ask the device for a zero-entry window.  The
    knob's counter must move, so the forced path is known to have run."""
    import subprocess
    import sys
    name = "synth_640x360_s3_q95"
    e = dict(MANIFEST["synthetic"][name])
    pkg = os.path.join(os.path.dirname(GOLDEN), "..", "guetzli-cuda-opencl_amd", "python")
    res = subprocess.run([sys.executable, "-c", _ENV_ENCODE, pkg, json.dumps(e)], env=dict(os.environ, **env),
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["sha"] == e["sha256"] and out["iters"] == e["iters"], out
    for knob, counters in _VARIANT_EVIDENCE.items():
        if knob in env:
            assert any(out["detail"].get(c, 0) > 0 for c in counters), (knob, out["detail"])
    if "GZ_SPEC_DECADES" in env:
        assert out["codes"] > 0, out


_ZIGZAG = [0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24,
           31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60, 21, 34, 37, 47, 50, 56,
           59, 61, 35, 36, 48, 49, 57, 58, 62, 63]


def _make_q(seed):
    """oracle/ref_driver.cc MakeQ: the stage fixtures' quantization matrix."""
    s = (2463534242 ^ (seed * 7919)) & 0xffffffff
    q = np.zeros((3, 64), np.int32)
    for c in range(3):
        for k in range(64):
            s ^= (s << 13) & 0xffffffff
            s ^= s >> 17
            s ^= (s << 5) & 0xffffffff
            q[c, k] = 1 + (_ZIGZAG[k] * (2 + c)) // 8 + s % 3
    return q


@pytest.mark.parametrize("name", sorted(MANIFEST.get("stage_hashes", {})))
def test_compare_stages_at_frame_size(gz, name):
    """Every Butteraugli intermediate of one Compare at the BASELINE frame
    sizes (configs[1] 1080p, configs[2] 4K) bit-identical to the
    reference's (tolerance 0; north_star asks for 1e-5): the reference's
    stage planes are committed as sha256 (tests/golden/make_stage_hashes.py),
    the device's are hashed the same way.  This pins the 4K-specific
    segment, strip and blur-group tiling and every distmap pixel, not only
    each block's maximum."""
    e = MANIFEST["stage_hashes"][name]
    w, h = e["w"], e["h"]
    rgb = gz.synthetic_frame(e["seed"], w, h)
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == e["input_sha256"]
    cand = _quantized(gz, rgb, w, h, _make_q(e["qseed"])).reshape(-1)
    assert hashlib.sha256(cand.tobytes()).hexdigest() == e["sha256"]["cand_coeffs"]
    cmp = gz.ButteraugliComparator(w, h, rgb, e["target"])
    st = cmp.compare_stages(cand)
    bad = [k for k in STAGES
           if hashlib.sha256(np.ascontiguousarray(st[k], np.float32).tobytes()).hexdigest() != e["sha256"][k]]
    assert not bad, "stages differing from the reference at %dx%d: %s" % (w, h, bad)
    assert np.float32(st["distance"]) == np.float32(e["distance"])
    # the kernels the search runs (fused edge term, fused low-frequency term,
    # subsampled B mask, LUT epilogue), per pixel at the same frame size
    del st
    pr = cmp.compare_stages_production(cand)
    bad = [k for k in PROD_STAGES
           if hashlib.sha256(np.ascontiguousarray(pr[k], np.float32).tobytes()).hexdigest() != e["sha256"][k]]
    assert not bad, "production stages differing from the reference at %dx%d: %s" % (w, h, bad)
    assert np.float32(pr["distance"]) == np.float32(e["distance"])
    assert np.float32(cmp.compare(cand)) == np.float32(e["distance"])
    dm = cmp.distmap()
    assert hashlib.sha256(np.ascontiguousarray(dm, np.float32).tobytes()).hexdigest() == e["sha256"]["distmap"]


def _interp_tables():
    """hf_dy / lf_dy as the library's table setup forms them (gz_device.hip,
    f32 running sums)."""
    hf = np.zeros(21, np.float32)
    lf = np.zeros(21, np.float32)
    hf[1] = np.float32(1.4103373714040413)
    for i in range(2, 21):
        hf[i] = hf[i - 1] + np.float32(0.7084088867024)
    for i in range(1, 21):
        lf[i] = lf[i - 1] + np.float32(5.2511644570349185)
    return hf, lf


@pytest.mark.parametrize("which", ["sqrt", "interp_hf", "interp_lf", "interp_random"])
def test_block_diff_sqrt_and_interp_exhaustive(which):
    """k_block_diff2's replacements, exhaustively on the device: its square root's
    hardware root + residual correction on 2^32-scaled inputs (sqrt_cr_big;
    the kernel carries the result scaled by 2^16) equals, scaled back, the compiler's
    correctly rounded sqrtf for every float in [0, 2^96) (the Y operands are
    |F|^2 * 0.000064 of bounded planes, far below 2^96), and interp_pair_f
    over the paired table equals interp_f (InterpolateOpt,
    clbutter_comparator.cpp:195-210) for every finite argument, on both
    tables the kernel uses and a random one (tests/native/sqrt_check.hip)."""
    import ctypes
    here = os.path.dirname(os.path.abspath(__file__))
    lib = ctypes.CDLL(os.path.join(here, "_build", "libgz_helper_check.so"))
    hf, lf = _interp_tables()
    tab = {"sqrt": hf, "interp_hf": hf, "interp_lf": lf,
           "interp_random": np.sort(np.random.default_rng(5).random(21, np.float32) * 40)}[which]
    tab = np.ascontiguousarray(tab, np.float32)
    out = (ctypes.c_ulonglong * 2)()
    rc = lib.gz_helper_check(0 if which == "sqrt" else 1, tab.ctypes.data_as(ctypes.c_void_p), out)
    assert rc == 0
    assert out[0] == 0, "%d mismatches, first bit pattern %#010x" % (out[0], out[1])
