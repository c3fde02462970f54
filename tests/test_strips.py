"""One frame over several GPUs: row strips with a halo (SURVEY.md §8e,
BASELINE configs[4]).

CPU (no GPU needed):
  * the layout tiles the image with aligned strips;
  * the halo claim on the CPU oracle: Butteraugli of a strip (owned rows +
    96-row halo) reproduces the full-image distance map and activity mask on
    the owned rows bit for bit;
  * the product's StripComparator over oracle comparators, ranks as threads,
    reproduces the reference's JPEG bytes (tests/native/strips_oracle_e2e.cc);
  * the torch.distributed binding of the collectives (gloo, world size 2).
GPU: every rank on cuda:0 (gloo exchange) reproduces the reference bytes.
"""
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle_lib import GOLDEN, lib as oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


@pytest.mark.parametrize("w,h,world", [(8192, 8192, 4), (444, 258, 2), (444, 258, 3), (64, 40, 4),
                                       (3840, 2160, 8), (100, 1000, 7)])
def test_strip_layout_tiles_the_image(gz, w, h, world):
    prev = 0
    for r in range(world):
        y0, y1, e0, e1 = gz.strip_layout(w, h, world, r)
        assert y0 == prev and y1 >= y0
        assert y0 % 24 == 0 or y0 == h
        if y1 > y0:
            assert e0 == max(0, y0 - 96) and e1 == min(h, y1 + 96)
        prev = y1
    assert prev == h


def _quantized_candidate(gz, rgb, w, h, seed):
    coeffs = gz.rgb_to_coeffs(rgb, w, h)
    rng = np.random.default_rng(seed)
    q = rng.integers(1, 14, size=(3, 64))
    nb = ((w + 7) // 8) * ((h + 7) // 8)
    c = coeffs.reshape(3, nb, 64).astype(np.int32)
    qq = q[:, None, :]
    r = np.fmod(c, qq)
    return (c + np.where(2 * r > qq, qq - r, np.where(-2 * r > qq, -qq - r, -r))).astype(np.int16)


@pytest.mark.parametrize("w,h,world,seed", [(72, 456, 3, 1), (40, 300, 2, 2)])
def test_oracle_strip_equals_full_image_on_owned_rows(gz, w, h, world, seed):
    """The halo claim of host/strips.h on the CPU oracle: distance map and
    (reference) activity mask of each strip equal the full image's on the
    rows the strip owns."""
    L = oracle()
    rgb = gz.synthetic_frame(seed, w, h)
    cand = _quantized_candidate(gz, rgb, w, h, seed)
    bw = (w + 7) // 8
    full = np.zeros(w * h, np.float32)
    L.gzo_compare(w, h, rgb.ravel(), cand.ravel(), full)
    full = full.reshape(h, w)

    def mask_of(img, hh):
        n = w * hh
        ref = np.zeros(3 * n, np.float32)
        L.gzo_srgb_to_linear_planes(w, hh, np.ascontiguousarray(img).ravel(), ref)
        L.gzo_opsin_dynamics(w, hh, ref)
        m = np.zeros(3 * n, np.float32)
        dc = np.zeros(3 * n, np.float32)
        L.gzo_mask(w, hh, ref, ref, m, dc)
        return m.reshape(3, hh, w), dc.reshape(3, hh, w)

    full_mask, full_dc = mask_of(rgb, h)
    for r in range(world):
        y0, y1, e0, e1 = gz.strip_layout(w, h, world, r)
        if y1 == y0:
            continue
        hs = e1 - e0
        sub_rgb = np.ascontiguousarray(rgb[e0:e1])
        sub = np.ascontiguousarray(cand[:, (e0 // 8) * bw:((e1 + 7) // 8) * bw, :])
        dm = np.zeros(w * hs, np.float32)
        L.gzo_compare(w, hs, sub_rgb.ravel(), sub.ravel(), dm)
        dm = dm.reshape(hs, w)
        got, want = dm[y0 - e0:y1 - e0], full[y0:y1]
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
            "rank %d: %d distance values differ" % (r, int((got != want).sum()))
        m, dc = mask_of(sub_rgb, hs)
        assert np.array_equal(m[:, y0 - e0:y1 - e0], full_mask[:, y0:y1])
        assert np.array_equal(dc[:, y0 - e0:y1 - e0], full_dc[:, y0:y1])


# The back end's order on a split frame (host/processor.cc StripOrder):
# from the ranks' own entries (default; tiny merge windows), every iteration
# exact (the whole frame's entries on every rank), and the switch to the
# exact order forced at the prefix / in mid-tail.
STRIP_ORDER_MODES = {
    "fast": {},
    "fast_window2": {"GZ_STRIP_WINDOW": "2"},
    "exact": {"GZ_STRIP_ORDER": "exact"},
    "open_prefix": {"GZ_STRIP_TEST_OPEN": "prefix"},
    "open_tail": {"GZ_STRIP_TEST_OPEN": "tail", "GZ_STRIP_WINDOW": "3"},
}


@pytest.mark.parametrize("mode", sorted(STRIP_ORDER_MODES))
@pytest.mark.parametrize("name,world", [("bees_q95", 2), ("bees_q84", 3)])
def test_strip_comparator_threads_reproduce_reference(strips_e2e_bin, name, world, mode, tmp_path):
    """StripComparator (product host code) with oracle strip comparators:
    every rank's bytes equal the reference `guetzli --c` known answer, in
    every mode of the back end's order."""
    e = MANIFEST["e2e"][name]
    out = tmp_path / "out.jpg"
    env = dict(os.environ, **STRIP_ORDER_MODES[mode])
    res = subprocess.run([strips_e2e_bin, os.path.join(GOLDEN, e["input"]), str(e["w"]),
                          str(e["h"]), str(e["quality"]), str(world), str(out)],
                         capture_output=True, text=True, timeout=600, env=env)
    assert res.returncode == 0, res.stderr
    info = json.loads(res.stdout)
    assert info["iters"] == e["iters"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == e["sha256"]
    if mode.startswith("fast"):
        assert info["strip_order_fast_iters"] > 0 and info["strip_order_fallbacks"] == 0, info
    elif mode == "exact":
        assert info["strip_order_fast_iters"] == 0 and info["strip_order_fallbacks"] == 0, info
    else:
        assert info["strip_order_fallbacks"] > 0, info


@pytest.mark.parametrize("kind,at", [("compare", 1), ("compare", 5), ("zeroing", 1)])
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_strip_rank_failure_fails_every_rank(strips_e2e_bin, kind, at, fail_rank, tmp_path):
    """One rank's comparator fails (its at-th Compare / zeroing call): the
    status word in every exchange makes all ranks return the error in that
    same exchange -- none is left blocked in the next all-gather."""
    e = MANIFEST["e2e"]["tex_64x48_q95"]
    res = subprocess.run([strips_e2e_bin, os.path.join(GOLDEN, e["input"]), str(e["w"]),
                          str(e["h"]), str(e["quality"]), "2", str(tmp_path / "o.jpg"),
                          str(fail_rank), kind, str(at)],
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 5, res.stdout + res.stderr
    lines = res.stdout.strip().splitlines()
    assert "injected" in lines[fail_rank]
    assert "rank %d failed" % fail_rank in lines[1 - fail_rank]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_selftest(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
    import torch.distributed as dist
    import guetzli_amd as gz
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        c = gz.Collectives.from_torch(dist, "cpu")
        c.selftest()
        q.put((rank, "ok"))
    except Exception as ex:  # reported to the parent
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_torch_collectives_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_selftest, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}


def _gpu_strip_rank(rank, world, port, e, q, force=False):
    import sys
    if force:  # (world 1 runs the strip machinery, not the single-engine search)
        os.environ["GZ_STRIP_FORCE"] = "1"
    sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
    import torch.distributed as dist
    import guetzli_amd as gz
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        if "seed" in e:
            rgb = gz.synthetic_frame(e["seed"], e["w"], e["h"])
        else:
            rgb = np.fromfile(os.path.join(GOLDEN, e["input"]), np.uint8)
        coll = gz.Collectives.from_torch(dist, "cpu")
        data = gz.process_strips(rgb, e["w"], e["h"], coll, gz.Params.for_quality(e["quality"]),
                                 device=0)
        q.put((rank, hashlib.sha256(data).hexdigest()))
    except Exception as ex:
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name,world,force", [("bees_q95", 1, True), ("bees_q95", 1, False), ("bees_q90", 2, False),
                                              ("synth_1366x768_s5_q88", 3, False),
                                              ("synth_2560x1440_s2_q92", 4, False),
                                              ("synth_8192x8192_s0_q84", 4, False)])
def test_gpu_strips_reproduce_reference(name, world, force):
    """`world` ranks, each a process with its strip's engine on cuda:0, the
    exchange over gloo: every rank returns the reference bytes -- including
    BASELINE configs[4] (8192x8192 q84 as 4 strips of 2048 rows + halo).  One
    rank: the single-engine search by default, the strip machinery with
    GZ_STRIP_FORCE=1 (force)."""
    import torch.multiprocessing as mp
    e = MANIFEST["e2e"].get(name) or MANIFEST["synthetic"][name]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_strip_rank, args=(r, world, port, e, q, force)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(60)
    assert len(res) == world and all(v == e["sha256"] for v in res.values()), res


_RCCL_CHILD = r"""
import hashlib, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import guetzli_amd as gz
w, h, quality, path, want = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6]
rgb = np.fromfile(path, np.uint8)
uid = gz.rccl_unique_id()
assert len(uid) == 128
coll = gz.Collectives.from_rccl(0, 0, 1, uid)
try:
    coll.selftest()
    data = gz.process_strips(rgb, w, h, coll, gz.Params.for_quality(quality), device=0)
finally:
    coll.close()
assert "torch" not in sys.modules
got = hashlib.sha256(data).hexdigest()
print(got)
sys.exit(0 if got == want else 3)
"""


_RCCL_TORCH_CHILD = r"""
import hashlib, os, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import guetzli_amd as gz
w, h, quality, path, want = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6]
# torch's HIP runtime initialised first, as in bench.py's ranks
x = torch.ones(1024, device="cuda:0")
torch.cuda.synchronize()
rgb = np.fromfile(path, np.uint8)
uid = gz.rccl_unique_id()
lib = gz.rccl_library()
coll = gz.Collectives.from_rccl(0, 0, 1, uid)
try:
    coll.selftest()
    data = gz.process_strips(rgb, w, h, coll, gz.Params.for_quality(quality), device=0)
finally:
    coll.close()
assert float(x.sum().item()) == 1024.0
got = hashlib.sha256(data).hexdigest()
print(lib)
print(got)
sys.exit(0 if got == want else 3)
"""


@pytest.mark.gpu
def test_rccl_collectives_beside_torch():
    """The library's RCCL communicator in a process that imported torch and
    initialised its device first (bench.py's ranks): the librccl is the one
    beside the HIP runtime torch mapped (the system RCCL fails in
    ncclCommInitRank against torch's runtime), its self-test passes and a
    strip encode over it gives the reference's bytes (world 1,
    GZ_STRIP_FORCE=1)."""
    e = MANIFEST["e2e"]["bees_q95"]
    r = subprocess.run([sys.executable, "-c", _RCCL_TORCH_CHILD,
                        os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"), str(e["w"]), str(e["h"]),
                        str(e["quality"]), os.path.join(GOLDEN, e["input"]), e["sha256"]],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, GZ_STRIP_FORCE="1"))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    import torch
    lib = r.stdout.strip().splitlines()[-2]
    assert os.path.dirname(lib) == os.path.join(os.path.dirname(torch.__file__), "lib"), lib


@pytest.mark.gpu
def test_rccl_collectives_reproduce_reference():
    """The library's own RCCL communicator (gz_rccl_create: host/
    rccl_collectives.cc, staged all-gathers on its own stream) as the strips'
    exchange: its self-test and a strip encode over it give the reference's
    bytes.  World 1 (one GPU on the test box: RCCL refuses two ranks on one
    device; GZ_STRIP_FORCE=1: the strip machinery, not the single-engine
    search a one-rank split runs); the multi-GPU wiring is the same calls with
    more ranks.  In a
    process of its own without torch, as the C++ callers it serves run (the
    communicator beside torch: test_rccl_collectives_beside_torch)."""
    e = MANIFEST["e2e"]["bees_q95"]
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"),
                        str(e["w"]), str(e["h"]), str(e["quality"]), os.path.join(GOLDEN, e["input"]),
                        e["sha256"]], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, GZ_STRIP_FORCE="1"))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def _bench_strip_rank(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import bench
    import guetzli_amd as gz
    torch.set_num_threads(1)
    dist = None
    try:
        _, _, _, dist = bench.dist_setup(world, backend="gloo")
        # every rank on cuda:0: the leg's group of ranks 0-3, its "cuda:0"
        # Collectives.from_torch branch and its max-over-ranks time
        q.put((rank, bench.large_frame(gz, dist, world, rank, 0, w=640, h=360, q=95, seed=3)))
    except Exception as ex:  # reported to the parent
        q.put((rank, repr(ex)))
    finally:
        if dist is not None:
            dist.destroy_process_group()


@pytest.mark.gpu
def test_bench_large_frame_strip_leg_world4():
    """bench.py's configs[4] leg as the driver's N >= 4 run takes it --
    dist.new_group([0, 1, 2, 3]), Collectives.from_torch(dist, "cuda:N",
    group=...), the all_reduce(MAX) of the time -- with 4 gloo ranks sharing
    cuda:0 and a small known-answer frame (640x360 q95 seed 3, 4 strips of
    96 rows + halo): every rank reports the reference's bytes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_strip_rank, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
    assert len(res) == 4, res
    for r, v in res.items():
        assert isinstance(v, dict), (r, v)
        assert v["gpus"] == 4 and "strips" in v["mode"] and v["bit_exact"], (r, v)
