#!/usr/bin/env python3
"""Benchmark of the MI355X Guetzli search path (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]

A step is the end-to-end `guetzli::Process` encode of a batch of
--frames-per-step synthetic sRGB frames per GPU (each frame is BASELINE.json
configs[1]: 1920x1080, q=95; the default batch of 8 per GPU is configs[3]'s
per-GPU share: 64 frames over 8 GPUs), encoded concurrently -- one host
thread and one engine (HIP stream + buffers) per frame, all on the rank's
GPU -- with the input frames already resident in HBM when the timed region
starts.  For N > 1 (launched by torch.distributed.run, one rank per GPU)
every rank encodes its own frames (image-level sharding, no data-path
collective) and the JPEG byte strings are gathered to rank 0 over RCCL at
the end of each step.  value = total pixels of all ranks / max-over-ranks
wall time.  `--gpus N` without a torch.distributed.run environment starts
the N ranks itself (one process per GPU, before any HIP call).

The first timed step of every rank encodes the synthetic frames whose
reference (`guetzli --c`) bytes are committed (tests/golden/manifest.json,
1080p q95 seeds 0..7); they are checked after the timed region ("verified"),
and a mismatch fails the run.

Also reported (one JSON line on rank 0):
  single_frame  one frame encoded alone after the timed region (latency).
  roofline      north_star's: the Butteraugli blur+mask pass at 4K against
                HBM -- one BASELINE configs[2] frame (3840x2160 q90, seed 0,
                bytes checked) encoded alone after the timed region, the
                pass's kernels timed with HIP events on the engine's own
                stream inside the library (gz_profile_*), SURVEY 8(d)'s
                272 algorithmic B/px over their summed time ("configs2_4k",
                "blur_mask_pass_4k").
  zeroing_roofline  the kernel with the most GPU time per frame (the
                per-block zeroing search) in the isolated 1080p frame: VALU /
                latency-bound, so `frac` is its vector issue utilisation from
                the committed SQ counters; its HBM fraction is `hbm_frac`.
  compare_roofline  the same for the dominant kernel of the Butteraugli
                Compare pass (block_diff), and blur_mask_pass for the
                blur+mask pass of the 1080p frame.
  cpu_baseline  the reference `guetzli --c` (oracle/_ref, built from the
                reference sources) on the host cores: one 1080p q95 frame per
                process, 8 concurrent processes (the bench workload's frames,
                bytes checked against the manifest), with the host's CPU
                model, nproc and the cores the GPU path itself consumes.
"""
import argparse
import concurrent.futures
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))

METRIC = "Mpixels/s end-to-end encode @ q=95; achieved HBM GB/s on Butteraugli pass"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# Algorithmic HBM bytes per pixel of each Compare-pass kernel: every input
# plane read once and every output plane written once (f32 = 4 B; res-grid
# arrays at 1/9 of a plane; blur h passes write a 1/step-wide plane, v passes
# read it and write 1/step^2).  Derivation in DESIGN.md §4.
def stage_bytes_per_px():
    s = {}
    s["coeffs_to_linear"] = 3 * 2 + 4              # int16 coeffs -> packed sRGB bytes (4 B/px)
    s["opsin_mhic"] = 4 + 3 * 4 + 6 * 4              # S1-S3 fused: sRGB bytes + ref XYB -> m0, m1
    s["edge_blur"] = 6 * 4 + 6 * 4                  # S4: 6 separable blurs, 6 -> 6
    s["edge_mask"] = 6 * 4 + 6 * 4 + 3 * 4          # S4 + S9-S11 fused: 6 -> 6 blurred + 3 mask front
    s["edge_map"] = 6 * 4 + 3 * 4 / 9.0              # (stage dumps only; fused into block_diff)
    # S6 + S5 fused: m0 / m1 and the edge-blurred planes -> dc, ac, edge
    s["block_diff"] = 6 * 4 + 6 * 4 + 9 * 4 / 9.0
    s["lowfreq_blur_h"] = 6 * 4 + 6 * 4 / 4.0
    s["lowfreq_blur_v"] = 6 * 4 / 4.0 + 6 * 4 / 16.0
    s["low_freq"] = 6 * 4 / 16.0 + 2 * 3 * 4 / 9.0   # (stage dumps only; fused into combine_channels)
    s["mask_front"] = 6 * 4 + 3 * 4                 # S9-S11 fused: 6 planes -> 3
    s["mask_blur_h"] = 3 * 4 + 4 * (1 / 3.0 + 1 / 4.0 + 1.0)
    s["mask_blur_v"] = 4 * (1 / 3.0 + 1 / 4.0 + 1.0) + 4 * (1 / 9.0 + 1 / 16.0 + 1.0)
    s["blur_h"] = s["lowfreq_blur_h"] + s["mask_blur_h"]    # S7 + S12 h passes, one launch
    # S7 + S12 v passes in one launch, with S13 (the mask LUT pair of every
    # blurred mask sample: one more decimated plane per channel)
    s["blur_v"] = s["lowfreq_blur_v"] + s["mask_blur_v"] + 4 * (1 / 9.0 + 1 / 16.0 + 1 / 9.0)
    s["combine"] = (3 * 4 + 3 * 4 + 3 * 4 + 3 * 4 + 4) / 9.0
    # S14/S15 + S8 fused: LUT'd mask samples + dc/ac/edge -> R, and the
    # sigma-14 planes (1/16 density) for the low-frequency term
    s["combine_channels"] = (6 * 4 + 9 * 4 + 4) / 9.0 + 6 * 4 / 16.0
    # S16 + S17 + the distance fused (k_diffmap): the res map in, the block
    # maxima out (the blur's intermediate planes stay on chip)
    s["diffmap"] = 4 / 9.0 + 4 / 64.0
    return s


# Per-block greedy zeroing search (k_block_zeroing, the search's compacted
# form), per 8x8 block: reads the candidate and q=1 coefficients (2 x 3 x 64
# int16), the block's RGB8 pixels (192 B) and its 3 mask scales, writes its
# kept-entry count; per kept entry (the search's candidates) one u8 index and
# one f32 error.
ZEROING_BYTES_PER_BLOCK = 384 + 384 + 192 + 12 + 4
ZEROING_BYTES_PER_KEPT = 1 + 4


# The launches of one search-loop Compare pass (each kernel once; the other
# entries above are the stage-dump path's or their fused parts).
PASS_KERNELS = ("coeffs_to_linear", "opsin_mhic", "edge_mask", "block_diff", "blur_h", "blur_v",
                "combine_channels", "diffmap")


# The device entropy coder, per MCU (4:4:4: one 8x8 block per component):
# k_jpeg_stage reads the 3 x 64 int16 stored coefficients (its histograms
# are a few KB per launch); k_jpeg_code reads them again and quantizes in
# place (the scan it writes, ~2-5 % of that at q95, is not counted; the code
# tables arrive as kernel arguments).
JPEG_STAGE_BYTES_PER_MCU = 3 * 64 * 2
JPEG_CODE_BYTES_PER_MCU = 3 * 64 * 2


def region_bytes(name, w, h, kept=None):
    """Algorithmic HBM bytes per launch of a profiled region, or None.
    kept: the zeroing search's kept entries (candidates) of the frame."""
    blocks = ((w + 7) // 8) * ((h + 7) // 8)
    if name == "block_zeroing":
        return ZEROING_BYTES_PER_BLOCK * blocks + ZEROING_BYTES_PER_KEPT * (kept or 0)
    if name == "jpeg_stage":
        return JPEG_STAGE_BYTES_PER_MCU * blocks
    if name == "jpeg_code":
        return JPEG_CODE_BYTES_PER_MCU * blocks
    bpp = stage_bytes_per_px()
    return bpp[name] * w * h if name in bpp else None


# The "blur+mask pass" of BASELINE.json / SURVEY.md 8(d): blurs S1, S4, S7,
# S16 and the mask chain S9-S13, 272 algorithmic B/px.  Kernels that carry
# those stages are timed whole (the opsin kernel also does the S2 transform
# and S3, edge_mask also the S4 blurs, blur_v the S13 LUTs, diffmap also
# S17, the block maxima and the distance), so the extra fused work only
# lowers the figure.  ("combine" carries S13 only in the
# stage-dump path; the search's passes run S14/S15 alone as combine_channels,
# which is outside the pass.)
BLUR_MASK_BYTES_PER_PX = 272.0
BLUR_MASK_STAGES = ("opsin_mhic", "edge_mask", "blur_h", "blur_v", "combine", "diffmap")

# Kernel symbol (rocprofv3 name prefix) of each profiled stage.
STAGE_SYMBOL = {
    "coeffs_to_linear": "gz::k_coeffs_to_srgb8(", "opsin_mhic": "gz::k_opsin_mhic_stream(",
    "edge_blur": "void gz::k_blur_stream<2>(", "edge_map": "gz::k_edge_map(",
    "block_diff": "gz::k_block_diff2(", "lowfreq_blur_h": "void gz::k_blur_h4<3,",
    "lowfreq_blur_v": "void gz::k_blur_vstream<3>(", "low_freq": "gz::k_low_freq(",
    "mask_front": "gz::k_mask_stream(", "edge_mask": "gz::k_edge_mask_stream(",
    "blur_h": "void gz::k_blur_h4<6,", "blur_v": "void gz::k_blur_vstream<6>(",
    "mask_blur_h": "void gz::k_blur_h4<4,", "mask_blur_v": "void gz::k_blur_vstream<4>(",
    "combine": "gz::k_combine(", "diffmap": "gz::k_diffmap(",
    "combine_channels": "gz::k_combine_channels(",
    "block_zeroing": "gz::k_block_zeroing(", "jpeg_stage": "gz::k_jpeg_stage(",
    "jpeg_code": "gz::k_jpeg_code(",
}


def measured_traffic(stage, w, h):
    """HBM bytes per launch of `stage` from the committed rocprofv3 PMC
    summary (tools/gpu_round.sh -> profiles/*traffic*.json: FETCH_SIZE x2
    + WRITE_SIZE, same frame size), or None."""
    import glob
    sym = STAGE_SYMBOL.get(stage)
    if sym is None:
        return None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*%dx%d*.json" % (w, h))),
                    reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in t.items():
            if k.startswith(sym) and v.get("fetch_bytes") is not None and v.get("write_bytes") is not None:
                return int(v["traffic_bytes"]), os.path.relpath(f, ROOT)
    return None, None


# gfx950 vector issue: a wave64 VALU instruction occupies its SIMD for 2
# cycles at full rate (MI355X_MICROARCH.md, execution model); 256 CUs x 4
# SIMDs, 2.4 GHz.  FP64 and transcendental instructions issue slower: their
# cycles per wave instruction come from the micro-benchmark
# tools/micro/valu_rate.hip (profiles/round3_valu_rate.json: fma_f64 4.95,
# mul_f64 4.59, add_f64 4.36, rsq_f64 16.1, ...), and the PMC summaries carry
# gfx950's per-type instruction counters (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_
# {F32,F64}, _INT32, _INT64, _CVT), so the ceiling weights each type by its
# measured cost; untyped instructions (moves, logic, compares, selects) count
# at the full-rate 2 cycles.
VALU_SIMDS, VALU_CYCLES_PER_INST, CLOCK_HZ = 1024, 2, 2.4e9
# counter -> micro-benchmark entry (cycles per wave instruction)
VALU_TYPE_RATE = {
    "SQ_INSTS_VALU_ADD_F64": "add_f64", "SQ_INSTS_VALU_MUL_F64": "mul_f64",
    "SQ_INSTS_VALU_FMA_F64": "fma_f64", "SQ_INSTS_VALU_TRANS_F64": "rsq_f64",
    "SQ_INSTS_VALU_TRANS_F32": "rsq_f32", "SQ_INSTS_VALU_FMA_F32": "fma_f32",
    "SQ_INSTS_VALU_ADD_F32": "add_f32", "SQ_INSTS_VALU_MUL_F32": "fma_f32",
    "SQ_INSTS_VALU_INT32": "mul_u32", "SQ_INSTS_VALU_CVT": "cvt_f64_f32_pair",
}


def valu_rates():
    """{micro-benchmark entry: cycles per wave instruction} from the newest
    committed profiles/*valu_rate*.json ({} when none)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*valu_rate*.json")), reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        out = {k: v["cycles_per_wave_inst"] for k, v in t.items() if isinstance(v, dict)}
        if "cvt_f64_f32_pair" in out:  # two conversions per timed step
            out["cvt_f64_f32_pair"] /= 2
        out["_source"] = os.path.relpath(f, ROOT)
        return out
    return {}


def valu_issue(stage, w, h, avg_ms):
    """VALU issue utilisation of `stage`'s kernel against the launch's
    HIP-event duration: its measured vector instructions per launch
    (committed rocprofv3 PMC summary profiles/*pmc_util_<WxH>.json) x their
    issue cycles over all SIMDs -- how close a VALU-bound kernel is to the
    vector issue ceiling (the HBM roofline does not bound it).  `frac` uses
    the per-type cycle costs where the summary has the typed counters
    (FP64 at ~4.4-5 cycles, see VALU_TYPE_RATE); `frac_flat` counts every
    instruction at 2 cycles."""
    import glob
    sym = STAGE_SYMBOL.get(stage)
    if sym is None:
        return None
    sym = sym.split("(")[0]
    rates = valu_rates()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_util*%dx%d*.json" % (w, h))),
                    reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        k = t.get(sym, {})
        v = k.get("SQ_INSTS_VALU")
        if not v:
            continue
        flat = v * VALU_CYCLES_PER_INST / VALU_SIMDS / CLOCK_HZ
        r = {"valu_insts_per_launch": int(v), "issue_ms_flat": round(flat * 1e3, 4),
             "frac_flat": round(flat / (avg_ms * 1e-3), 4), "source": os.path.relpath(f, ROOT)}
        typed = {c: k[c] for c in VALU_TYPE_RATE if c in k}
        if typed and all(VALU_TYPE_RATE[c] in rates for c in typed):
            cyc, rest = 0.0, float(v)
            for c, n in typed.items():
                cyc += n * rates[VALU_TYPE_RATE[c]]
                rest -= n
            cyc += max(rest, 0.0) * VALU_CYCLES_PER_INST
            busy = cyc / VALU_SIMDS / CLOCK_HZ
            f64 = sum(k.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
            r.update({"issue_ms": round(busy * 1e3, 4), "frac": round(busy / (avg_ms * 1e-3), 4),
                      "fp64_inst_share": round(f64 / v, 4),
                      "fp64_cycle_share": round(sum(k.get(c, 0) * rates[VALU_TYPE_RATE[c]] for c in (
                          "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                          "SQ_INSTS_VALU_TRANS_F64")) / cyc, 4),
                      "rates_source": rates["_source"]})
        else:
            r.update({"issue_ms": r["issue_ms_flat"], "frac": r["frac_flat"]})
        return r
    return None


def _thread_cpu():
    """{tid: (cpu seconds, name)} of this process's threads."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            st = open("/proc/self/task/%s/stat" % tid).read()
            f = st[st.rindex(")") + 2:].split()
            out[tid] = ((int(f[11]) + int(f[12])) / tick, st[st.index("(") + 1:st.rindex(")")])
        except (OSError, ValueError):
            pass
    return out


def launch_ranks(n_gpus):
    """`--gpus N` outside torch.distributed.run: run this script as N ranks
    (one process per GPU) under torch.distributed.run on 127.0.0.1 and exit
    with its status.  Called before anything touches the GPU."""
    import socket
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n_gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(n_gpus, backend=None):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if os.environ.get("GZ_BENCH_ONE_DEVICE") == "1":
            # (rehearsal of the N-rank flow on a one-GPU box: every rank on
            # device 0, collectives over gloo on host tensors)
            local = 0
            backend = "gloo"
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local, dist


def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity_cores": len(os.sched_getaffinity(0))}


def known_answers(w, h, q):
    """{seed: (sha256, iterations)} of the reference's bytes for synthetic
    frames of this size / quality (tests/golden/manifest.json)."""
    path = os.path.join(ROOT, "tests", "golden", "manifest.json")
    try:
        m = json.load(open(path))
    except (OSError, ValueError):
        return {}
    out = {}
    for e in m.get("synthetic", {}).values():
        if (e["w"], e["h"], e["quality"]) == (w, h, q) and not e.get("mode"):
            out[e["seed"]] = (e["sha256"], e["iters"])
    return out


def cpu_baseline(width, height, quality, processes=8):
    """Reference `guetzli --c` (oracle/_ref) on the host cores: `processes`
    concurrent single-threaded processes (the reference has no threads), one
    frame of the bench workload each (synthetic seeds 0.., whose reference
    bytes are committed: checked here too), MP/s = pixels / wall."""
    import hashlib
    ref = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")
    info = host_info()
    if not os.path.exists(ref):
        return dict(info, value=None, unit="Mpixels/s", cores=0, kind="reference",
                    sample="oracle/_ref/guetzli_ref not built")
    import guetzli_amd as gz
    cores = max(1, min(processes, info["affinity_cores"]))
    kn = known_answers(width, height, quality)
    tmp = tempfile.mkdtemp(prefix="gz_cpu_")
    procs = []
    t0 = time.time()
    for i in range(cores):
        rgb = gz.synthetic_frame(i, width, height)
        path = os.path.join(tmp, "f%d.rgb" % i)
        rgb.tofile(path)
        procs.append(subprocess.Popen([ref, "encode", path, str(width), str(height), str(quality),
                                       os.path.join(tmp, "f%d.jpg" % i), "c"],
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL))
    outs = [json.loads(p.communicate()[0]) for p in procs]
    wall = time.time() - t0
    matched = 0
    for i in range(cores):
        sha = hashlib.sha256(open(os.path.join(tmp, "f%d.jpg" % i), "rb").read()).hexdigest()
        if i in kn and kn[i][0] == sha:
            matched += 1
    px = cores * width * height
    return dict(info, value=px / wall / 1e6, unit="Mpixels/s", cores=cores, kind="reference",
                sample="%d concurrent single-threaded `guetzli --c` processes, one synthetic "
                       "%dx%d q%d frame each (seeds 0..%d: the bench workload), %.1f s wall, "
                       "%.1f s CPU" % (cores, width, height, quality, cores - 1, wall,
                                       sum(o["seconds"] for o in outs)),
                per_process_seconds=[round(o["seconds"], 2) for o in outs],
                reference_bytes_match_manifest="%d/%d" % (matched, cores))


def strip_collectives(gz, dist, group, rank, dev):
    """The strips' exchange for ranks 0-3: the library's own RCCL
    communicator (gz_rccl_create: all-gathers on its own stream, no Python
    in the exchange) when every rank can load RCCL and the four ranks sit on
    four different GPUs (RCCL refuses two ranks on one device -- the
    one-GPU test runs four ranks on cuda:0), else torch.distributed's
    collectives through the ctypes callback.  The decision is taken
    together, so no rank waits in ncclCommInitRank for one that fell back."""
    import torch
    ok = 0
    try:
        ok = 1 if gz.rccl_library() else 0
    except Exception:
        ok = 0
    tdev = "cuda:%d" % dev
    # (the decision's own exchange: on the device for the nccl backend, on
    # the host for gloo -- the one-GPU test's four ranks)
    cdev = tdev if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([ok, dev], dtype=torch.int64, device=cdev)
    got = [torch.zeros_like(t) for _ in range(4)]
    dist.all_gather(got, t, group=group)
    oks = [int(g[0].item()) for g in got]
    devs = [int(g[1].item()) for g in got]
    if all(oks) and len(set(devs)) == 4 and os.environ.get("GZ_STRIP_TORCH_EXCHANGE") != "1":
        obj = [gz.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return gz.Collectives.from_rccl(dev, rank, 4, obj[0]), "RCCL, library communicator"
    return gz.Collectives.from_torch(dist, tdev, group=group), "torch.distributed exchange"


def large_frame(gz, dist, world, rank, dev, w=8192, h=8192, q=84, seed=0):
    """BASELINE configs[4] after the timed region: one synthetic 8192x8192
    frame at q=84 (seed 0, whose reference bytes are committed).  With N >= 4
    GPUs it is split into 4 row strips with a halo over ranks 0-3 (their own
    GPUs, RCCL all-gathers over xGMI: host/strips.h), else encoded by one
    engine.  One untimed encode first (engine creation), then one timed;
    wall time is the max over the participating ranks; bytes checked.
    (w, h, q, seed: a smaller known-answer frame -- tests/test_strips.py runs
    this leg on one GPU with 4 gloo ranks.)"""
    import hashlib
    import torch
    kn = known_answers(w, h, q).get(seed)
    rgb = gz.synthetic_frame(seed, w, h)
    params = gz.Params.for_quality(q)
    strips = world >= 4
    group = None
    if strips:
        group = dist.new_group([0, 1, 2, 3])
        if rank >= 4:
            return None
        coll, exchange = strip_collectives(gz, dist, group, rank, dev)

        def run():
            return gz.process_strips(rgb, w, h, coll, params, device=dev)
    elif rank == 0:
        def run():
            return gz.process(rgb, w, h, params, device=dev)
    else:
        return None
    run()  # (engine creation, first touch)
    if strips:
        dist.barrier(group=group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    data = run()
    elapsed = time.perf_counter() - t0
    if strips:
        coll.close()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(t.item())
    sha = hashlib.sha256(data).hexdigest()
    return {"config": "BASELINE configs[4]: synthetic %dx%d q%d (seed %d)" % (w, h, q, seed),
            "mode": "4 row strips + halo over GPUs 0-3 (%s)" % exchange if strips else "one engine, 1 GPU",
            "gpus": 4 if strips else 1, "seconds": round(elapsed, 3),
            "Mpixels_per_s": round(w * h / elapsed / 1e6, 3), "bytes": len(data),
            "bit_exact": bool(kn and kn[0] == sha), "against": "reference guetzli --c sha256"}


def dist_selftest(args):
    """The multi-rank skeleton of main() on CPU: every rank (launched by
    launch_ranks) joins a gloo group, "encodes" its frames into stand-in byte
    strings (the synthetic frames' raw bytes, distinct lengths), gathers
    them as the real run does and takes the max-over-ranks time; rank 0
    prints one JSON line."""
    import torch
    import guetzli_amd as gz
    from guetzli_amd import sharding
    world, rank, _, dist = dist_setup(args.gpus, backend="gloo")
    t0 = time.perf_counter()
    blobs = [gz.synthetic_frame(rank * 100 + f, 16 + f, 8).tobytes()[:37 * (f + 1) + rank]
             for f in range(args.frames_per_step)]
    got = sharding.gather_bytes(blobs, dist, "cpu") if dist is not None else [blobs]
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    expect = [[gz.synthetic_frame(r * 100 + f, 16 + f, 8).tobytes()[:37 * (f + 1) + r]
               for f in range(args.frames_per_step)] for r in range(world)]
    if rank == 0:
        print(json.dumps({"selftest": True, "n_gpus": world, "gather_ok": got == expect,
                          "max_seconds": float(t.item()),
                          "frames": sum(len(r) for r in got)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0 if got == expect else 1


def frame_report(prof, w, h, kept):
    """Per-launch HIP-event report of one isolated frame (gz_profile_*):
    stages, the Compare pass, the blur+mask pass and the kernel rooflines.
    kept: the frame's kept zeroing entries."""
    bpp = stage_bytes_per_px()
    stages = {}
    regions = []
    for name, (cnt, ms) in prof.items():
        if not cnt:
            continue
        avg = ms / cnt
        b = region_bytes(name, w, h, kept)
        row = {"launches": cnt, "avg_ms": round(avg, 4), "frame_ms": round(ms, 4)}
        if b is not None:
            row["algo_GBps"] = round(b / (avg * 1e-3) / 1e9, 1)
        if name in bpp or name in ("block_zeroing", "jpeg_stage", "jpeg_code"):
            stages[name] = row
        if name != "compare_pass":
            regions.append((ms, name, cnt))
    regions.sort(reverse=True)

    def roof_of(name):
        cnt, ms = prof[name]
        avg = ms / cnt
        b = region_bytes(name, w, h, kept)
        achieved = b / (avg * 1e-3) / 1e9
        traffic, tsrc = measured_traffic(name, w, h)
        r = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
             "traffic": traffic, "traffic_source": tsrc, "algo_bytes_per_launch": int(b),
             "avg_launch_ms": round(avg, 4), "launches_per_frame": cnt,
             "frame_gpu_ms": round(ms, 4)}
        vi = valu_issue(name, w, h, avg)
        if vi:
            r["valu_issue"] = vi
        return r

    # the kernel with the most GPU time in the frame (the per-block zeroing
    # search): VALU/latency-bound, so its ceiling is the vector issue rate
    # (valu_issue.frac); its HBM fraction is kept beside it as hbm_frac
    dominant = next((n for _, n, _ in regions if region_bytes(n, w, h) is not None), None)
    dom = roof_of(dominant) if dominant else None
    if dom is not None:
        dom["gpu_time_share_of_frame"] = round(prof[dominant][1] / sum(ms for ms, _, _ in regions), 4)
        if "valu_issue" in dom:
            dom["hbm_frac"] = dom["frac"]
            dom.update({"bound": "valu", "unit": "VALU issue fraction",
                        "achieved": dom["valu_issue"]["frac"], "peak": 1.0,
                        "frac": dom["valu_issue"]["frac"]})
    # the dominant kernel of the Butteraugli Compare pass
    cmp_rows = sorted(((prof[n][1], n) for n in bpp if n in prof and prof[n][0]), reverse=True)
    compare_roof = roof_of(cmp_rows[0][1]) if cmp_rows else None
    bm_ms = sum(stages[k]["avg_ms"] for k in BLUR_MASK_STAGES if k in stages)
    blur_mask = None
    if bm_ms > 0:
        bm_bytes = BLUR_MASK_BYTES_PER_PX * w * h
        blur_mask = {"algo_bytes": int(bm_bytes), "ms": round(bm_ms, 4),
                     "achieved_GBps": round(bm_bytes / (bm_ms * 1e-3) / 1e9, 1),
                     "frac": round(bm_bytes / (bm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "stages": [k for k in BLUR_MASK_STAGES if k in stages],
                     "stage_ms": {k: stages[k]["avg_ms"] for k in BLUR_MASK_STAGES if k in stages}}
        # measured HBM bytes of the same launches (committed PMC summary of
        # this frame size), where every stage has one
        tr = [measured_traffic(k, w, h)[0] for k in blur_mask["stages"]]
        if tr and all(t is not None for t in tr):
            blur_mask["traffic"] = int(sum(tr))
            blur_mask["traffic_GBps"] = round(sum(tr) / (bm_ms * 1e-3) / 1e9, 1)
    cp = prof.get("compare_pass")
    pass_bytes = sum(bpp[k] for k in PASS_KERNELS) * w * h
    compare_pass = None
    if cp and cp[0]:
        avg = cp[1] / cp[0]
        compare_pass = {"launches": cp[0], "avg_ms": round(avg, 4),
                        "algo_bytes": int(pass_bytes),
                        "algo_GBps": round(pass_bytes / (avg * 1e-3) / 1e9, 1)}
    return {"stages": stages, "regions": regions, "dominant": dom, "compare_roofline": compare_roof,
            "blur_mask_pass": blur_mask, "compare_pass": compare_pass}


def frame_config(w, h, q):
    """Which BASELINE config a bench frame is."""
    if (w, h) == (1920, 1080):
        return "each frame = BASELINE configs[1] (there at q=95)%s; 8 per GPU = configs[3]'s " \
               "per-GPU share" % ("" if q == 95 else ", here at q=%d" % q)
    if (w, h) == (3840, 2160):
        return "each frame = BASELINE configs[2] (there at q=90)%s" % ("" if q == 90 else ", here at q=%d" % q)
    if (w, h) == (8192, 8192):
        return "each frame = BASELINE configs[4] (there at q=84)"
    return "not a BASELINE frame size"


def uhd_frame(gz, dev):
    """BASELINE configs[2] after the timed region: one synthetic 3840x2160
    frame at q=90 (seed 0, whose reference bytes are committed), resident in
    HBM, encoded alone with per-launch HIP-event timing -- north_star's
    roofline is the Butteraugli blur+mask pass at 4K.  Bytes checked."""
    import hashlib
    import torch
    w, h, q = 3840, 2160, 90
    kn = known_answers(w, h, q).get(0)
    t = torch.from_numpy(gz.synthetic_frame(0, w, h).reshape(-1)).to("cuda:%d" % dev)
    torch.cuda.synchronize()
    params = gz.Params.for_quality(q)
    gz.profile_reset()
    gz.profile_enable(True)
    t0 = time.perf_counter()
    data, st = gz.process_device(t.data_ptr(), w, h, params, device=dev, return_stats=True)
    sec = time.perf_counter() - t0
    gz.profile_enable(False)
    prof = gz.profile_read()
    detail = gz.last_process_detail()
    rep = frame_report(prof, w, h, int(detail.get("candidates", 0)))
    sha = hashlib.sha256(data).hexdigest()
    return {"config": "BASELINE configs[2]: synthetic 3840x2160 q90 (seed 0), one frame alone",
            "seconds": round(sec, 4), "iterations": st.iterations,
            "bit_exact": bool(kn and (kn[0], kn[1]) == (sha, st.iterations)),
            "against": "reference guetzli --c sha256 + iterations (tests/golden/manifest.json)",
            "blur_mask_pass": rep["blur_mask_pass"], "compare_pass": rep["compare_pass"],
            "compare_roofline": rep["compare_roofline"], "zeroing_roofline": rep["dominant"],
            "stages": rep["stages"]}


def north_star_roofline(uhd):
    """The line's `roofline` (north_star): the Butteraugli blur+mask pass at
    4K against HBM -- SURVEY 8(d)'s 272 algorithmic B/px over the summed
    HIP-event time of the kernels carrying those stages; traffic from the
    committed 4K PMC summary of the same kernels."""
    bm = uhd and uhd.get("blur_mask_pass")
    if not bm:
        return None
    return {"bound": "hbm", "kernel": "blur+mask pass (%s)" % ", ".join(bm["stages"]),
            "achieved": bm["achieved_GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": bm["frac"], "traffic": bm.get("traffic"),
            "algo_bytes_per_launch": bm["algo_bytes"], "avg_launch_ms": bm["ms"],
            "stage_ms": bm["stage_ms"],
            "workload": "BASELINE configs[2] frame (3840x2160 q90), %s" % (
                "bytes verified" if uhd["bit_exact"] else "BYTES NOT VERIFIED")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=95)
    ap.add_argument("--frames-per-step", type=int, default=8,
                    help="frames per GPU per step, encoded concurrently")
    ap.add_argument("--in-flight", type=int, default=8,
                    help="frames encoded at once per GPU (0: the frames of one step; 8 measured best "
                         "in round 5, profiles/round5_inflight_sweep.txt)")
    ap.add_argument("--host-threads", type=int, default=0,
                    help="host pool threads per process, caller included (sets GZ_HOST_THREADS "
                         "unless that is set; 0: the library's default, min(16, usable CPUs); "
                         "the pool runs at most that minus the encodes in progress at once)")
    ap.add_argument("--lockstep", action="store_true",
                    help="start a step's frames only after the previous step's last frame "
                         "finished (default: the timed steps' frames go through one queue, "
                         "--in-flight at a time, so a frame starts when any frame finishes)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-processes", type=int, default=8)
    ap.add_argument("--no-large-frame", action="store_true",
                    help="skip the BASELINE configs[4] leg (8192x8192 q84: one engine at N < 4, "
                         "4 row strips over GPUs 0-3 at N >= 4)")
    ap.add_argument("--no-uhd-frame", action="store_true",
                    help="skip the BASELINE configs[2] leg (one 3840x2160 q90 frame encoded alone "
                         "after the timed region: the north_star blur+mask roofline at 4K)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU check of the multi-rank path (launcher, gloo, byte gather, "
                         "max-over-ranks timing) with stand-in payloads; no GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.dist_selftest:
        return dist_selftest(args)
    world, rank, local, dist = dist_setup(args.gpus)
    if args.host_threads > 0:
        os.environ.setdefault("GZ_HOST_THREADS", str(args.host_threads))
    import hashlib
    import torch
    import guetzli_amd as gz
    from guetzli_amd import sharding

    dev = local
    torch.cuda.set_device(dev)
    # (collective tensors: on the device for RCCL, on the host for gloo)
    cdev = "cpu" if dist is not None and dist.get_backend() == "gloo" else "cuda:%d" % dev
    w, h, q = args.width, args.height, args.quality
    params = gz.Params.for_quality(q)
    nsteps = args.warmup + args.steps
    # distinct frames per (rank, step, slot), uploaded to HBM before timing;
    # the first timed step of every rank is the known-answer frames (seeds
    # 0..) where the manifest has them
    kn = known_answers(w, h, q)
    seeds = []
    for s in range(nsteps):
        row = []
        for f in range(args.frames_per_step):
            if s == args.warmup and f in kn:
                row.append(f)
            else:
                row.append(1000 + rank * 100000 + s * 100 + f)
        seeds.append(row)
    frames = [[torch.from_numpy(gz.synthetic_frame(sd, w, h).reshape(-1)).to(f"cuda:{dev}")
               for sd in row] for row in seeds]
    torch.cuda.synchronize()

    in_flight = args.in_flight if args.in_flight > 0 else args.frames_per_step
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=in_flight)

    def encode(t):
        return gz.process_device(t.data_ptr(), w, h, params, device=dev, return_stats=True)

    def submit(s):
        return [pool.submit(encode, t) for t in frames[s]]

    def step(s, futs=None):
        res = [f.result() for f in (futs if futs is not None else submit(s))]
        out = [r[0] for r in res]
        if dist is not None:
            # the final gather of the JPEG byte strings over RCCL/xGMI
            gathered = sharding.gather_bytes(out, dist, cdev)
            assert gathered[rank] == out
        return out, [r[1] for r in res]

    for s in range(args.warmup):
        step(s)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    import resource
    t_before = _thread_cpu() if os.environ.get("GZ_THREAD_CPU") else {}
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    iters = []
    conc = {}
    checked = []
    keys = ("seconds_total", "seconds_setup", "seconds_write", "seconds_quantize",
            "seconds_backend", "seconds_compare", "seconds_zeroing")
    # Streaming (default): every timed frame is queued at once and the pool
    # keeps in_flight of them encoding, so the steps' frames overlap at step
    # boundaries (no per-step tail, no frames entering their host-heavy
    # phases together); each step's outputs are gathered once its frames are
    # done.  --lockstep: a step starts when the previous one has finished.
    futs = {} if args.lockstep else {s: submit(s) for s in range(args.warmup, nsteps)}
    for s in range(args.warmup, nsteps):
        out, stats = step(s, futs.get(s))
        if s == args.warmup:
            checked = [(seeds[s][f], out[f], stats[f].iterations)
                       for f in range(len(out)) if seeds[s][f] in kn]
        iters.extend(st.iterations for st in stats)
        for st in stats:
            for k in keys:
                conc[k] = conc.get(k, 0.0) + getattr(st, k) / (args.steps * len(stats))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    if os.environ.get("GZ_THREAD_CPU"):
        # per-thread CPU seconds spent inside the timed region (diagnostic)
        t_after = _thread_cpu()
        rows = sorted(((c - t_before.get(k, (0.0, ""))[0], n) for k, (c, n) in t_after.items()),
                      reverse=True)
        print("thread cpu:", [(round(c, 3), n) for c, n in rows[:24] if c > 0.001], file=sys.stderr)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    cpu_per_frame = cpu_s / (args.steps * args.frames_per_step)
    # verification of the known-answer frames (after the timed region)
    ok = sum(1 for sd, data, it in checked
             if (hashlib.sha256(data).hexdigest(), it) == kn[sd])
    counts = [len(checked), ok]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor(counts, dtype=torch.int64, device=cdev)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        counts = [int(v) for v in c.tolist()]

    # isolated frame: latency, host breakdown and per-kernel HIP-event timing
    gz.profile_reset()
    gz.profile_enable(True)
    t1 = time.perf_counter()
    _, st1 = encode(frames[0][0])
    single_s = time.perf_counter() - t1
    gz.profile_enable(False)
    prof = gz.profile_read()
    host = {}
    for k in keys:
        host[k] = getattr(st1, k)
    host.update(gz.last_process_detail())

    out = None
    if rank == 0:
        total_px = world * args.steps * args.frames_per_step * w * h
        value = total_px / elapsed / 1e6

        rep = frame_report(prof, w, h, int(host.get("candidates", 0)))
        regions = rep["regions"]
        uhd = None if args.no_uhd_frame else uhd_frame(gz, dev)
        gpu_frame_ms = sum(ms for ms, _, _ in regions)

        out = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": "%d synthetic %dx%d sRGB frames per GPU per step, %d encoding "
                                   "at once, q=%d, guetzli::Process end to end (%s)" % (
                                       args.frames_per_step, w, h, in_flight, q, frame_config(w, h, q)),
                       "width": w, "height": h, "quality": q,
                       "frames_per_gpu_per_step": args.frames_per_step,
                       "frames_in_flight": in_flight,
                       "host_pool_threads": int(os.environ.get("GZ_HOST_THREADS", "0")) or "library default",
                       "schedule": "lockstep steps" if args.lockstep else
                                   "one queue over the timed steps' frames",
                       "parallelism": "image-sharded over %d GPU(s)%s" % (
                           world, ", RCCL all_gather of JPEG bytes" if world > 1 else ""),
                       "search_iterations": iters},
            "verified": {"frames": counts[0], "bit_exact": counts[1],
                         "against": "reference guetzli --c sha256 + iterations "
                                    "(tests/golden/manifest.json)"},
            "roofline": north_star_roofline(uhd) or rep["dominant"],
            "zeroing_roofline": rep["dominant"],
            "compare_roofline": rep["compare_roofline"],
            "compare_pass": rep["compare_pass"],
            "blur_mask_pass": rep["blur_mask_pass"],
            "stages": rep["stages"],
            "gpu_ms_per_frame_isolated": round(gpu_frame_ms, 3),
            "gpu_regions_ms_per_frame": {n: round(ms, 4) for ms, n, _ in regions},
            "concurrent_frame_breakdown_seconds": {k: round(v, 4) for k, v in conc.items()},
            "host_cpu_seconds_per_frame": round(cpu_per_frame, 4),
            "host_cores_busy_per_gpu": round(cpu_s / elapsed, 2),
            "host_cpu_user_system_seconds_per_frame": [
                round((ru1.ru_utime - ru0.ru_utime) / (args.steps * args.frames_per_step), 4),
                round((ru1.ru_stime - ru0.ru_stime) / (args.steps * args.frames_per_step), 4)],
            "single_frame": {"seconds": round(single_s, 4),
                             "Mpixels_per_s": round(w * h / single_s / 1e6, 4),
                             "iterations": st1.iterations,
                             "host_breakdown_seconds": {k: round(v, 4) for k, v in host.items()}},
        }
        if uhd is not None:
            out["configs2_4k"] = uhd
            out["blur_mask_pass_4k"] = uhd["blur_mask_pass"]
    large = None
    if not args.no_large_frame:
        # (a side leg after the timed region: a failure there is reported in
        # the line instead of losing it; with N >= 4 its strip ranks exchange
        # through collectives, and a watchdog prints the line without the leg
        # and ends every rank if the leg has not finished in
        # GZ_STRIP_LEG_LIMIT seconds)
        watchdog = None
        if world >= 4:
            import threading
            leg_done = threading.Event()
            limit = float(os.environ.get("GZ_STRIP_LEG_LIMIT", "240"))

            def watch():
                if leg_done.wait(limit):
                    return
                if rank == 0:
                    out["configs4_8192"] = {"config": "BASELINE configs[4]",
                                            "error": "strip leg unfinished after %.0f s" % limit}
                    print(json.dumps(out), flush=True)
                print("configs[4] leg unfinished after %.0f s on rank %d: exiting" % (limit, rank),
                      file=sys.stderr, flush=True)
                os._exit(3 if counts[1] != counts[0] else 0)
            watchdog = threading.Thread(target=watch, daemon=True)
            watchdog.start()
        try:
            large = large_frame(gz, dist, world, rank, dev)
        except Exception as e:  # noqa: BLE001
            large = {"config": "BASELINE configs[4]", "error": repr(e)[:400]}
            print("configs[4] leg failed on rank %d: %r" % (rank, e), file=sys.stderr, flush=True)
        if watchdog is not None:
            leg_done.set()
    if rank != 0:
        pool.shutdown()
        if dist is not None:
            dist.destroy_process_group()
        return
    if large is not None:
        out["configs4_8192"] = large
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(w, h, q, args.cpu_baseline_processes)
    print(json.dumps(out), flush=True)
    pool.shutdown()
    if dist is not None:
        dist.destroy_process_group()
    if counts[1] != counts[0]:
        print("bench: %d of %d known-answer frames differ from the reference" % (
            counts[0] - counts[1], counts[0]), file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
