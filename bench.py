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
wall time.

Also reported (one JSON line on rank 0):
  single_frame  one frame encoded alone after the timed region (latency).
  roofline      dominant HBM-bound kernel of the Butteraugli pass, timed with
                HIP events on the engine's own stream inside the library
                (gz_profile_*) during that isolated frame, against
                algorithmic bytes per launch.
  cpu_baseline  the reference `guetzli --c` (oracle/_ref, built from the
                reference sources) on the host cores, on a bounded sample.
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
    s["coeffs_to_linear"] = 3 * 2 + 3 * 4          # int16 coeffs -> 3 f32 planes
    s["opsin_mhic"] = 3 * 4 + 3 * 4 + 6 * 4          # S1-S3 fused: linear + ref XYB -> m0, m1
    s["edge_blur"] = 6 * 4 + 6 * 4                  # S4: 6 separable blurs, 6 -> 6
    s["edge_map"] = 6 * 4 + 3 * 4 / 9.0
    s["block_diff"] = 6 * 4 + 6 * 4 / 9.0
    s["lowfreq_blur_h"] = 6 * 4 + 6 * 4 / 4.0
    s["lowfreq_blur_v"] = 6 * 4 / 4.0 + 6 * 4 / 16.0
    s["low_freq"] = 6 * 4 / 16.0 + 2 * 3 * 4 / 9.0
    s["mask_front"] = 6 * 4 + 3 * 4                 # S9-S11 fused: 6 planes -> 3
    s["mask_blur_h"] = 3 * 4 + 4 * (1 / 3.0 + 1 / 4.0 + 1.0)
    s["mask_blur_v"] = 4 * (1 / 3.0 + 1 / 4.0 + 1.0) + 4 * (1 / 9.0 + 1 / 16.0 + 1.0)
    s["combine"] = (3 * 4 + 3 * 4 + 3 * 4 + 3 * 4 + 4) / 9.0
    s["diffmap_blur_h"] = 4 / 9.0 + 4 / 2.0
    s["diffmap_blur_v"] = 4 / 2.0 + 4 / 4.0
    s["diffmap_final"] = 4 / 9.0 + 4 / 4.0 + 4 / 64.0
    return s


# The "blur+mask pass" of BASELINE.json / SURVEY.md 8(d): blurs S1, S4, S7,
# S16 and the mask chain S9-S13, 272 algorithmic B/px.  Kernels that carry
# those stages (the opsin kernel also does the S2 transform and S3, combine the S13 LUTs with
# S14/S15) are timed whole, so the extra fused work only lowers the figure.
BLUR_MASK_BYTES_PER_PX = 272.0
BLUR_MASK_STAGES = ("opsin_mhic", "edge_blur", "lowfreq_blur_h",
                    "lowfreq_blur_v", "mask_front", "mask_blur_h", "mask_blur_v", "combine", "diffmap_blur_h",
                    "diffmap_blur_v")

# Kernel symbol (rocprofv3 name prefix) of each profiled stage.
STAGE_SYMBOL = {
    "coeffs_to_linear": "gz::k_coeffs_to_linear(", "opsin_mhic": "gz::k_opsin_mhic_stream(",
    "edge_blur": "void gz::k_blur_stream<2>(", "edge_map": "gz::k_edge_map(",
    "block_diff": "gz::k_block_diff(", "lowfreq_blur_h": "void gz::k_blur_h4<3,",
    "lowfreq_blur_v": "void gz::k_blur_vstream<3>(", "low_freq": "gz::k_low_freq(",
    "mask_front": "gz::k_mask_stream(",
    "mask_blur_h": "void gz::k_blur_h4<4,", "mask_blur_v": "void gz::k_blur_vstream<4>(",
    "combine": "gz::k_combine(", "diffmap_blur_h": "void gz::k_blur_h4<5,",
    "diffmap_blur_v": "void gz::k_blur_vstream<5>(", "diffmap_final": "gz::k_diffmap_final(",
}


def measured_traffic(stage, w, h):
    """HBM bytes per launch of `stage` from the committed rocprofv3 PMC
    summary (tools/gpu_profile.sh -> profiles/*traffic*.json: FETCH_SIZE x2
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


# gfx950 vector issue: a wave64 VALU instruction occupies its SIMD-32 for 2
# cycles (MI355X_MICROARCH.md, execution model); 256 CUs x 4 SIMDs, 2.4 GHz.
VALU_SIMDS, VALU_CYCLES_PER_INST, CLOCK_HZ = 1024, 2, 2.4e9


def valu_issue(stage, w, h, avg_ms):
    """VALU issue utilisation of `stage`'s kernel: its measured vector
    instructions per launch (SQ_INSTS_VALU, committed rocprofv3 PMC summary
    profiles/*pmc_util_<WxH>.json) x 2 cycles over all SIMDs, against the
    launch's HIP-event duration -- how close a VALU-bound kernel is to the
    vector issue ceiling (the HBM roofline does not bound it)."""
    import glob
    sym = STAGE_SYMBOL.get(stage)
    if sym is None:
        return None
    sym = sym.split("(")[0]
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_util*%dx%d*.json" % (w, h))),
                    reverse=True):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        v = t.get(sym, {}).get("SQ_INSTS_VALU")
        if v:
            busy = v * VALU_CYCLES_PER_INST / VALU_SIMDS / CLOCK_HZ
            return {"valu_insts_per_launch": int(v), "issue_ms": round(busy * 1e3, 4),
                    "frac": round(busy / (avg_ms * 1e-3), 4), "source": os.path.relpath(f, ROOT)}
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


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local, dist


def cpu_baseline(width, height, quality, seconds_budget=25.0):
    """Reference `guetzli --c` (oracle/_ref) on host cores: concurrent single-
    threaded processes on distinct synthetic frames of the workload's kind,
    scaled down so the sample is ~10-30 s of CPU work."""
    ref = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")
    if not os.path.exists(ref):
        return {"value": None, "unit": "Mpixels/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/guetzli_ref not built"}
    import guetzli_amd as gz
    cores = max(1, min(8, len(os.sched_getaffinity(0))))
    # ~24.5 us/px single-threaded (survey: 1080p in 47-51 s); size the frame so
    # each process runs ~seconds_budget / cores ... capped to a quarter frame.
    sw, sh = width // 2, height // 2
    tmp = tempfile.mkdtemp(prefix="gz_cpu_")
    procs = []
    t0 = time.time()
    for i in range(cores):
        rgb = gz.synthetic_frame(1000 + i, sw, sh)
        path = os.path.join(tmp, "f%d.rgb" % i)
        rgb.tofile(path)
        procs.append(subprocess.Popen([ref, "encode", path, str(sw), str(sh), str(quality),
                                       os.path.join(tmp, "f%d.jpg" % i), "c"],
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL))
    outs = [json.loads(p.communicate()[0]) for p in procs]
    wall = time.time() - t0
    px = cores * sw * sh
    return {"value": px / wall / 1e6, "unit": "Mpixels/s", "cores": cores, "kind": "reference",
            "sample": "%d concurrent single-threaded `guetzli --c` processes, one synthetic "
                      "%dx%d q%d frame each (seeds 1000..%d), %.1f s wall, %.1f s CPU" % (
                          cores, sw, sh, quality, 999 + cores, wall,
                          sum(o["seconds"] for o in outs)),
            "per_process_seconds": [round(o["seconds"], 2) for o in outs]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=95)
    ap.add_argument("--frames-per-step", type=int, default=8,
                    help="frames per GPU per step, encoded concurrently")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world, rank, local, dist = dist_setup(args.gpus)
    import torch
    import guetzli_amd as gz
    from guetzli_amd import sharding

    dev = local
    torch.cuda.set_device(dev)
    w, h, q = args.width, args.height, args.quality
    params = gz.Params.for_quality(q)
    nsteps = args.warmup + args.steps
    # distinct frames per (rank, step, slot), uploaded to HBM before timing
    frames = []
    for s in range(nsteps):
        row = []
        for f in range(args.frames_per_step):
            seed = rank * 100000 + s * 100 + f
            rgb = gz.synthetic_frame(seed, w, h)
            row.append(torch.from_numpy(rgb.reshape(-1)).to(f"cuda:{dev}"))
        frames.append(row)
    torch.cuda.synchronize()

    pool = concurrent.futures.ThreadPoolExecutor(max_workers=args.frames_per_step)

    def encode(t):
        return gz.process_device(t.data_ptr(), w, h, params, device=dev, return_stats=True)

    def step(s):
        res = list(pool.map(encode, frames[s]))
        out = [r[0] for r in res]
        if dist is not None:
            # the final gather of the JPEG byte strings over RCCL/xGMI
            gathered = sharding.gather_bytes(out, dist, "cuda:%d" % dev)
            assert gathered[rank] == out
        return [len(o) for o in out], [r[1] for r in res]

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
    keys = ("seconds_total", "seconds_setup", "seconds_write", "seconds_quantize",
            "seconds_backend", "seconds_compare", "seconds_zeroing")
    for s in range(args.warmup, nsteps):
        sizes, stats = step(s)
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
    cpu_per_frame = ((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / (
        args.steps * args.frames_per_step)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # isolated frame: latency, host breakdown and per-kernel HIP-event timing
    gz.profile_reset()
    gz.profile_enable(True)
    t1 = time.perf_counter()
    _, st1 = encode(frames[0][0])
    single_s = time.perf_counter() - t1
    gz.profile_enable(False)
    prof = gz.profile_read()
    host = {}
    for k in ("seconds_total", "seconds_setup", "seconds_write", "seconds_quantize",
              "seconds_backend", "seconds_compare", "seconds_zeroing"):
        host[k] = getattr(st1, k)
    host.update(gz.last_process_detail())

    if rank != 0:
        pool.shutdown()
        if dist is not None:
            dist.destroy_process_group()
        return
    total_px = world * args.steps * args.frames_per_step * w * h
    value = total_px / elapsed / 1e6

    # roofline of the dominant kernel of the Butteraugli pass (by total time
    # in the isolated, HIP-event-timed frame)
    bpp = stage_bytes_per_px()
    rows = []
    for name, (cnt, ms) in prof.items():
        if name in bpp and cnt:
            rows.append((ms, name, cnt))
    rows.sort(reverse=True)
    roof = None
    stages = {}
    for ms, name, cnt in rows:
        avg = ms / cnt
        gbs = bpp[name] * w * h / (avg * 1e-3) / 1e9
        stages[name] = {"launches": cnt, "avg_ms": round(avg, 4), "algo_GBps": round(gbs, 1)}
    if rows:
        ms, name, cnt = rows[0]
        avg = ms / cnt
        achieved = bpp[name] * w * h / (avg * 1e-3) / 1e9
        traffic, tsrc = measured_traffic(name, w, h)
        roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": tsrc,
                "algo_bytes_per_launch": int(bpp[name] * w * h),
                "avg_launch_ms": round(avg, 4)}
        vi = valu_issue(name, w, h, avg)
        if vi:
            roof["valu_issue"] = vi
    bm_ms = sum(stages[k]["avg_ms"] for k in BLUR_MASK_STAGES if k in stages)
    blur_mask = None
    if bm_ms > 0:
        bm_bytes = BLUR_MASK_BYTES_PER_PX * w * h
        blur_mask = {"algo_bytes": int(bm_bytes), "ms": round(bm_ms, 4),
                     "achieved_GBps": round(bm_bytes / (bm_ms * 1e-3) / 1e9, 1),
                     "frac": round(bm_bytes / (bm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "stages": [k for k in BLUR_MASK_STAGES if k in stages]}
        # measured HBM bytes of the same launches (committed PMC summary of
        # this frame size), where every stage has one
        tr = [measured_traffic(k, w, h)[0] for k in blur_mask["stages"]]
        if tr and all(t is not None for t in tr):
            blur_mask["traffic"] = int(sum(tr))
            blur_mask["traffic_GBps"] = round(sum(tr) / (bm_ms * 1e-3) / 1e9, 1)
    cp = prof.get("compare_pass")
    pass_bytes = sum(bpp.values()) * w * h
    compare_pass = None
    if cp and cp[0]:
        avg = cp[1] / cp[0]
        compare_pass = {"launches": cp[0], "avg_ms": round(avg, 4),
                        "algo_bytes": int(pass_bytes),
                        "algo_GBps": round(pass_bytes / (avg * 1e-3) / 1e9, 1)}
    bz = prof.get("block_zeroing")

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
        "config": {"workload": "%d concurrent synthetic %dx%d sRGB frames per GPU per step, "
                               "q=%d, guetzli::Process end to end (each frame = BASELINE "
                               "configs[1]; 8 per GPU = configs[3]'s per-GPU share)" % (
                                   args.frames_per_step, w, h, q),
                   "width": w, "height": h, "quality": q,
                   "frames_per_gpu_per_step": args.frames_per_step,
                   "parallelism": "image-sharded over %d GPU(s)%s" % (
                       world, ", RCCL all_gather of JPEG bytes" if world > 1 else ""),
                   "search_iterations": iters},
        "roofline": roof,
        "compare_pass": compare_pass,
        "blur_mask_pass": blur_mask,
        "block_zeroing": {"launches": bz[0], "avg_ms": round(bz[1] / bz[0], 3)} if bz else None,
        "stages": stages,
        "concurrent_frame_breakdown_seconds": {k: round(v, 4) for k, v in conc.items()},
        "host_cpu_seconds_per_frame": round(cpu_per_frame, 4),
        "single_frame": {"seconds": round(single_s, 4),
                         "Mpixels_per_s": round(w * h / single_s / 1e6, 4),
                         "iterations": st1.iterations,
                         "host_breakdown_seconds": {k: round(v, 4) for k, v in host.items()}},
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(w, h, q)
    print(json.dumps(out))
    pool.shutdown()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
