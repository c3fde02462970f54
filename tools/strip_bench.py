#!/usr/bin/env python3
"""One large frame split over the GPUs of a node by row strips (BASELINE
configs[4]: 8192x8192 q=84 over 4 MI355X; strong scaling).

  python tools/strip_bench.py [--width 8192 --height 8192 --quality 84] [--check]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
      tools/strip_bench.py ...

Each rank passes the whole synthetic frame to gz_process_rgb_strips with its
own GPU; the exchange (block maxima, zeroing candidates) is an all-gather
over RCCL (nccl backend) for N > 1.  Prints one JSON line on rank 0.
--check (N = 1): also encodes the frame with the single-engine path
(gz_process_rgb) and compares the bytes."""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=8192)
    ap.add_argument("--height", type=int, default=8192)
    ap.add_argument("--quality", type=int, default=84)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--warmup", type=int, default=0,
                    help="untimed encodes of the frame first (engine creation, first-touch)")
    ap.add_argument("--backend", default="nccl",
                    help="nccl (RCCL over xGMI, one GPU per rank) or gloo (host exchange)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on device 0 (rehearsal of the split on one GPU; gloo)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch
    import guetzli_amd as gz
    # the ranks' host work runs on the library's pool; torch's intra-op
    # threads (the gathered blocks' copies) would spin after each collective
    # on every rank at once
    torch.set_num_threads(1)
    dist = None
    if args.one_device:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "gloo":
            dist.init_process_group("gloo")
            coll = gz.Collectives.from_torch(dist, "cpu")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            coll = gz.Collectives.from_torch(dist, "cuda:%d" % local)
    else:
        coll = gz.Collectives(0, 1, lambda b: b)
    w, h = args.width, args.height
    rgb = gz.synthetic_frame(args.seed, w, h)
    params = gz.Params.for_quality(args.quality)
    for _ in range(args.warmup):
        process_strips_once = gz.process_strips(rgb, w, h, coll, params, device=local)
        del process_strips_once
    if dist is not None:
        dist.barrier()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    th0 = _thread_cpu()
    t0 = time.perf_counter()
    data, st = gz.process_strips(rgb, w, h, coll, params, device=local, return_stats=True)
    elapsed = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    th1 = _thread_cpu()
    threads = {}
    import threading
    main_tid = str(threading.get_native_id())
    per_tid = []
    for k, (c, n) in th1.items():
        d = c - th0.get(k, (0.0, n))[0]
        threads[n] = threads.get(n, 0.0) + d
        per_tid.append((d, ("main:" if k == main_tid else "") + n))
    per_tid.sort(reverse=True)
    detail = gz.last_process_detail()
    host_cpu = [cpu]
    if dist is not None:
        c = torch.tensor([cpu] * world, dtype=torch.float64)
        if args.backend != "gloo":
            c = c.to("cuda:%d" % local)
        cs = [torch.zeros_like(c[:1]) for _ in range(world)]
        dist.all_gather(cs, c[:1])
        host_cpu = [float(x.item()) for x in cs]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % local)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    out = {"metric": "Mpixels/s, one frame split over GPUs (row strips + halo)",
           "value": round(w * h / elapsed / 1e6, 4), "unit": "Mpixels/s", "n_gpus": world,
           "scaling": "strong", "seconds": round(elapsed, 3), "width": w, "height": h,
           "quality": args.quality, "iterations": st.iterations, "bytes": len(data),
           "sha256": hashlib.sha256(data).hexdigest(),
           "rank0": {k: round(getattr(st, k), 3) for k in (
               "seconds_compare", "seconds_zeroing", "seconds_write", "seconds_quantize",
               "seconds_backend", "seconds_setup")},
           "strip": gz.strip_layout(w, h, world, rank), "warmup": args.warmup,
           "host_cpu_seconds_per_rank": [round(x, 3) for x in host_cpu],
           "rank0_thread_cpu_seconds": {n: round(c, 3) for n, c in
                                        sorted(threads.items(), key=lambda x: -x[1]) if c > 0.01},
           "rank0_top_threads": [[n, round(c, 3)] for c, n in per_tid[:8]],
           "detail": detail}
    if args.check and rank == 0:
        # the single-engine path on this rank's GPU (the others wait)
        ref = gz.process(rgb, w, h, params, device=local)  # (warm: engine pooled)
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t1 = time.perf_counter()
        ref = gz.process(rgb, w, h, params, device=local)
        out["single_engine_seconds"] = round(time.perf_counter() - t1, 3)
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        out["single_engine_host_cpu_seconds"] = round(
            (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime), 3)
        out["single_engine_identical"] = ref == data
    if dist is not None:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
