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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=8192)
    ap.add_argument("--height", type=int, default=8192)
    ap.add_argument("--quality", type=int, default=84)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--warmup", type=int, default=0,
                    help="untimed encodes of the frame first (engine creation, first-touch)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    import torch
    import guetzli_amd as gz
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
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
    t0 = time.perf_counter()
    data, st = gz.process_strips(rgb, w, h, coll, params, device=local, return_stats=True)
    elapsed = time.perf_counter() - t0
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
           "detail": gz.last_process_detail()}
    if args.check and world == 1:
        t1 = time.perf_counter()
        ref = gz.process(rgb, w, h, params, device=local)
        out["single_engine_seconds"] = round(time.perf_counter() - t1, 3)
        out["single_engine_identical"] = ref == data
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
