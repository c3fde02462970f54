#!/usr/bin/env python3
"""Host cost of concurrent encodes: N threads each encode `--steps` distinct
synthetic frames (device-resident input, as bench.py), and the per-frame
averages of the library's detail map (wall seconds per phase, the calling
thread's CPU seconds: thread_cpu_s, compare_thread_cpu_s) are printed with
the process's CPU seconds per frame.

  python tools/conc_detail.py [--threads 8] [--steps 3] [--width 1920 --height 1080 --quality 95]
"""
import argparse
import concurrent.futures
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=95)
    a = ap.parse_args()
    import torch
    import guetzli_amd as gz
    params = gz.Params.for_quality(a.quality)
    frames = [[torch.from_numpy(gz.synthetic_frame(1000 + 100 * s + t, a.width, a.height).reshape(-1)).to("cuda:0")
               for t in range(a.threads)] for s in range(a.steps + 1)]
    torch.cuda.synchronize()

    def enc(t):
        gz.process_device(t.data_ptr(), a.width, a.height, params, device=0)
        return gz.last_process_detail()

    pool = concurrent.futures.ThreadPoolExecutor(max_workers=a.threads)
    list(pool.map(enc, frames[0]))  # warm-up (engines, graphs)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    details = []
    for s in range(1, a.steps + 1):
        details.extend(pool.map(enc, frames[s]))
    wall = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    n = len(details)
    avg = {}
    for d in details:
        for k, v in d.items():
            avg[k] = avg.get(k, 0.0) + v / n
    print(json.dumps({"threads": a.threads, "frames": n, "wall_s": round(wall, 4),
                      "ms_per_frame": round(1e3 * wall / n, 2),
                      "process_cpu_s_per_frame": round(cpu / n, 4),
                      "detail_avg": {k: round(v, 4) for k, v in sorted(avg.items())}}, indent=1))


if __name__ == "__main__":
    main()
