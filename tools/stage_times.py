#!/usr/bin/env python3
"""Per-kernel (GZ_TIMED region) times of one isolated end-to-end encode.

  python tools/stage_times.py [--width W] [--height H] [--quality Q]

Encodes one synthetic frame untimed (warm-up), then again with the library's
HIP-event profiling on, and prints every region's launches, average and
total ms, sorted by total."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--quality", type=int, default=95)
    args = ap.parse_args()
    import guetzli_amd as gz
    rgb = gz.synthetic_frame(0, args.width, args.height)
    params = gz.Params.for_quality(args.quality)
    gz.process(rgb, args.width, args.height, params)
    gz.profile_reset()
    gz.profile_enable(True)
    t0 = time.perf_counter()
    gz.process(rgb, args.width, args.height, params)
    wall = time.perf_counter() - t0
    gz.profile_enable(False)
    detail = gz.last_process_detail()
    p = gz.profile_read()
    tot = sum(v[1] for v in p.values())
    print(f"frame {args.width}x{args.height}: wall {wall * 1e3:.1f} ms, timed regions {tot:.2f} ms")
    print("host detail:", {k: round(v, 4) for k, v in detail.items()})
    for k, (n, ms) in sorted(p.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:28s} {n:5d} x {ms / max(n, 1):8.4f} ms = {ms:8.3f} ms")


if __name__ == "__main__":
    main()
