#!/usr/bin/env python3
"""Fixed Butteraugli workload for profiler passes (rocprofv3 --pmc / traces).

  python tools/compare_loop.py [--width W] [--height H] [--compares N] [--zeroing]

Runs N full Compare passes (graph-launched, as in the search loop) of a
synthetic frame against a globally re-quantized version of itself, plus
optionally one batched block-zeroing search.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--compares", type=int, default=5)
    ap.add_argument("--zeroing", action="store_true")
    args = ap.parse_args()
    import guetzli_amd as gz
    w, h = args.width, args.height
    rgb = gz.synthetic_frame(0, w, h)
    orig = gz.rgb_to_coeffs(rgb, w, h).reshape(3, -1, 64).astype(np.int32)
    q = np.array([[1 + (k % 9) for k in range(64)]] * 3)[:, None, :]
    r = np.fmod(orig, q)
    cur = (orig + np.where(2 * r > q, q - r, np.where(-2 * r > q, -q - r, -r))).astype(np.int16)
    target = gz.butteraugli_score_for_quality(95)
    cmp = gz.ButteraugliComparator(w, h, rgb, target)
    t0 = time.perf_counter()
    d = None
    for _ in range(args.compares):
        d = cmp.compare(cur.reshape(-1))
    t1 = time.perf_counter()
    out = {"width": w, "height": h, "compares": args.compares, "distance": float(d),
           "ms_per_compare": (t1 - t0) / args.compares * 1e3}
    if args.zeroing:
        t2 = time.perf_counter()
        z = cmp.block_zeroing_orders(cur.reshape(-1), orig.astype(np.int16).reshape(-1), target)
        out["zeroing_ms"] = (time.perf_counter() - t2) * 1e3
        out["zeroing_entries"] = int((z["block_err"] > 0).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
