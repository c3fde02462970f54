#!/usr/bin/env python3
"""Times the 4:2:0 pass (Params::force_420 / try_420) on a synthetic frame
next to the plain 4:4:4 encode, with the library's per-stage profile.

  python tools/bench420.py [W H [QUALITY]]     (GPU box)
Prints one JSON line per mode."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"))
import guetzli_amd as gz  # noqa: E402


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
    q = int(sys.argv[3]) if len(sys.argv) > 3 else 95
    rgb = gz.synthetic_frame(0, w, h)
    gz.process(rgb, w, h, gz.Params.for_quality(q))  # warm the engine pool
    for mode in ("444", "force_420", "try_420"):
        p = gz.Params.for_quality(q, force_420=mode == "force_420", try_420=mode == "try_420")
        t0 = time.perf_counter()
        data, st = gz.process(rgb, w, h, p, return_stats=True)
        dt = time.perf_counter() - t0
        detail = gz.last_process_detail()
        # a second run with per-launch timing (no graphs: slower, for the split)
        gz.profile_enable(True)
        gz.profile_reset()
        gz.process(rgb, w, h, p)
        prof = gz.profile_read()
        gz.profile_enable(False)
        kern = {n: [c, round(t, 3)] for n, (c, t) in prof.items() if t > 0.5}
        print(json.dumps({"mode": mode, "w": w, "h": h, "quality": q, "seconds": round(dt, 4),
                          "bytes": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                          "iterations": st.iterations, "compares": st.compares,
                          "seconds_zeroing": round(st.seconds_zeroing, 4),
                          "seconds_compare": round(st.seconds_compare, 4),
                          "seconds_write": round(st.seconds_write, 4),
                          "seconds_backend": round(st.seconds_backend, 4),
                          "seconds_quantize": round(st.seconds_quantize, 4),
                          "kernel_ms_total": kern, "detail": detail}), flush=True)


if __name__ == "__main__":
    main()
