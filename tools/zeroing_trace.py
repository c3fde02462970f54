#!/usr/bin/env python3
"""Timeline of one k_block_zeroing launch: encodes a synthetic frame with
GZ_BZ_TRACE set (the engine records each block's start / end on the 100 MHz
wall clock, its greedy step count and when its candidate list was sorted; with a library built with
-DGZ_BZ_PHASES also its shader-clock cycles per search phase) and reports the span, the per-block
duration distribution, how much of the span the longest blocks alone take
(the launch's critical path) and how many blocks are in flight over time.

  python tools/zeroing_trace.py [W H [QUALITY]]      (GPU box)"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
    q = int(sys.argv[3]) if len(sys.argv) > 3 else 95
    path = os.path.join(ROOT, "gpurun_out", "bz_trace_%dx%d.bin" % (w, h))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    env = dict(os.environ, GZ_BZ_TRACE=path)
    code = ("import sys; sys.path.insert(0, %r); import guetzli_amd as gz; "
            "rgb = gz.synthetic_frame(0, %d, %d); gz.process(rgb, %d, %d, gz.Params.for_quality(%d))"
            % (os.path.join(ROOT, "guetzli-cuda-opencl_amd", "python"), w, h, w, h, q))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    raw = np.fromfile(path, dtype=np.int64)
    nb = ((w + 7) // 8) * ((h + 7) // 8)
    words = raw.size // nb
    t = raw.reshape(nb, words)
    phases = None
    if words >= 12:
        names = ["pixel", "dc_edge_sums", "row_fft", "col_fft", "csf", "ac_lf", "error", "choose_update"]
        ph = t[:, 4:12].sum(axis=0).astype(np.float64)
        phases = {n: round(float(v / ph.sum()), 4) for n, v in zip(names, ph)}
        phases["cycles_per_step"] = round(float(ph.sum() / max(int(t[:, 2].sum()), 1)), 1)
    census = None
    if words >= 14:
        # resident blocks per CU over time from HW_ID (cu 11:8, sh 12, se 15:13)
        # and XCC_ID: the maximum and the mean at 20 instants
        hw, xcc = t[:, 12].astype(np.int64), t[:, 13].astype(np.int64) & 0xf
        cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xf)
        simd = (cu << 2) | ((hw >> 4) & 3)
        st, en = t[:, 0], t[:, 1]
        inst = np.linspace(st.min(), en.max(), 22)[1:-1]
        per_cu, per_simd = [], []
        for m in inst:
            live = (st <= m) & (en > m)
            _, c = np.unique(cu[live], return_counts=True)
            _, c2 = np.unique(simd[live], return_counts=True)
            per_cu.append((int(c.max()) if c.size else 0, round(float(c.mean()), 2) if c.size else 0))
            per_simd.append(int(c2.max()) if c2.size else 0)
        census = {"cus_seen": int(np.unique(cu).size), "per_cu_max_mean": per_cu, "per_simd_max": per_simd}
    start, end, steps, sorted_t = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    setup = (sorted_t - start) / 100.0  # us: reference opsin, IDCT, candidate keys + sort
    t0 = start.min()
    dur = (end - start) / 100.0  # us
    span = (end.max() - t0) / 100.0
    order = np.argsort(-dur)
    bins = np.linspace(0, span, 21)
    mid = (bins[:-1] + bins[1:]) / 2
    s_us, e_us = (start - t0) / 100.0, (end - t0) / 100.0
    inflight = [int(np.sum((s_us <= m) & (e_us > m))) for m in mid]
    per_step = dur / np.maximum(steps, 1)
    print(json.dumps({
        "width": w, "height": h, "quality": q, "blocks": int(len(t)),
        "span_us": round(span, 1),
        "block_us": {"mean": round(float(dur.mean()), 2), "median": round(float(np.median(dur)), 2),
                     "p99": round(float(np.percentile(dur, 99)), 1), "max": round(float(dur.max()), 1)},
        "setup_us": {"mean": round(float(setup.mean()), 2), "median": round(float(np.median(setup)), 2),
                     "p99": round(float(np.percentile(setup, 99)), 1), "sum": round(float(setup.sum()), 0)},
        "steps": {"mean": round(float(steps.mean()), 2), "max": int(steps.max()),
                  "total": int(steps.sum())},
        "us_per_step": {"median": round(float(np.median(per_step[steps > 0])), 3),
                        "p10": round(float(np.percentile(per_step[steps > 0], 10)), 3),
                        "p90": round(float(np.percentile(per_step[steps > 0], 90)), 3)},
        "longest_blocks": [{"block": int(b), "us": round(float(dur[b]), 1), "steps": int(steps[b]),
                            "start_us": round(float(s_us[b]), 1)} for b in order[:5]],
        "last_start_us": round(float(s_us.max()), 1),
        "inflight_over_time": inflight,
        "sum_block_us": round(float(dur.sum()), 0),
        "phase_share": phases,
        "census": census,
    }))


if __name__ == "__main__":
    main()
