#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 kernel trace (CSV).

  python tools/busy_frac.py gpurun_out/prof8/.../run_kernel_trace.csv [--window MS]

Merges the [start, end] intervals of all kernels (any stream) and prints the
busy fraction over the whole trace and over the busiest `--window` ms span
(the timed region of a bench run), plus the top kernels by summed time."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=300.0)
    args = ap.parse_args()
    iv = []
    per = collections.Counter()
    with open(args.trace) as f:
        for row in csv.DictReader(f):
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            iv.append((s, e))
            per[row["Kernel_Name"].split("(")[0][:60]] += e - s
    iv.sort()
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    span = merged[-1][1] - merged[0][0]
    busy = sum(e - s for s, e in merged)
    print(f"trace span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({busy / span:.1%})")
    # busiest window
    w = int(args.window * 1e6)
    best, lo = (0, 0), 0
    starts = [s for s, _ in merged]
    for i, (s, _) in enumerate(merged):
        t_end = s + w
        tot = 0
        for s2, e2 in merged[i:]:
            if s2 >= t_end:
                break
            tot += min(e2, t_end) - s2
        if tot > best[0]:
            best = (tot, s)
        if i > 2000:
            break
    print(f"busiest {args.window:.0f} ms window: {best[0] / w:.1%} busy")
    total = sum(per.values())
    for name, t in per.most_common(15):
        print(f"  {t / 1e6:9.2f} ms  {t / total:6.1%}  {name}")


if __name__ == "__main__":
    main()
