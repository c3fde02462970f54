#!/usr/bin/env python3
"""Concurrency profile of a rocprofv3 kernel trace (CSV) of the concurrent bench.

  python tools/conc_profile.py <run_kernel_trace.csv> [--window MS]

Over the busiest --window ms span (the timed region): the GPU busy fraction,
the time-weighted distribution of the number of kernels running at once, the
busy fraction per hardware queue, and the idle gaps by length.  Answers
whether idle time comes from too few kernels in flight (queue structure, host
latency) or from kernels that do not fill the device."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=300.0)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q,
                         r["Kernel_Name"].split("(")[0][:48]))
    rows.sort()
    # busiest window by merged busy time
    w = int(args.window * 1e6)
    starts = [s for s, _, _, _ in rows]
    best_lo, best_busy = rows[0][0], -1
    ev = []
    for s, e, _, _ in rows:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()

    def busy_in(lo, hi):
        n, last, busy = 0, lo, 0
        for t, d in ev:
            t = min(max(t, lo), hi)
            if n > 0:
                busy += t - last
            last = t
            n += d
        return busy

    step = max(1, len(rows) // 200)
    for i in range(0, len(rows), step):
        lo = starts[i]
        b = busy_in(lo, lo + w)
        if b > best_busy:
            best_busy, best_lo = b, lo
    lo, hi = best_lo, best_lo + w
    # concurrency histogram + gaps
    hist = collections.Counter()
    gaps = []
    n, last = 0, lo
    for t, d in ev:
        tt = min(max(t, lo), hi)
        if tt > last:
            hist[n] += tt - last
            if n == 0:
                gaps.append(tt - last)
        last = tt
        n += d
    if hi > last:
        hist[n] += hi - last
    tot = sum(hist.values())
    print("window %.1f ms from t=%d: busy %.1f%%" % (w / 1e6, lo, 100.0 * (tot - hist[0]) / tot))
    print("kernels running at once (time share):")
    for k in sorted(hist):
        print("  %2d: %5.1f%%" % (k, 100.0 * hist[k] / tot))
    gaps.sort()
    if gaps:
        g = [x / 1e3 for x in gaps]
        print("idle gaps: %d, total %.2f ms, median %.1f us, p90 %.1f us, max %.1f us; gaps > 50 us: %.1f%% of idle"
              % (len(g), sum(g) / 1e3, g[len(g) // 2], g[int(len(g) * 0.9)], g[-1],
                 100.0 * sum(x for x in g if x > 50) / max(sum(g), 1e-9)))
    perq = collections.defaultdict(list)
    for s, e, q, _ in rows:
        if e > lo and s < hi:
            perq[q].append((max(s, lo), min(e, hi)))
    print("per queue busy (merged):")
    for q, iv in sorted(perq.items(), key=lambda x: str(x[0])):
        iv.sort()
        m = []
        for s, e in iv:
            if m and s <= m[-1][1]:
                m[-1][1] = max(m[-1][1], e)
            else:
                m.append([s, e])
        print("  queue %s: %5.1f%% (%d kernels)" % (q, 100.0 * sum(e - s for s, e in m) / w, len(iv)))


if __name__ == "__main__":
    main()
