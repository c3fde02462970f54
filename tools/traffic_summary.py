#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from the two rocprofv3 --pmc passes of
tools/gpu_profile.sh (FETCH_SIZE and WRITE_SIZE, KB per dispatch).

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section).  Prints JSON:
{kernel: {"launches", "fetch_bytes", "write_bytes", "traffic_bytes"}}."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "pmc_" + counter, "**", "*counter_collection.csv"),
                      recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    d = sys.argv[1]
    fetch = load(d, "FETCH_SIZE")
    write = load(d, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        n = max(len(f), len(w))
        fb = 2.0 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        out[k] = {"launches": n, "fetch_bytes": fb, "write_bytes": wb,
                  "traffic_bytes": (fb or 0) + (wb or 0)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
