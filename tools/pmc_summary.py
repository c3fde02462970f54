#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs.

  python tools/pmc_summary.py gpurun_out/pmck [--filter NAME]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", action="store_true", help="per-dispatch averages as JSON")
    args = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    names = set()
    for f in glob.glob(os.path.join(args.root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0] if args.json else row["Kernel_Name"].split("(")[0][:48]
                if args.filter not in k:
                    continue
                c = row["Counter_Name"]
                names.add(c)
                acc[k][c] += float(row["Counter_Value"])
                cnt[k][(c, row.get("Dispatch_Id", ""))] = 1
    cols = sorted(names)
    if args.json:
        import json
        out = {}
        for k in sorted(acc):
            nd = max(1, len({d for (c, d) in cnt[k] if c == cols[0]}))
            out[k] = {c: acc[k][c] / nd for c in cols}
        print(json.dumps(out, indent=1, sort_keys=True))
        return
    print("kernel".ljust(48), " ".join(c[3:15].rjust(12) for c in cols))
    for k in sorted(acc):
        nd = max(1, len({d for (c, d) in cnt[k] if c == cols[0]}))
        print(k.ljust(48), " ".join(("%.3g" % (acc[k][c] / nd)).rjust(12) for c in cols))


if __name__ == "__main__":
    main()
