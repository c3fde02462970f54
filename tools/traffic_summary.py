#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, KB per dispatch), corrected by measured
bytes-per-count factors.

  python tools/traffic_summary.py DIR [--factors profiles/round2_fetch_calibration.json]
  python tools/traffic_summary.py --calibrate CALIB_DIR   (tools/micro/fetch_calib runs)

FETCH_SIZE is not a byte count on gfx950: MI355X_MICROARCH.md measured it at
exactly half the bytes of 16-B-per-lane streaming reads.  The factor for the
access widths the kernels actually use (4 / 8 / 16 B per lane, partial lines)
comes from --calibrate over tools/micro/fetch_calib.hip (known byte counts,
1 GiB buffers past the Infinity Cache) and is applied per kernel by its
dominant global-load width (static instruction counts of the gfx950 code).
Prints JSON {kernel: {"launches", "fetch_bytes", "write_bytes",
"traffic_bytes", "read_width"}}."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# dominant global load width (bytes per lane) of each kernel, from the
# gfx950 assembly (global_load_dword / _dwordx2 / _dwordx4 counts)
READ_WIDTH = {"k_blur_vstream": 8, "k_block_diff2": 8, "k_block_diff": 8, "k_jpeg_stage": 16}


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


def calibrate(d):
    """bytes per counted byte, by access pattern, from the fetch_calib runs."""
    known = json.load(open(os.path.join(d, "bytes.json")))
    fetch = load(d, "FETCH_SIZE")
    write = load(d, "WRITE_SIZE")
    out = {"read": {}, "write": {}, "raw": {}}
    for k, vals in list(fetch.items()) + list(write.items()):
        # "void k_read<HIP_vector_type<float, 2u> >(...)" -> "k_read<float2>"
        short = k.split("(")[0].replace("void ", "")
        short = short.replace("HIP_vector_type<float, 2u> ", "float2")
        short = short.replace("HIP_vector_type<float, 4u> ", "float4")
        name = short.split(" ")[-1]
        for key, b in known.items():
            if key.replace("<", "").replace(">", "") == name.replace("<", "").replace(">", ""):
                counted = 1024.0 * sum(vals) / len(vals)
                kind = "write" if name.startswith("k_write") else "read"
                ctr_vals = fetch.get(k) if kind == "read" else write.get(k)
                if not ctr_vals:
                    continue
                counted = 1024.0 * sum(ctr_vals) / len(ctr_vals)
                out[kind][key] = b / counted if counted else None
                out["raw"][key] = {"bytes": b, "counted_bytes": counted}
    return out


def factor_for(kernel, factors):
    width = 4
    for k, v in READ_WIDTH.items():
        if k in kernel:
            width = v
    key = {4: "k_read<float>", 8: "k_read<float2>", 16: "k_read<float4>"}[width]
    f = (factors or {}).get("read", {}).get(key)
    return width, (f if f else 2.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?")
    ap.add_argument("--calibrate")
    ap.add_argument("--factors", default=os.path.join(ROOT, "profiles",
                                                       "round2_fetch_calibration.json"))
    args = ap.parse_args()
    if args.calibrate:
        print(json.dumps(calibrate(args.calibrate), indent=1, sort_keys=True))
        return
    factors = json.load(open(args.factors)) if os.path.exists(args.factors) else None
    wf = (factors or {}).get("write", {}).get("k_write<float>") or 1.0
    fetch = load(args.dir, "FETCH_SIZE")
    write = load(args.dir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        n = max(len(f), len(w))
        width, rf = factor_for(k, factors)
        fb = rf * 1024 * sum(f) / len(f) if f else None
        wb = wf * 1024 * sum(w) / len(w) if w else None
        out[k] = {"launches": n, "fetch_bytes": fb, "write_bytes": wb,
                  "traffic_bytes": (fb or 0) + (wb or 0), "read_width": width,
                  "fetch_factor": rf, "write_factor": wf}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
