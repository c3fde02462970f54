#!/bin/bash
# A/B of library builds on one box: for each build (a path to an alternative
# libguetzli_hip.so, or "default" for the in-tree one) a kernel-trace run of
# the concurrent bench (per-kernel avg ms; skipped with GZ_AB_NO_PROF=1),
# then GZ_AB_RUNS rounds of plain bench lines, the builds interleaved within
# each round (so drift of the box hits every build alike).
#   bash tools/gpu_ab.sh default _variants/base/libguetzli_hip.so
# Output: gpurun_out/ab/<i>_*.  Each GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
BENCH="bench.py --steps ${GZ_AB_STEPS:-4} --warmup 1 --no-cpu-baseline --no-large-frame --no-uhd-frame"
use() {
  if [ "$1" = default ]; then unset GZ_LIB_PATH; else export GZ_LIB_PATH=$PWD/$1; fi
}
if [ -z "$GZ_AB_NO_PROF" ]; then
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    use "$lib"
    echo "== $i: $lib"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$i -o run --output-format csv \
      -- python $BENCH > $O/${i}_prof.json 2> $O/${i}_prof.err || { tail $O/${i}_prof.err; exit 1; }
    python - $O/prof$i/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("  %-40s calls %6s avg %8.1f us  %5.1f%%" % (r["Name"].split("(")[0][-40:], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
  done
fi
for r in $(seq ${GZ_AB_RUNS:-2}); do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    use "$lib"
    f=$O/${i}_bench$r
    timeout -k 10 200 python $BENCH > $f.json 2> $f.err || { tail $f.err; exit 1; }
    # throughput, host CPU per frame, and the isolated frame's per-region ms
    python -c "
import json
d = json.loads(open('$f.json').read().strip().splitlines()[-1])
g = d.get('gpu_regions_ms_per_frame', {})
print('$i', '$lib'[-28:], d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['verified']['bit_exact'],
      {k: g.get(k) for k in '${GZ_AB_REGIONS:-jpeg_code jpeg_stage bulk_apply block_zeroing}'.split()})"
  done
done
