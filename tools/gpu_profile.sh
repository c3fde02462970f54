#!/bin/bash
# Profiles for profiles/: (1) rocprofv3 kernel trace + stats of the isolated
# single-frame bench (the configuration bench.py's roofline is measured on),
# (2)/(3) HBM traffic counters FETCH_SIZE and WRITE_SIZE in separate --pmc
# passes (they do not fit one pass on gfx950) over a fixed Compare workload.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${GZ_PROF_W:-1920}; H=${GZ_PROF_H:-1080}
OUT=gpurun_out/${GZ_PROF_TAG:-prof}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python bench.py --steps 2 --warmup 1 --frames-per-step 1 --no-cpu-baseline \
     --width $W --height $H ${GZ_PROF_BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/trace.err" || exit $?
echo "trace ok"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr -d "$OUT/pmc_$ctr" -o run --output-format csv \
    -- python tools/compare_loop.py --width $W --height $H --compares 3 --zeroing \
    > "$OUT/pmc_$ctr.json" 2> "$OUT/pmc_$ctr.err" || exit $?
  echo "pmc $ctr ok"
done
python tools/traffic_summary.py "$OUT" > "$OUT/traffic.json" && echo "summary ok"
