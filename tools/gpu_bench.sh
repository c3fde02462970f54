#!/bin/bash
# GPU-box bench + kernel-trace profile.  Each GPU step time-limited; stops on
# anything other than success.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py ${GZ_BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $rc -ne 0 ] && exit $rc
if [ -n "${GZ_PROFILE-1}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
    -- python bench.py --steps 2 --warmup 1 --frames-per-step 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.err
  find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
