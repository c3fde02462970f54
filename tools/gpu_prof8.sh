#!/bin/bash
# Kernel trace of the concurrent (8 frames/GPU) bench: GPU busy fraction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 ${GZ_ROCPROF_EXTRA:-} --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv \
  -- python bench.py --steps 2 --warmup 1 --frames-per-step ${GZ_FRAMES:-8} --no-cpu-baseline --no-large-frame --no-uhd-frame \
  > gpurun_out/prof8_bench.json 2> gpurun_out/prof8.err
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof8.err; cat gpurun_out/prof8_bench.json | cut -c1-300
exit $rc
