#!/bin/bash
# Throughput sweep over concurrent frames per GPU (no CPU baseline, no rocprof).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${GZ_SWEEP_FRAMES:-4 8 16}; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --frames-per-step $f --no-cpu-baseline \
    > gpurun_out/sweep_$f.json 2> gpurun_out/sweep_$f.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/sweep_$f.json'));print($f, d['value'], d['ms_per_step'])"
done
