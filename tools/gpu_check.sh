#!/bin/bash
# One GPU visit: -m gpu tests, two default-shape bench lines (no 4K / 8192
# legs), a kernel trace of the concurrent bench (gpu_prof8.sh) with its
# concurrency profile, and the configs[4] strip bench.  Each step under its
# own time limit; stops at the first failure.  Output: gpurun_out/check/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-large-frame --no-uhd-frame \
    > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified']['bit_exact'])"
done
if [ -z "$GZ_CHECK_NO_TRACE" ]; then
  bash tools/gpu_prof8.sh > $O/prof8.txt 2>&1 || { tail $O/prof8.txt; exit 1; }
  python tools/conc_profile.py gpurun_out/prof8/run_kernel_trace.csv --window 150 > $O/conc.txt
  python tools/busy_frac.py gpurun_out/prof8/run_kernel_trace.csv --window 150 > $O/busy.txt
  head -12 $O/conc.txt
fi
if [ -z "$GZ_CHECK_NO_STRIPS" ]; then
  bash tools/gpu_strips.sh > $O/strips.txt 2>&1 || { tail -30 $O/strips.txt; exit 1; }
  cut -c1-400 $O/strips.txt
fi
