#!/bin/bash
# GPU-box check of the current tree: -m gpu tests and smoke (unless
# GZ_SKIP_TESTS=1), then the bench's two schedules interleaved (the default
# single queue over the timed steps' frames vs --lockstep), each run under
# its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab
mkdir -p $O
if [ -z "$GZ_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
ARGS="--no-cpu-baseline --no-large-frame --steps ${GZ_AB_STEPS:-3} --warmup 1"
for r in 1 2; do
  for mode in stream lockstep; do
    extra=""
    [ $mode = lockstep ] && extra="--lockstep"
    timeout -k 10 300 python bench.py $ARGS $extra > $O/bench_${mode}_$r.json 2> $O/bench_${mode}_$r.err \
      || { tail $O/bench_${mode}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/bench_${mode}_$r.json')); print('$mode', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified'])"
  done
done
