#!/bin/bash
# GPU-box step for a kernel change: the -m gpu tests on the in-tree library
# (all of them, or GZ_TEST_K=<pytest -k expression>), then interleaved
# per-kernel stage times of the variants under _variants/ (tools/variant_ab.sh;
# GZ_VARIANTS, GZ_AB_ARGS, GZ_AB_FILTER pass through), then optionally
# (GZ_BENCH=1) the default bench line of the in-tree library.  Each step has
# its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$GZ_SKIP_TESTS" ]; then
  K=()
  [ -n "$GZ_TEST_K" ] && K=(-k "$GZ_TEST_K")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread "${K[@]}" > gpurun_out/vtests.log 2>&1 || { tail -30 gpurun_out/vtests.log; exit 1; }
  tail -1 gpurun_out/vtests.log
fi
if [ -n "$GZ_VARIANTS" ]; then
  bash tools/variant_ab.sh || exit 1
fi
if [ -n "$GZ_BENCH" ]; then
  timeout -k 10 600 python bench.py ${GZ_BENCH_ARGS:---no-cpu-baseline --no-large-frame} \
    > gpurun_out/vbench.json 2> gpurun_out/vbench.err || { tail gpurun_out/vbench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/vbench.json')); print('bench', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['verified'], d['gpu_regions_ms_per_frame'])"
fi
