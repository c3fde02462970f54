#!/bin/bash
# Round checkpoint on the GPU box: all -m gpu tests + smoke, the default
# bench line, and the rocprofv3 kernel-trace / PMC-traffic profiles at 1080p
# and 4K (tools/gpu_profile.sh).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  > gpurun_out/round_tests.log 2>&1 || { tail -30 gpurun_out/round_tests.log; exit 1; }
tail -3 gpurun_out/round_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/round_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/round_bench.json 2> gpurun_out/round_bench.err || exit $?
head -c 600 gpurun_out/round_bench.json; echo
GZ_PROF_TAG=prof1080 bash tools/gpu_profile.sh || exit $?
GZ_PROF_W=3840 GZ_PROF_H=2160 GZ_PROF_TAG=prof4k GZ_PROF_BENCH_ARGS="--quality 90" bash tools/gpu_profile.sh || exit $?
mkdir -p gpurun_out/util
for sz in "1920 1080" "3840 2160"; do
  set -- $sz
  rm -rf gpurun_out/pmck
  GZ_PMC_ARGS="--width $1 --height $2 --compares 3" bash tools/gpu_pmc_kernels.sh > /dev/null 2>&1 || exit $?
  python tools/pmc_summary.py gpurun_out/pmck --json > gpurun_out/util/pmc_util_$1x$2.json || exit $?
  echo "pmc util $1x$2 ok"
done
