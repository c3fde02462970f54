#!/bin/bash
# Kernel iteration loop on the GPU box: parity tests (stage bit-exactness and
# known answers), then per-kernel stage times of one isolated frame at 1080p
# and 4K.  Every GPU step has its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q -p no:cacheprovider --timeout 300 \
  ${GZ_PYTEST_ARGS:-} > gpurun_out/iter_tests.log 2>&1
rc=$?
tail -5 gpurun_out/iter_tests.log
[ $rc -ne 0 ] && exit $rc
for sz in ${GZ_ITER_SIZES:-1920x1080x95 3840x2160x90}; do
  [ "$sz" = none ] && continue
  IFS=x read -r W H Q <<< "$sz"
  timeout -k 10 300 python tools/stage_times.py --width $W --height $H --quality $Q \
    > gpurun_out/iter_stages_${W}x${H}.txt 2>&1 || exit $?
  head -30 gpurun_out/iter_stages_${W}x${H}.txt
done
if [ -n "${GZ_ITER_PMC:-}" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/iter_pmc
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
    -d gpurun_out/iter_pmc -o run --output-format csv -- python tools/compare_loop.py --width 3840 --height 2160 --compares 2 \
    > gpurun_out/iter_pmc.json 2> gpurun_out/iter_pmc.err || exit $?
  python tools/pmc_summary.py gpurun_out/iter_pmc > gpurun_out/iter_pmc.txt && cat gpurun_out/iter_pmc.txt
fi
if [ -n "${GZ_ITER_PMC2:-}" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/iter_pmc2
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES TA_TA_BUSY_sum GRBM_GUI_ACTIVE \
    -d gpurun_out/iter_pmc2 -o run --output-format csv -- python tools/compare_loop.py --width 3840 --height 2160 --compares 2 \
    > gpurun_out/iter_pmc2.json 2> gpurun_out/iter_pmc2.err || exit $?
  python tools/pmc_summary.py gpurun_out/iter_pmc2 > gpurun_out/iter_pmc2.txt && cat gpurun_out/iter_pmc2.txt
fi
