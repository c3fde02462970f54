#!/bin/bash
# Block-zeroing search diagnostics at 1080p: per-phase cycle totals
# (GZ_ZEROING_TIMERS) and SQ utilisation counters (own --pmc pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/zprobe
export TMPDIR=/tmp
timeout -k 10 120 python tools/compare_loop.py --compares 1 --zeroing > gpurun_out/zprobe/plain.json 2>&1 || exit $?
GZ_ZEROING_TIMERS=1 timeout -k 10 120 python tools/compare_loop.py --compares 1 --zeroing > gpurun_out/zprobe/timers.json 2>&1 || exit $?
rm -rf gpurun_out/zprobe/sq
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
  -d gpurun_out/zprobe/sq -o run --output-format csv -- python tools/compare_loop.py --compares 1 --zeroing \
  > gpurun_out/zprobe/sq.json 2> gpurun_out/zprobe/sq.err || exit $?
python tools/pmc_summary.py gpurun_out/zprobe/sq --filter zeroing
cat gpurun_out/zprobe/plain.json gpurun_out/zprobe/timers.json
