#!/bin/bash
# Utilisation counters (VALU / TA / LDS / waves) of the block-zeroing search
# and the Compare kernels at 1080p (tools/compare_loop.py --zeroing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmcz
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES TA_TA_BUSY_sum GRBM_GUI_ACTIVE \
  -d gpurun_out/pmcz -o run --output-format csv -- python tools/compare_loop.py --compares 2 --zeroing \
  > gpurun_out/pmcz.json 2> gpurun_out/pmcz.err || exit $?
cat gpurun_out/pmcz.json
