#!/bin/bash
# SQ counters of the block-zeroing kernel (its own --pmc pass, kernel filter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcz
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmcz/counters.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d gpurun_out/pmcz/sq -o run --output-format csv \
  -- python tools/compare_loop.py --compares 1 --zeroing > gpurun_out/pmcz/out.json 2> gpurun_out/pmcz/err.txt
echo "rc=$?"
