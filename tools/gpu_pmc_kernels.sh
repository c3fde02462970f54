#!/bin/bash
# SQ stall counters of every kernel of a fixed Compare workload (own --pmc
# passes, no tracing domains).  Summarise with tools/pmc_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmck
export TMPDIR=/tmp
ARGS="${GZ_PMC_ARGS:---compares 3}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  -d gpurun_out/pmck/p1 -o run --output-format csv -- python tools/compare_loop.py $ARGS > gpurun_out/pmck/o1.json 2> gpurun_out/pmck/e1.txt &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d gpurun_out/pmck/p2 -o run --output-format csv -- python tools/compare_loop.py $ARGS > gpurun_out/pmck/o2.json 2> gpurun_out/pmck/e2.txt
echo "rc=$?"
