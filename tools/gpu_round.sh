#!/bin/bash
# Round checkpoint on the GPU box: -m gpu tests, smoke, the default bench
# line, and profiles of the bench's isolated frame at 1080p and 4K: kernel
# trace + stats, HBM traffic (FETCH_SIZE / WRITE_SIZE passes, corrected by
# the committed calibration) and the SQ counters by instruction type (the
# FP64-aware VALU ceiling in bench.py reads them).  One rocprofv3 pass per
# counter group, each under its own time limit; stops at the first failure.
# GZ_SKIP_TESTS=1 skips the tests, GZ_SIZES overrides the sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r${GZ_ROUND:-4}
mkdir -p $O
if [ -z "$GZ_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
if [ -z "$GZ_SKIP_BENCH" ]; then
  timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  head -c 300 $O/bench.json; echo
fi
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
avail() {  # the counters of "$@" that rocprofv3 -L lists
  local out=""
  for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done
  echo $out
}
G1=$(avail SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32)
G2=$(avail SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES)
G3=$(avail SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM)
G4=$(avail SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS)
for sz in ${GZ_SIZES:-1920x1080x95 3840x2160x90}; do
  IFS=x read -r W H Q <<< "$sz"
  P=$O/prof_${W}x${H}
  rm -rf $P; mkdir -p $P
  BARGS="--steps 1 --warmup 1 --frames-per-step 1 --no-cpu-baseline --no-large-frame --no-uhd-frame --width $W --height $H --quality $Q"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv \
    -- python bench.py $BARGS > $P/bench.json 2> $P/trace.err || { tail -5 $P/trace.err; exit 1; }
  echo "trace ${W}x${H} ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr -d $P/pmc_$ctr -o run --output-format csv \
      -- python bench.py $BARGS > /dev/null 2> $P/pmc_$ctr.err || { tail -5 $P/pmc_$ctr.err; exit 1; }
  done
  python tools/traffic_summary.py $P > $P/traffic.json || exit 1
  i=0
  for G in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i + 1))
    [ -z "$G" ] && continue
    timeout -k 10 600 rocprofv3 --pmc $G -d $P/sq$i -o run --output-format csv \
      -- python bench.py $BARGS > /dev/null 2> $P/sq$i.err || { tail -5 $P/sq$i.err; exit 1; }
  done
  python tools/pmc_summary.py $P --json > $P/pmc_util.json || exit 1
  echo "pmc ${W}x${H} ok"
done
