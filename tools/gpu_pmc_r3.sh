#!/bin/bash
# Round-3 counter passes for the kernels the verdict names (k_block_zeroing's
# instruction mix by type and its stall counters; the coder kernels): one
# rocprofv3 --pmc pass per counter group over one isolated 1080p frame of the
# bench, each under its own time limit.  Counters gfx950 does not expose are
# dropped from a group (checked against rocprofv3 -L first).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_r3
rm -rf $O; mkdir -p $O
BARGS="--steps 1 --warmup 1 --frames-per-step 1 --no-cpu-baseline --no-large-frame"
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { tail -5 $O/counters.txt; exit 1; }
avail() {  # the counters of "$@" that rocprofv3 -L lists
  local out=""
  for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done
  echo $out
}
G1=$(avail SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32)
G2=$(avail SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES)
G3=$(avail SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM)
G4=$(avail SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_F64 SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS)
echo "groups: [$G1] [$G2] [$G3] [$G4]" | tee $O/groups.txt
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i + 1))
  [ -z "$G" ] && continue
  timeout -k 10 300 rocprofv3 --pmc $G -d $O/p$i -o run --output-format csv \
    -- python bench.py $BARGS > /dev/null 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 1; }
  echo "pass $i ok"
done
python tools/pmc_summary.py $O --json > $O/pmc.json && echo summary ok
