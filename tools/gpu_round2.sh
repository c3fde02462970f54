#!/bin/bash
# Round-2 checkpoint on the GPU box: -m gpu tests, smoke, the default bench
# line, FETCH/WRITE_SIZE calibration, and profiles (kernel trace + stats of
# the bench's isolated frame at 1080p and 4K; HBM traffic and SQ counters of
# the bench workload itself).  Every GPU step has its own time limit; the
# script stops at the first failure.  GZ_R2_SKIP_TESTS=1 skips the tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
O=gpurun_out/r2
if [ -z "$GZ_R2_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { cat $O/bench.err | tail; exit 1; }
head -c 400 $O/bench.json; echo
# FETCH_SIZE / WRITE_SIZE calibration (known byte counts)
mkdir -p $O/calib
./tools/micro/fetch_calib > $O/calib/bytes.json || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/calib/pmc_$ctr -o run --output-format csv \
    -- ./tools/micro/fetch_calib > /dev/null 2> $O/calib/$ctr.err || exit 1
done
python tools/traffic_summary.py --calibrate $O/calib > $O/calib/factors.json && cat $O/calib/factors.json | head -30
for sz in "1920 1080 95" "3840 2160 90"; do
  set -- $sz
  P=$O/prof_$1x$2
  rm -rf $P; mkdir -p $P
  BARGS="--steps 1 --warmup 1 --frames-per-step 1 --no-cpu-baseline --width $1 --height $2 --quality $3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv \
    -- python bench.py $BARGS > $P/bench.json 2> $P/trace.err || exit 1
  echo "trace $1x$2 ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr -d $P/pmc_$ctr -o run --output-format csv \
      -- python bench.py $BARGS > /dev/null 2> $P/pmc_$ctr.err || exit 1
  done
  python tools/traffic_summary.py $P --factors $O/calib/factors.json > $P/traffic.json || exit 1
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d $P/pmc_sq -o run --output-format csv -- python bench.py $BARGS > /dev/null 2> $P/pmc_sq.err || exit 1
  python tools/pmc_summary.py $P/pmc_sq --json > $P/pmc_util.json || exit 1
  echo "pmc $1x$2 ok"
done
