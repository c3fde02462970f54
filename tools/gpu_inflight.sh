#!/bin/bash
# The bench line over frames in flight (GZ_INFLIGHT, default "6 7 8 9 10"),
# GZ_RUNS interleaved rounds, each run under its own time limit; stops at
# the first failure.  Output: gpurun_out/inflight/<n>_<round>.json and one
# summary line per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/inflight
mkdir -p $O
for r in $(seq ${GZ_RUNS:-2}); do
  for n in ${GZ_INFLIGHT:-6 7 8 9 10}; do
    timeout -k 10 300 python bench.py --steps ${GZ_STEPS:-4} --warmup 1 --no-cpu-baseline --no-large-frame \
      --no-uhd-frame --in-flight $n > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail $O/${n}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['verified']['bit_exact'])" $O/${n}_$r.json $n
  done
done
