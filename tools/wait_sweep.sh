#!/bin/bash
# Host wait-mode sweep of the default bench workload (1080p q95, 8 frames per
# step): the runtime's polling wait against poll-then-sleep waits
# (GZ_WAIT_SPIN_US / GZ_WAIT_SLEEP_US) at several frames in flight.  One line
# per run in gpurun_out/wait_sweep.txt: spin sleep in_flight MP/s cpu_s/frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ws
out=gpurun_out/wait_sweep.txt
: > $out
run() {  # spin sleep inflight
  local tag=ws_$1_$2_$3
  GZ_WAIT_SPIN_US=$1 GZ_WAIT_SLEEP_US=$2 timeout -k 10 200 python bench.py --no-cpu-baseline \
    --steps ${STEPS:-6} --warmup 1 --frames-per-step $3 > gpurun_out/ws/$tag.json 2> gpurun_out/ws/$tag.err || return 1
  python - "$1" "$2" "$3" gpurun_out/ws/$tag.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], sys.argv[3], d["value"], d.get("host_cpu_seconds_per_frame"),
      d["verified"]["bit_exact"], flush=True)
PY
  tail -1 $out
}
for cfg in ${CONFIGS:-"0 0 8" "100 20 8" "100 20 10" "100 20 12" "200 50 10" "0 10 10" "50 5 10" "0 0 8"}; do
  run $cfg || exit 1
done
