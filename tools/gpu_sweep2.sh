#!/bin/bash
# Host-thread / concurrency sweep: "threads:frames" pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for tf in ${GZ_SWEEP_TF:-16:8 8:8 32:8 16:16}; do
  t=${tf%%:*}; f=${tf##*:}
  GZ_HOST_THREADS=$t timeout -k 10 300 python bench.py --steps 2 --warmup 1 --frames-per-step $f --no-cpu-baseline \
    > gpurun_out/sw2_${t}_$f.json 2> gpurun_out/sw2_${t}_$f.err || exit $?
  python - "$t" "$f" <<'PY'
import json, sys
t, f = sys.argv[1], sys.argv[2]
d = json.load(open("gpurun_out/sw2_%s_%s.json" % (t, f)))
print("threads", t, "frames", f, d["value"], d["ms_per_step"], "cpu/frame", d["host_cpu_seconds_per_frame"],
      d["concurrent_frame_breakdown_seconds"])
PY
done
