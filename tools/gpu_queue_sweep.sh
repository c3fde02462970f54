#!/bin/bash
# Hardware queues (GPU_MAX_HW_QUEUES, <= 32) x end-of-candidate wait
# (GZ_SYNC_WAIT: hostfunc / event) x frames in flight of the default library
# on the GPU box: throughput and host CPU.  Each run is bounded; the sweep
# stops at the first run that fails or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/queues
mkdir -p $O
ARGS="--no-cpu-baseline --no-large-frame --no-uhd-frame --steps ${GZ_STEPS:-4} --warmup 1"
for r in $(seq ${GZ_ROUNDS:-1}); do
for n in ${GZ_INFLIGHT:-10}; do
  for cfg in ${GZ_CONFIGS:-4:hostfunc 8:event 4:event}; do
    q=${cfg%%:*}; w=${cfg##*:}
    f=$O/q${q}_${w}_n${n}_r$r
    GPU_MAX_HW_QUEUES=$q GZ_SYNC_WAIT=$w timeout -k 10 ${GZ_RUN_LIMIT:-150} python bench.py $ARGS --in-flight $n > $f.json 2> $f.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "queues $q wait $w inflight $n: rc=$rc"; exit $rc; fi
    python -c "import json; d=json.load(open('$f.json')); print('queues $q wait $w inflight $n', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified']['bit_exact'])"
  done
done
done
