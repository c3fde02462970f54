#!/bin/bash
# Host pool size x frames in flight on the GPU box (GZ_HOST_THREADS sets the
# pool's threads, caller included): throughput and host CPU (user, system).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pool
mkdir -p $O
ARGS="--no-cpu-baseline --no-large-frame --steps 4 --warmup 1"
for t in ${GZ_THREADS_LIST:-16 8 4}; do
  for n in ${GZ_INFLIGHT:-8 12}; do
    GZ_HOST_THREADS=$t timeout -k 10 300 python bench.py $ARGS --in-flight $n > $O/t${t}_n$n.json 2> $O/t${t}_n$n.err \
      || { tail $O/t${t}_n$n.err; exit 1; }
    python -c "import json; d=json.load(open('$O/t${t}_n$n.json')); print('threads $t inflight $n', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cpu_user_system_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified']['bit_exact'])"
  done
done
