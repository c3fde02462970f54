#!/bin/bash
# Host-side CPU accounting of the concurrent bench on the GPU box: the pool's
# CPU seconds per ParallelFor call site (GZ_POOL_PROFILE) and the per-thread
# CPU of the timed region (GZ_THREAD_CPU), then the throughput at several
# frames-in-flight counts (GZ_INFLIGHT, default "8 10 12").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/host
mkdir -p $O
ARGS="--no-cpu-baseline --no-large-frame --steps 4 --warmup 1"
GZ_POOL_PROFILE=1 GZ_THREAD_CPU=1 timeout -k 10 300 python bench.py $ARGS > $O/prof.json 2> $O/prof.err \
  || { tail $O/prof.err; exit 1; }
python -c "import json; d=json.load(open('$O/prof.json')); print('prof', d['value'], d['host_cpu_seconds_per_frame'], d['concurrent_frame_breakdown_seconds'])"
for n in ${GZ_INFLIGHT:-8 10 12}; do
  timeout -k 10 300 python bench.py $ARGS --in-flight $n > $O/if_$n.json 2> $O/if_$n.err || { tail $O/if_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/if_$n.json')); print('inflight $n', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified']['bit_exact'])"
done
