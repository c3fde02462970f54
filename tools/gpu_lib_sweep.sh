#!/bin/bash
# Throughput and host CPU of library variants (_variants/<name>) x frames in
# flight, interleaved, on the GPU box (GZ_VARIANTS, GZ_INFLIGHT, GZ_ROUNDS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/libs
mkdir -p $O
ARGS="--no-cpu-baseline --no-large-frame --steps ${GZ_STEPS:-4} --warmup 1"
for r in $(seq ${GZ_ROUNDS:-1}); do
for n in ${GZ_INFLIGHT:-8 12}; do
  for v in ${GZ_VARIANTS:-C D}; do
    f=$O/${v}_n${n}_r$r
    GZ_LIB_PATH=_variants/$v/libguetzli_hip.so timeout -k 10 300 python bench.py $ARGS --in-flight $n > $f.json 2> $f.err \
      || { tail $f.err; exit 1; }
    python -c "import json; d=json.load(open('$f.json')); print('$v inflight $n', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['host_cpu_user_system_seconds_per_frame'], d['host_cores_busy_per_gpu'], d['verified']['bit_exact'])"
  done
done
done
