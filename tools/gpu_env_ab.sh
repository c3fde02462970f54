#!/bin/bash
# Interleaved bench lines for environment settings of one build:
#   bash tools/gpu_env_ab.sh "base:" "r16:GZ_OPSIN_ROWS=16" ...
# (GZ_AB_RUNS rounds; per line: name, MP/s, ms/step, host CPU s/frame, bit-exact frames,
# the isolated frame's GPU regions, its wall seconds and host back-end seconds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/envab
mkdir -p $O
BENCH="bench.py --steps ${GZ_AB_STEPS:-4} --warmup 1 --no-cpu-baseline --no-large-frame --no-uhd-frame"
for r in $(seq ${GZ_AB_RUNS:-2}); do
  for cfg in "$@"; do
    name=${cfg%%:*}
    envs=${cfg#*:}
    f=$O/${name}_$r
    env $envs timeout -k 10 200 python $BENCH > $f.json 2> $f.err || { tail $f.err; exit 1; }
    python -c "
import json
d = json.loads(open('$f.json').read().strip().splitlines()[-1])
g = d.get('gpu_regions_ms_per_frame', {})
sf = d.get('single_frame', {})
print('$name', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['verified']['bit_exact'],
      {k: g.get(k) for k in '${GZ_AB_REGIONS:-opsin_mhic edge_mask blur_h blur_v}'.split()},
      sf.get('seconds'), sf.get('host_breakdown_seconds', {}).get('seconds_backend'))"
  done
done
