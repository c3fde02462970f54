#!/bin/bash
# A/B of library builds on the north_star figure: one 4K (configs[2]) frame
# per build, its blur+mask pass fraction of HBM peak and the per-kernel event
# times, the builds interleaved over two rounds.
#   bash tools/gpu_ab4k.sh default _variants/x/libguetzli_hip.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab4k
mkdir -p $O
for r in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    if [ "$lib" = default ]; then unset GZ_LIB_PATH; else export GZ_LIB_PATH=$PWD/$lib; fi
    f=$O/${i}_$r
    timeout -k 10 200 python bench.py --steps 1 --warmup 1 --frames-per-step 1 --in-flight 1 --width 3840 \
      --height 2160 --quality 90 --no-cpu-baseline --no-large-frame --no-uhd-frame > $f.json 2> $f.err ||
      { tail $f.err; exit 1; }
    python -c "
import json
d = json.loads(open('$f.json').read().strip().splitlines()[-1])
b = d['blur_mask_pass']
print('$i', '$lib'[-30:], 'frac', b['frac'], 'ms', b['ms'], b['stage_ms'], 'verified', d['verified']['bit_exact'])"
  done
done
