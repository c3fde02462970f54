#!/bin/bash
# Interleaved stage times of the library variants under _variants/ (built by
# tools/variant_build.sh):  GZ_VARIANTS="A B" GZ_AB_ARGS="--width 3840 --height 2160 --quality 90"
#   GZ_AB_FILTER=regex bash tools/variant_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for v in ${GZ_VARIANTS:-A B}; do
    GZ_LIB_PATH=_variants/$v/libguetzli_hip.so timeout -k 10 120 python tools/stage_times.py ${GZ_AB_ARGS:-} \
      > gpurun_out/ab_$v.log 2>&1 || { cat gpurun_out/ab_$v.log; exit 1; }
    grep -E "${GZ_AB_FILTER:-frame}" gpurun_out/ab_$v.log | sed "s/^/[$v] /"
  done
done
