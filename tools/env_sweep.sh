#!/bin/bash
# Stage-time sweep of one environment knob:
#   GZ_SW_VAR=NAME GZ_SW_VALUES="a b c" GZ_SW_FILTER=regex [GZ_SW_ARGS="--width 3840 --height 2160"] bash tools/env_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in $GZ_SW_VALUES; do
  env ${GZ_SW_VAR}=$v timeout -k 10 120 python tools/stage_times.py ${GZ_SW_ARGS:-} 2>&1 | grep -E "${GZ_SW_FILTER:-compare_pass}" | sed "s/^/[${GZ_SW_VAR}=$v] /"
done
