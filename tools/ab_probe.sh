#!/bin/bash
# A/B of an environment switch on the isolated per-kernel stage times:
#   GZ_AB_VAR=NAME GZ_AB_FILTER=regex bash tools/ab_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "" 1; do
  env ${GZ_AB_VAR}=$v timeout -k 10 120 python tools/stage_times.py 2>&1 | grep -E "${GZ_AB_FILTER:-compare_pass}" | sed "s/^/[${GZ_AB_VAR}=$v] /"
done
