#!/bin/bash
# A/B of an environment switch on the isolated per-kernel stage times
# (unset vs =1):  GZ_AB_VAR=NAME GZ_AB_FILTER=regex bash tools/ab_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
env -u ${GZ_AB_VAR} timeout -k 10 120 python tools/stage_times.py ${GZ_AB_ARGS:-} 2>&1 | grep -E "${GZ_AB_FILTER:-compare_pass}" | sed "s/^/[${GZ_AB_VAR} unset] /"
env ${GZ_AB_VAR}=1 timeout -k 10 120 python tools/stage_times.py ${GZ_AB_ARGS:-} 2>&1 | grep -E "${GZ_AB_FILTER:-compare_pass}" | sed "s/^/[${GZ_AB_VAR}=1] /"
