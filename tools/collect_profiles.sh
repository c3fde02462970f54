#!/bin/bash
# Copies the summaries of a tools/gpu_round.sh run (gpurun_out/, scratch)
# into profiles/ (tracked) under the round's names.
set -e
cd "$(dirname "$0")/.."
R=${GZ_ROUND:-round1}
cp gpurun_out/round_bench.json profiles/${R}_bench_default.json
for t in "prof1080 1920x1080" "prof4k 3840x2160"; do
  set -- $t
  cp gpurun_out/$1/trace/run_kernel_stats.csv profiles/${R}_kernel_stats_$2.csv
  tail -1 gpurun_out/$1/bench.json > profiles/${R}_bench_rocprof_$2.json
  cp gpurun_out/$1/traffic.json profiles/${R}_traffic_$2.json
  [ -f gpurun_out/util/pmc_util_$2.json ] && cp gpurun_out/util/pmc_util_$2.json profiles/${R}_pmc_util_$2.json
done
ls -la profiles/
