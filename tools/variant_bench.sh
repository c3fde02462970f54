#!/bin/bash
# Interleaved default-bench throughput of the library variants under
# _variants/ (tools/variant_build.sh):  GZ_VARIANTS="A B" GZ_ROUNDS=3 bash tools/variant_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in $(seq 1 ${GZ_ROUNDS:-3}); do
  for v in ${GZ_VARIANTS:-A B}; do
    GZ_LIB_PATH=_variants/$v/libguetzli_hip.so timeout -k 10 300 python bench.py --steps ${GZ_STEPS:-4} --warmup 2 \
      --no-cpu-baseline --no-large-frame > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.err || { tail -5 gpurun_out/vb_$v.err; exit 1; }
    python - "$v" <<'PY'
import json, sys
for l in open("gpurun_out/vb_%s.json" % sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("[%s] %.1f MP/s  cpu %.4f s/frame  cores %.2f  verified %s" % (
            sys.argv[1], d["value"], d["host_cpu_seconds_per_frame"], d["host_cores_busy_per_gpu"],
            d["verified"]["bit_exact"]))
PY
  done
done
