#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel of one library variant (GZ_LIB_PATH) over
# the Compare loop: GZ_PMC_TAG=name GZ_LIB_PATH=... bash tools/gpu_pmc_variant.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${GZ_PMC_TAG:-pmcv}
rm -rf "$OUT"; mkdir -p "$OUT"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr -d "$OUT/pmc_$ctr" -o run --output-format csv \
    -- python tools/compare_loop.py --width ${GZ_PROF_W:-3840} --height ${GZ_PROF_H:-2160} --compares 3 \
    > "$OUT/pmc_$ctr.json" 2> "$OUT/pmc_$ctr.err" || exit $?
done
python tools/traffic_summary.py "$OUT" > "$OUT/traffic.json"
python - "$OUT/traffic.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if any(t in k for t in ("vstream", "h4", "blur_stream", "mask_stream", "opsin_mhic")):
        print("%-40s %8.1f MB" % (k[:40], v["traffic_bytes"] / 1e6))
PY
