#!/bin/bash
# The A/B driver: runs of several variants on one box, interleaved within
# each round (drift of the box hits every variant alike), each GPU step
# under its own time limit, stopping at the first failure.
#
#   bash tools/gpu_ab.sh VARIANT ...
#
# VARIANT = name[:spec[,spec...]], spec one of
#   lib=PATH    an alternative libguetzli_hip.so (GZ_LIB_PATH; tools/build_variant.sh builds one under _abv/)
#   tree=DIR    bench.py, Python binding and library of another tree (e.g. a
#               previous round's checkout copied under _ab/)
#   K=V         an environment setting (GZ_SPIN_US=0, GPU_MAX_HW_QUEUES=8 ...)
# e.g.  bash tools/gpu_ab.sh base r4:tree=_ab/r4tree
#       GZ_AB_MODE=frame GZ_AB_SIZE="3840 2160 90" bash tools/gpu_ab.sh base x:lib=_ab/x/libguetzli_hip.so
#       GZ_AB_MODE=pmc GZ_AB_PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" bash tools/gpu_ab.sh base x:GZ_BD_LDS=1
#
# GZ_AB_MODE  bench  (default) the throughput bench line (--steps GZ_AB_STEPS,
#                    default 4, no side legs): MP/s, ms/step, host CPU per
#                    frame, bit-exact frames, GZ_AB_REGIONS of the isolated
#                    frame's per-region GPU ms, its host back-end seconds
#             frame  one frame of GZ_AB_SIZE ("W H Q", default 1920 1080 95):
#                    its per-region ms and the blur+mask pass fraction
#             prof   a rocprofv3 kernel trace of the bench line, the top kernels
#             pmc    one rocprofv3 --pmc pass of GZ_AB_PMC over a single 1080p frame
#                    (<= 8 SQ / 4 TCC counters: one pass, no traces beside it)
# GZ_AB_RUNS rounds (default 2; prof and pmc: 1).  GZ_AB_ARGS: more bench.py
# arguments.  Output: gpurun_out/${GZ_AB_OUT:-ab}/<name>_<round>.{json,err}
# and one summary line per run on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export TMPDIR=/tmp
O=$ROOT/gpurun_out/${GZ_AB_OUT:-ab}
mkdir -p "$O"
MODE=${GZ_AB_MODE:-bench}
SIDE="--no-cpu-baseline --no-large-frame --no-uhd-frame"
case $MODE in
  bench) ARGS="--steps ${GZ_AB_STEPS:-4} --warmup 1 $SIDE"; RUNS=${GZ_AB_RUNS:-2} ;;
  frame) read -r W H Q <<< "${GZ_AB_SIZE:-1920 1080 95}"
         ARGS="--steps 1 --warmup 1 --frames-per-step 1 --in-flight 1 --width $W --height $H --quality $Q $SIDE"
         RUNS=${GZ_AB_RUNS:-2} ;;
  prof)  ARGS="--steps ${GZ_AB_STEPS:-4} --warmup 1 $SIDE"; RUNS=${GZ_AB_RUNS:-1} ;;
  pmc)   ARGS="--steps 1 --warmup 0 --frames-per-step 1 --width 1920 --height 1080 --quality 95 $SIDE"
         RUNS=${GZ_AB_RUNS:-1} ;;
  *) echo "unknown GZ_AB_MODE $MODE"; exit 2 ;;
esac
ARGS="$ARGS ${GZ_AB_ARGS:-}"

summary() {  # $1 json, $2 name
  python3 - "$1" "$2" "$MODE" "${GZ_AB_REGIONS:-block_diff edge_mask opsin_mhic order_select bulk_apply}" <<'PY'
import json, sys
path, name, mode, regions = sys.argv[1:5]
d = json.loads(open(path).read().strip().splitlines()[-1])
g = d.get("gpu_regions_ms_per_frame", {})
sf = d.get("single_frame", {})
if mode == "frame":
    b = d.get("blur_mask_pass", {})
    print(name, "frame_gpu_ms", d.get("gpu_ms_per_frame_isolated"), "blur_mask_frac", b.get("frac"),
          {k: g.get(k) for k in regions.split()}, "bit_exact", d["verified"]["bit_exact"])
else:
    print(name, d["value"], d["ms_per_step"], d.get("host_cpu_seconds_per_frame"), d["verified"]["bit_exact"],
          {k: g.get(k) for k in regions.split()},
          sf.get("host_breakdown_seconds", {}).get("seconds_backend"))
PY
}
top_kernels() {  # $1 kernel_stats.csv
  python3 - "$1" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("  %-40s calls %6s avg %8.1f us  %5.1f%%" % (r["Name"].split("(")[0][-40:], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
}

for r in $(seq "$RUNS"); do
  for v in "$@"; do
    name=${v%%:*}
    specs=""
    [ "$v" != "$name" ] && specs=${v#*:}
    dir=$ROOT
    envs=()
    IFS=',' read -ra parts <<< "$specs"
    for p in "${parts[@]}"; do
      case $p in
        lib=*) envs+=("GZ_LIB_PATH=$ROOT/${p#lib=}") ;;
        tree=*) dir=$ROOT/${p#tree=} ;;
        ?*=*) envs+=("$p") ;;
      esac
    done
    f=$O/${name}_$r
    cd "$dir" || exit 1
    case $MODE in
      bench|frame)
        env "${envs[@]}" timeout -k 10 300 python bench.py $ARGS > "$f.json" 2> "$f.err" || { tail "$f.err"; exit 1; }
        summary "$f.json" "$name" ;;
      prof)
        env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$f.prof" -o run --output-format csv \
          -- python bench.py $ARGS > "$f.json" 2> "$f.err" || { tail "$f.err"; exit 1; }
        echo "== $name"; summary "$f.json" "$name"; top_kernels "$f.prof/run_kernel_stats.csv" ;;
      pmc)
        env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc ${GZ_AB_PMC:?counters} -d "$f.pmc" -o run \
          --output-format csv -- python bench.py $ARGS > "$f.json" 2> "$f.err" || { tail "$f.err"; exit 1; }
        echo "== $name: $f.pmc" ;;
    esac
    cd "$ROOT"
  done
done
