cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sf
for r in 1 2 3; do
for lib in default _variants/base/libguetzli_hip.so; do
  if [ "$lib" = default ]; then unset GZ_LIB_PATH; else export GZ_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-large-frame --no-uhd-frame > gpurun_out/sf/o.json 2> gpurun_out/sf/o.err || { tail gpurun_out/sf/o.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/sf/o.json').read().strip().splitlines()[-1])
h = d['single_frame']['host_breakdown_seconds']
print('${lib:0:12}', d['value'], d['single_frame']['seconds'], h['seconds_backend'], h.get('backend_order_s'), h.get('backend_changes_s'))"
done
done
