# -m gpu tests, then the host pool profile of concurrent encodes and two bench runs
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
GZ_POOL_PROFILE=1 timeout -k 10 300 python tools/conc_detail.py > gpurun_out/cd.json 2> gpurun_out/cd.err; grep "pool site" gpurun_out/cd.err; grep -E "cpu|ms_per" gpurun_out/cd.json
for m in 1 2; do timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err && python -c "import json;d=json.load(open('gpurun_out/b.json'));print('bench',d['value'],d['ms_per_step'],d['host_cpu_seconds_per_frame'],d['verified']['bit_exact'])"; done
