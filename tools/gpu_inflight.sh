cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/inf
for r in 1 2; do
for n in 10 12 14; do
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-large-frame --no-uhd-frame --in-flight $n > gpurun_out/inf/n${n}_$r.json 2> gpurun_out/inf/n${n}_$r.err || { tail gpurun_out/inf/n${n}_$r.err; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/inf/n${n}_$r.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d['host_cpu_seconds_per_frame'], d['verified']['bit_exact'])"
done
done
