#!/bin/bash
# configs[4] check on one GPU box: the single engine vs the strip
# split (world 1, and 4 ranks sharing device 0 over gloo), warm, 8192^2 q84.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/strips_${GZ_TAG:-r5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/strip_bench.py --warmup 1 --check > $O/w1.json 2> $O/w1.err || { tail -20 $O/w1.err; exit 1; }
head -c 600 $O/w1.json; echo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29611 tools/strip_bench.py --warmup 1 --backend gloo --one-device > $O/w4.json 2> $O/w4.err || { tail -30 $O/w4.err; exit 1; }
head -c 900 $O/w4.json; echo
