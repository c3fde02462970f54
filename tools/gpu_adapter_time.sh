#!/bin/bash
# Wall time of the drop-in adapters on bees q95 (oracle/_ref/adapter_e2e:
# the reference's own Processor on HipButteraugliComparator, and ProcessHip),
# for the in-tree library and, given as arguments, alternative builds
# (loaded through LD_LIBRARY_PATH, which the binary's RUNPATH yields to).
#   bash tools/gpu_adapter_time.sh [_variants/x ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/adt
mkdir -p $O
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/$lib; fi
    for m in comparator process; do
      t0=$(date +%s%N)
      timeout -k 10 120 oracle/_ref/adapter_e2e $m tests/golden/bees.rgb 444 258 95 $O/$m.jpg > $O/$m.out 2>&1 ||
        { cat $O/$m.out; exit 1; }
      t1=$(date +%s%N)
      echo "$lib $m $(( (t1 - t0) / 1000000 )) ms $(cat $O/$m.out) $(sha256sum < $O/$m.jpg | cut -c1-16)"
    done
  done
done
