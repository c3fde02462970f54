#!/bin/bash
# A/B of library variants (tools/variant_build.sh): the -m gpu tests on the
# last variant named in GZ_VARIANTS, then interleaved stage times of all.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${GZ_VARIANTS:?variants}
LAST=${V##* }
GZ_LIB_PATH=_variants/$LAST/libguetzli_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
  -p no:cacheprovider --timeout 300 > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
GZ_AB_FILTER="${GZ_AB_FILTER:-frame|block_diff|jpeg|compare_pass}" bash tools/variant_ab.sh
