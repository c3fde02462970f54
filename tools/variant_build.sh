#!/bin/bash
# Builds the current tree's library as variant NAME under _variants/NAME/
# (A/B timing on the GPU box with GZ_LIB_PATH=_variants/NAME/libguetzli_hip.so).
set -e
cd "$(dirname "$0")/.."
N=${1:?variant name}
mkdir -p _variants/$N
make -C guetzli-cuda-opencl_amd/csrc -j8 OUT_DIR=$PWD/_variants/$N BUILD=/tmp/gz_variant_$N >/dev/null
ls -la _variants/$N/libguetzli_hip.so
