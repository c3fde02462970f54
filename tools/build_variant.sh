#!/bin/bash
# A library variant for tools/gpu_ab.sh: the device object rebuilt with extra
# preprocessor definitions and linked with the current host objects, into
# _abv/<name>/libguetzli_hip.so (git-ignored scratch that travels to the GPU box: delete it after the A/B).
#   bash tools/build_variant.sh NAME -DGZ_OS_WAVES=8 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s -C guetzli-cuda-opencl_amd/csrc > /dev/null
mkdir -p _abv/$name build/ab_$name
cd guetzli-cuda-opencl_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-value -I. -I../../include \
  --offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero "$@" -c kernels/gz_device.hip -o ../../build/ab_$name/gz_device.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../_abv/$name/libguetzli_hip.so \
  $(ls ../../build/csrc/host_*.o) ../../build/ab_$name/gz_device.o -pthread -lz -ldl
echo "_abv/$name/libguetzli_hip.so"
