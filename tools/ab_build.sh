#!/bin/bash
# Build a library variant with extra compile definitions into lib/ab/libgsplat_NAME.so (A/B runs
# select it with GSPLAT_LIB).  Usage: bash tools/ab_build.sh NAME "-DFOO=1 -DBAR"
set -e
NAME=$1; DEFS=$2
D=$(cd "$(dirname "$0")/.." && pwd)/gaussian-splatting-web_amd
mkdir -p $D/build/ab $D/lib/ab
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-gpu-rdc -munsafe-fp-atomics -mllvm -amdgpu-atomic-optimizer-strategy=DPP $DEFS -c $D/csrc/gs_kernels.hip -o $D/build/ab/k_$NAME.o
$HIPCC -O2 -std=c++17 -fPIC -Wall -ffp-contract=off -x hip --offload-arch=gfx950 $DEFS -c $D/csrc/gs_api.cpp -o $D/build/ab/a_$NAME.o
$HIPCC --offload-arch=gfx950 -shared -fPIC -o $D/lib/ab/libgsplat_$NAME.so $D/build/ab/k_$NAME.o $D/build/ab/a_$NAME.o $D/build/gs_host.o -fopenmp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libgsplat_$NAME.so
echo built $D/lib/ab/libgsplat_$NAME.so
