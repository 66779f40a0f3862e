#!/bin/bash
# Build the last commit's library into lib/ab/libgsplat_prev.so (A/B against the working tree).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/gaussian-splatting-web_amd/csrc $T/include
for f in gs_kernels.hip gs_api.cpp gs_device.h gs_host.cpp; do git -C $R show HEAD:gaussian-splatting-web_amd/csrc/$f > $T/gaussian-splatting-web_amd/csrc/$f; done
git -C $R show HEAD:include/gsplat.h > $T/include/gsplat.h
H=/opt/rocm/bin/hipcc; D=$T/gaussian-splatting-web_amd
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-gpu-rdc -munsafe-fp-atomics -mllvm -amdgpu-atomic-optimizer-strategy=DPP -c $D/csrc/gs_kernels.hip -o $T/k.o
$H -O2 -std=c++17 -fPIC -Wall -ffp-contract=off -x hip --offload-arch=gfx950 -c $D/csrc/gs_api.cpp -o $T/a.o
g++ -O2 -std=c++17 -fPIC -Wall -ffp-contract=off -fopenmp -c $D/csrc/gs_host.cpp -o $T/h.o
mkdir -p $R/gaussian-splatting-web_amd/lib/ab
$H --offload-arch=gfx950 -shared -fPIC -o $R/gaussian-splatting-web_amd/lib/ab/libgsplat_prev.so $T/k.o $T/a.o $T/h.o -fopenmp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libgsplat_prev.so
rm -rf $T
echo built libgsplat_prev.so
