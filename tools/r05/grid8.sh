#!/bin/bash
# GPU box: the k_cull paths a 2048-workgroup grid only reaches above ~266 M Gaussians (a workgroup's
# partition list past its 128 LDS entries, its unit buffer flushed mid-loop), forced with an
# 8-workgroup cull grid (build first: bash tools/ab_build.sh grid8 "-DGS_CULL_GRID=8"), against the
# parity, sequence and config tests.
set -o pipefail
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_grid8.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_bench_sequences.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 300 --timeout-method thread
