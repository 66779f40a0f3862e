#!/bin/bash
# round 3 first GPU pass: full iteration + composite diag counters
set -o pipefail
bash tools/gpu_iter.sh r03a || exit 1
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/libgsplat_diag.so timeout -k 10 120 python3 tools/diag/comp_stats.py > gpurun_out/r03a/comp_stats.log 2>&1 || { tail -20 gpurun_out/r03a/comp_stats.log; exit 1; }
cat gpurun_out/r03a/comp_stats.log
