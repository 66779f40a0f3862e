#!/bin/bash
# GPU box: composite phase cycles (GS_COMP_PHASE diag build) at 1080p full / strip and 4K strip.
set -o pipefail
TAG=${1:-ph}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
D=gaussian-splatting-web_amd/lib/libgsplat_diag.so
PHASE=1 GSPLAT_LIB=$D timeout -k 10 150 python -u tools/diag/comp_stats.py > $OUT/full.txt 2>&1 || { tail -20 $OUT/full.txt; exit 1; }
PHASE=1 GSPLAT_LIB=$D G=8 STRIP=4 timeout -k 10 150 python -u tools/diag/comp_stats.py > $OUT/strip8.txt 2>&1 || { tail -20 $OUT/strip8.txt; exit 1; }
PHASE=1 GSPLAT_LIB=$D N=50000000 W=3840 H=2160 SEED=50 G=8 STRIP=4 timeout -k 10 300 python -u tools/diag/comp_stats.py > $OUT/strip8_4k.txt 2>&1 || { tail -20 $OUT/strip8_4k.txt; exit 1; }
grep -h "phase\|kernel span\|composite" $OUT/*.txt
echo done
