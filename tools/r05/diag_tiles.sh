#!/bin/bash
# GPU box: per-tile composite spans (diagnostics build) for the full bench frame and G=8 strips,
# plus the strip bound at 1080p.  Usage: bash tools/r05/diag_tiles.sh TAG
set -o pipefail
TAG=${1:-dt}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
D=gaussian-splatting-web_amd/lib/libgsplat_diag.so
GSPLAT_LIB=$D timeout -k 10 150 python -u tools/diag/comp_stats.py > $OUT/full.txt 2>&1 || { tail -20 $OUT/full.txt; exit 1; }
for s in ${STRIPS:-1 4}; do
  GSPLAT_LIB=$D G=8 STRIP=$s timeout -k 10 150 python -u tools/diag/comp_stats.py > $OUT/strip8_$s.txt 2>&1 || { tail -20 $OUT/strip8_$s.txt; exit 1; }
done
timeout -k 10 200 python -u tools/strip_bench.py > $OUT/strips.txt 2>&1 || { tail -20 $OUT/strips.txt; exit 1; }
cat $OUT/strips.txt
echo done
