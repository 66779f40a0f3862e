#!/bin/bash
# GPU box: rocprof kernel stats of one 50 M / 4K G = 8 strip (strip 0, 60 frames) with and without
# the per-tile cut.  Usage: bash tools/ab_strip_prof.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-asp}; mkdir -p $OUT
export TMPDIR=/tmp
for v in cut nocut; do
  env=""; [ $v = nocut ] && env="GS_TILE_CUT=0"
  env $env N=50000000 W=3840 H=2160 SEED=50 GS=8 STRIP=0 TIMING=0 WARMUP=10 FRAMES=60 timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/strip_bench.py > $OUT/$v.log 2>&1 || exit 1
  echo "== $v: $(grep -o 'G=8 worst [0-9.]* ms' $OUT/$v.log)"
  python3 tools/kstats.py $OUT/$v/run_kernel_stats.csv 14 || true
done
