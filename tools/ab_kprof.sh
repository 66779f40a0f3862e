#!/bin/bash
# GPU box: rocprof kernel durations (median / min per kernel) of the bench command for the
# committed build and lib/ab/libgsplat_X.so variants (GS_TILE_CUT=0 unless CUT=1).
# Usage: bash tools/ab_kprof.sh TAG V...   (V = cur or X)
set -o pipefail
OUT=gpurun_out/${1:-akp}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  env="GS_TILE_CUT=${CUT:-0}"
  [ $v != cur ] && env="$env GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so"
  env $env timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-extra > $OUT/$v.log 2>&1 || exit 1
  echo "== $v"
  python3 tools/trace_median.py $OUT/$v/run_kernel_trace.csv 2>/dev/null | head -14 || true
done
