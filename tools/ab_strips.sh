#!/bin/bash
# GPU box: row-strip bounds (tools/strip_bench.py, 1080p and 50 M / 4K, G = 1 and 8), interleaved
# over variants: "cut" (the committed build), "nocut" (GS_TILE_CUT=0), or the name X of a
# library lib/ab/libgsplat_X.so (e.g. r05: the round-5 build).  Usage: bash tools/ab_strips.sh TAG REPS V...
set -o pipefail
OUT=gpurun_out/${1:-abs}; REPS=${2:-2}; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
for rep in $(seq $REPS); do
  for v in "$@"; do
    env=""
    [ $v = nocut ] && env="GS_TILE_CUT=0"
    [ $v != nocut ] && [ $v != cut ] && env="GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so"
    env $env GS=1,8 TIMING=2 timeout -k 10 120 python3 tools/strip_bench.py > $OUT/s1080_${v}_$rep.log 2>&1 || exit 1
    env $env N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=2 WARMUP=10 timeout -k 10 300 python3 tools/strip_bench.py > $OUT/s4k_${v}_$rep.log 2>&1 || exit 1
    echo "$v $rep 1080p: $(grep -o 'G=[18] worst [0-9.]* ms' $OUT/s1080_${v}_$rep.log | tr '\n' ' ') 4K: $(grep -o 'G=[18] worst [0-9.]* ms' $OUT/s4k_${v}_$rep.log | tr '\n' ' ')"
  done
done
