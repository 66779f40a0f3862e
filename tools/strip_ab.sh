#!/bin/bash
# GPU box: the G = 8 strip bound at 1080p and 50 M / 4K under environment variants (tools/strip_bench.py,
# TIMING=2), interleaved.  Usage: bash tools/strip_ab.sh REPS "NAME=VAL,..." ...   ("-" = none)
set -o pipefail
REPS=${1:-1}; shift
for rep in $(seq $REPS); do
  for v in "$@"; do
    env=""; [ "$v" != "-" ] && env=$(echo $v | tr ',' ' ')
    a=$(env $env GS=1,8 TIMING=2 timeout -k 10 200 python3 tools/strip_bench.py 2>&1 | grep "G=8" | cut -c1-40) || exit 1
    b=$(env $env N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=2 timeout -k 10 300 python3 tools/strip_bench.py 2>&1 | grep "G=8" | cut -c1-40) || exit 1
    echo "$v $rep | 1080p $a | 4K $b"
  done
done
