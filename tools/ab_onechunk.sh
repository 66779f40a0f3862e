#!/bin/bash
# GPU box: one-chunk frame wall times (tools/diag/onechunk_probe.py) for the committed build and
# lib/ab/libgsplat_X.so variants or environment settings, interleaved REPS times.
# Usage: bash tools/ab_onechunk.sh TAG REPS WHICH V...   (WHICH = cfg4|sparse|bench; V = cur, X or VAR=value)
set -o pipefail
OUT=gpurun_out/${1:-abo}; REPS=${2:-2}; WHICH=${3:-cfg4}; shift 3
mkdir -p $OUT
for rep in $(seq $REPS); do
  for v in "$@"; do
    env=""
    case $v in cur) ;; *=*) env="$v" ;; *) env="GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so" ;; esac
    env $env timeout -k 10 200 python3 tools/diag/onechunk_probe.py $WHICH 10 > "$OUT/${v}_$rep.log" 2>&1 || { tail -5 "$OUT/${v}_$rep.log"; exit 1; }
    echo "$v $rep $(grep one-chunk "$OUT/${v}_$rep.log")"
  done
done
