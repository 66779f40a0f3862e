#!/bin/bash
# GPU box: HIP runtime environment settings against the G = 8 strip bound (1080p) and the
# strip frame's host enqueue time.  Usage: bash tools/r05/envsweep.sh TAG "VAR=v VAR2=v ..."
set -o pipefail
TAG=${1:-env}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for kv in none $2; do
  if [ "$kv" = none ]; then E=""; else E="$kv"; fi
  env $E GS=8 TIMING=2 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | grep "G=8" | cut -c1-50 | sed -e "s/^/$kv /"
done
echo done
