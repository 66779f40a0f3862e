#!/bin/bash
# GPU box (round 4): tests (pytest -k expr, or all with "all"), then optional diag scripts.
# Usage: bash tools/gpu_r04.sh TAG "k-expr|all|" "python tools/diag/x.py ..." ...
set -o pipefail
TAG=${1:-r4}; K=${2:-}
shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" = "all" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
elif [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 400 $cmd > $OUT/step$i.log 2>&1 || { echo "step $i failed: $cmd"; tail -40 $OUT/step$i.log; exit 1; }
  echo "== $cmd"; tail -25 $OUT/step$i.log
done
echo done
