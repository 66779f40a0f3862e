#!/bin/bash
# GPU box: optional tests (pytest -k), then tools/cold_probe.py for configs 3 and 4.
set -o pipefail
OUT=gpurun_out/${1:-probe}; K=${2:-}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for C in 3 4; do
  timeout -k 10 300 python tools/cold_probe.py $C > $OUT/cold$C.log 2>&1 || { tail -20 $OUT/cold$C.log; exit 1; }
  cat $OUT/cold$C.log
done
