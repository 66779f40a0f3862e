#!/bin/bash
# GPU box: list-split tests, then the strip bound with and without the split (1080p).
set -o pipefail
TAG=${1:-s3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -3
TIMING=2 LIST_SPLIT=1 timeout -k 10 200 python -u tools/strip_bench.py > $OUT/strips_split.txt 2>&1 || { tail -20 $OUT/strips_split.txt; exit 1; }
cat $OUT/strips_split.txt
TIMING=2 LIST_SPLIT=0 timeout -k 10 200 python -u tools/strip_bench.py > $OUT/strips_exact.txt 2>&1 || { tail -20 $OUT/strips_exact.txt; exit 1; }
cat $OUT/strips_exact.txt
echo done
