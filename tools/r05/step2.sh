#!/bin/bash
# GPU box: sort-guard + group tests, the 50 M / 4K strip bound, one-chunk 4K trace.
set -o pipefail
TAG=${1:-s2}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_group.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
N=50000000 W=3840 H=2160 SEED=50 TIMING=2 WARMUP=10 timeout -k 10 400 python -u tools/strip_bench.py > $OUT/strips_cfg4.txt 2>&1 || { tail -20 $OUT/strips_cfg4.txt; exit 1; }
cat $OUT/strips_cfg4.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/oc -o run -- python3 tools/diag/onechunk_probe.py cfg4 5 > $OUT/oc.log 2>&1 || { tail -30 $OUT/oc.log; exit 1; }
grep "one-chunk" $OUT/oc.log
python3 tools/kstats.py $OUT/oc/run_kernel_stats.csv 8 || true
echo done
