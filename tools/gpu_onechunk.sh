#!/bin/bash
# GPU box: kernel traces of one-chunk frames (the non-saturated path).  Usage: bash tools/gpu_onechunk.sh TAG
set -o pipefail
TAG=${1:-oc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for w in sparse cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w -o run -- python3 tools/diag/onechunk_probe.py $w 5 > $OUT/$w.log 2>&1 || { tail -30 $OUT/$w.log; exit 1; }
  grep "one-chunk" $OUT/$w.log
  python3 tools/kstats.py $OUT/$w/run_kernel_stats.csv 6 || true
done
echo done
