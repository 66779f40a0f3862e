#!/bin/bash
# Kernel trace of one row strip (default: strip 1 of 8) on one GPU: per-kernel median durations.
# Usage (GPU box): bash tools/strip_prof.sh TAG [G] [STRIP]
set -o pipefail
TAG=${1:-sp}; G=${2:-8}; S=${3:-1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp GS=$G STRIP=$S
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/strip_bench.py \
    > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
grep "G=" $OUT/log
python3 tools/trace_median.py $OUT/prof/run_kernel_trace.csv
