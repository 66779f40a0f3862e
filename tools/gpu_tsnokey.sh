#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-nk}
mkdir -p $OUT
export TMPDIR=/tmp
for e in 0 1; do
  GS_DIAG_TS_NOKEY=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c$e -o run -- python3 tools/diag/onechunk_probe.py cfg4 5 > $OUT/c$e.log 2>&1 || { tail -30 $OUT/c$e.log; exit 1; }
  echo "NOKEY=$e"; grep "one-chunk" $OUT/c$e.log; python3 tools/kstats.py $OUT/c$e/run_kernel_stats.csv 6 | grep tile_sort
  GS_DIAG_TS_NOKEY=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b$e -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra > $OUT/b$e.log 2>&1 || { tail -30 $OUT/b$e.log; exit 1; }
  python3 tools/kstats.py $OUT/b$e/run_kernel_stats.csv | grep tile_sort
done
