#!/bin/bash
# GPU box: orbit frames (bench scene) with the list split off / on: stage times and kernel traces.
set -o pipefail
TAG=${1:-ob}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
for ls in 0 1; do
  LIST_SPLIT=$ls timeout -k 10 200 python -u tools/orbit_probe.py > $OUT/probe_ls$ls.txt 2>&1 || { tail -20 $OUT/probe_ls$ls.txt; exit 1; }
  cat $OUT/probe_ls$ls.txt
  (cd /tmp && LIST_SPLIT=$ls MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k$ls -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k$ls.log 2>&1) || { tail -20 $OUT/k$ls.log; exit 1; }
  python3 tools/kstats.py $OUT/k$ls/run_kernel_stats.csv 65 | head -24
done
echo done
