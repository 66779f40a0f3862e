#!/bin/bash
# GPU box: kernel statistics of orbit frames with the stages serialised (timing=1: every kernel
# alone on the GPU) against the adaptive frames in flight.
set -o pipefail
TAG=${1:-ost}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
for m in adaptive_staged adaptive; do
(cd /tmp && MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/$m -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/$m.log 2>&1) || { tail -20 $OUT/$m.log; exit 1; }
echo "== $m"; grep -v "^[EWI]2026" $OUT/$m.log | tail -2
python3 tools/kstats.py $OUT/$m/run_kernel_stats.csv 65 | head -22
done
echo done
