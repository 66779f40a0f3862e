#!/bin/bash
# GPU box: everything profiles/<TAG>_* holds for a round: the rocprof kernel stats and PMC passes
# of the bench command (tools/collect_profiles.sh), the bench line itself, the strip bound for
# G = 1, 2, 4, 8 and a traced G = 8 strip timeline, and the 50 M / 4K bench line with its kernel stats.
# Usage: bash tools/round_profiles.sh TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/collect_profiles.sh $TAG || exit 1
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
GS=1,2,4,8 TIMING=2 timeout -k 10 200 python3 tools/strip_bench.py > $OUT/strips.log 2>&1 || { tail -20 $OUT/strips.log; exit 1; }
GS=8 STRIP=1 TIMING=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 tools/strip_bench.py > $OUT/tl.log 2>&1 || { tail -20 $OUT/tl.log; exit 1; }
python3 tools/timeline.py $OUT/tl/run_kernel_trace.csv 400 > $OUT/strip8_timeline.txt
timeout -k 10 400 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_cfg4.log 2>&1 || { tail -20 $OUT/bench_cfg4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 1; }
N=50000000 W=3840 H=2160 SEED=50 GS=1 TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c4s -o run -- python3 tools/strip_bench.py > $OUT/c4s.log 2>&1 || { tail -20 $OUT/c4s.log; exit 1; }
echo round profiles done
