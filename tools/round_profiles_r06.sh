#!/bin/bash
# GPU box: the round-6 evidence beside profiles/r06_{kernel_stats,pmc,frame,bench}: the strip bound
# at 1080p and 50 M / 4K (G = 1, 2, 4, 8), the orbit's per-kernel times (1080p and 4K), the 50 M /
# 4K bench line and the one-chunk frames.  Output: gpurun_out/r06/.  Usage: bash tools/round_profiles_r06.sh
set -o pipefail
OUT=gpurun_out/r06; mkdir -p $OUT
export TMPDIR=/tmp
GS=1,2,4,8 TIMING=2 timeout -k 10 200 python3 tools/strip_bench.py > $OUT/strips.txt 2>&1 || { tail -20 $OUT/strips.txt; exit 1; }
N=50000000 W=3840 H=2160 SEED=50 GS=1,2,4,8 TIMING=2 timeout -k 10 400 python3 tools/strip_bench.py > $OUT/strips_cfg4.txt 2>&1 || { tail -20 $OUT/strips_cfg4.txt; exit 1; }
for c in 3 4; do
  CONFIG=$c MODE=adaptive STEPS=60 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/orb$c -o run -- python3 tools/orbit_probe.py > $OUT/orb$c.log 2>&1 || { tail -20 $OUT/orb$c.log; exit 1; }
  { grep adaptive $OUT/orb$c.log; python3 tools/kstats.py $OUT/orb$c/run_kernel_stats.csv; } > $OUT/orbit_cfg$c.txt
done
timeout -k 10 400 python3 bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_cfg4.log 2>&1 || { tail -20 $OUT/bench_cfg4.log; exit 1; }
tail -1 $OUT/bench_cfg4.log > $OUT/bench_cfg4.json
bash tools/gpu_onechunk.sh r06oc > $OUT/onechunk.txt 2>&1 || { tail -20 $OUT/onechunk.txt; exit 1; }
echo r06 profiles done
