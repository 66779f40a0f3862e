#!/bin/bash
# GPU box: orbit probe at 1080p and 4K with kernel stats of staged orbit frames.
set -o pipefail
mkdir -p gpurun_out/orb4
export TMPDIR=/tmp
for c in 3 4; do
  CONFIG=$c STEPS=30 timeout -k 10 300 python3 tools/orbit_probe.py > gpurun_out/orb4/probe$c.txt 2>&1 || { tail -20 gpurun_out/orb4/probe$c.txt; exit 1; }
  cat gpurun_out/orb4/probe$c.txt
  CONFIG=$c STEPS=30 MODE=adaptive_staged timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/orb4/p$c -o run -- python3 tools/orbit_probe.py > gpurun_out/orb4/prof$c.log 2>&1 || { tail -20 gpurun_out/orb4/prof$c.log; exit 1; }
  python3 tools/kstats.py gpurun_out/orb4/p$c/run_kernel_stats.csv 35 | head -24
done
