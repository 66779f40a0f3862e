#!/bin/bash
# GPU box: moving-camera frame times (tools/orbit_probe.py, every mode) and the kernel stats of
# staged orbit frames (rocprofv3, launches serialised by the stage events) -> gpurun_out/orb/
set -o pipefail
mkdir -p gpurun_out/orb
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/orbit_probe.py > gpurun_out/orb/probe.txt 2>&1 || { tail -20 gpurun_out/orb/probe.txt; exit 1; }
MODE=adaptive_staged timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/orb/p -o run -- python3 tools/orbit_probe.py > gpurun_out/orb/prof.log 2>&1 || { tail -20 gpurun_out/orb/prof.log; exit 1; }
cp gpurun_out/orb/p/run_kernel_stats.csv gpurun_out/orb/stats.csv
python3 tools/timeline.py gpurun_out/orb/p/run_kernel_trace.csv 700 > gpurun_out/orb/timeline.txt
rm -rf gpurun_out/orb/p
cat gpurun_out/orb/probe.txt
python3 tools/kstats.py gpurun_out/orb/stats.csv 2>/dev/null | head -30 || true
