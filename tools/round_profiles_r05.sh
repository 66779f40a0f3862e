#!/bin/bash
# GPU box: the round-5 profile set (profiles/r05_*): the standard set (tools/round_profiles.sh:
# kernel stats + PMC passes of the bench command, bench line, 1080p strip bounds G = 1, 2, 4, 8,
# a traced G = 8 strip timeline, the 50 M / 4K line and its stats), the 50 M / 4K strip bounds
# G = 1, 2, 4, 8 (strip_bench), one-chunk kernel stats (sparse scene, 50 M / 4K), the device-group
# host time, and orbit-frame kernel stats (frames in flight and stages serialised).
# Usage: bash tools/round_profiles_r05.sh TAG
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/round_profiles.sh $TAG || exit 1
N=50000000 W=3840 H=2160 SEED=50 GS=1,2,4,8 TIMING=2 WARMUP=10 timeout -k 10 400 python3 tools/strip_bench.py > $OUT/strips_cfg4.log 2>&1 || { tail -20 $OUT/strips_cfg4.log; exit 1; }
bash tools/gpu_onechunk.sh oc_$TAG > $OUT/onechunk.txt 2>&1 || { tail -20 $OUT/onechunk.txt; exit 1; }
timeout -k 10 300 python3 tools/diag/group_host_time.py > $OUT/group_host_time.txt 2>&1 || { tail -20 $OUT/group_host_time.txt; exit 1; }
bash tools/r05/orbstaged.sh orbit_$TAG > $OUT/orbit.txt 2>&1 || { tail -20 $OUT/orbit.txt; exit 1; }
echo "round $TAG profiles done"
