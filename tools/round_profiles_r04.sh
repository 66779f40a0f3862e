#!/bin/bash
# GPU box: the round-4 profile set (profiles/r04_*): the standard set (tools/round_profiles.sh:
# kernel stats + PMC passes of the bench command, bench line, strip bounds, strip timeline, 50 M / 4K
# line and stats), plus one-chunk kernel stats (sparse scene, 50 M / 4K), the device-group host
# time, and orbit-frame kernel stats.  Usage: bash tools/round_profiles_r04.sh TAG
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/round_profiles.sh $TAG || exit 1
bash tools/gpu_onechunk.sh oc_$TAG > $OUT/onechunk.txt 2>&1 || { tail -20 $OUT/onechunk.txt; exit 1; }
timeout -k 10 300 python3 tools/diag/group_host_time.py > $OUT/group_host_time.txt 2>&1 || { tail -20 $OUT/group_host_time.txt; exit 1; }
echo "round $TAG profiles done"
