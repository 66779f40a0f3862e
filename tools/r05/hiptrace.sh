#!/bin/bash
# GPU box: HIP API + kernel traces of G=8 strip frames (1080p and 50 M / 4K), list split off.
set -o pipefail
TAG=${1:-ht}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
LIST_SPLIT=0 GS=8 STRIP=4 TIMING=0 WARMUP=20 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $R/$OUT/s1080 -o run -- python3 $R/tools/strip_bench.py > $R/$OUT/s1080.log 2>&1 || { tail -30 $R/$OUT/s1080.log; exit 1; }
tail -2 $R/$OUT/s1080.log
LIST_SPLIT=0 N=50000000 W=3840 H=2160 SEED=50 GS=8 STRIP=4 TIMING=0 WARMUP=20 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/s4k -o run -- python3 $R/tools/strip_bench.py > $R/$OUT/s4k.log 2>&1 || { tail -30 $R/$OUT/s4k.log; exit 1; }
tail -2 $R/$OUT/s4k.log
ls $R/$OUT/s1080 $R/$OUT/s4k
echo done
