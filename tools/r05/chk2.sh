#!/bin/bash
set -o pipefail
OUT=gpurun_out/chk2; mkdir -p $OUT
export TMPDIR=/tmp
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_chk.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
grep -E "DENSE" $OUT/t.log | sort | uniq -c | head -30
tail -3 $OUT/t.log
echo rc=$rc
