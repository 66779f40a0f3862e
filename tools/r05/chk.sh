#!/bin/bash
set -o pipefail
OUT=gpurun_out/chk; mkdir -p $OUT
export TMPDIR=/tmp
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_chk.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "lower_sh" --timeout 100 --timeout-method thread > $OUT/t.log 2>&1; rc=$?
grep -E "DENSE|PASS|FAIL|passed|failed|Error" $OUT/t.log | head -30
echo rc=$rc
