#!/bin/bash
# GPU box: the GPU test suite against one lib/ab variant, then tools/ab_run.sh over the given variants.
# Usage: bash tools/ab_tests.sh VARIANT "base v1 v2"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests_$1.log 2>&1 || { tail -30 gpurun_out/ab/tests_$1.log; exit 1; }
tail -1 gpurun_out/ab/tests_$1.log
bash tools/ab_run.sh "$2"
