#!/bin/bash
# GPU box: the GPU test suite (optionally -k), then bench lines of the default library and lib/ab
# variants, then the composite diag counters.  Usage: bash tools/gpu_ab_tests.sh "base old" [k-expr]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ -n "$2" ]; then KARG=(-k "$2"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/ab/tests.log 2>&1 || { tail -40 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
bash tools/ab_run.sh "$1" || exit 1
GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/libgsplat_diag.so timeout -k 10 120 python3 tools/diag/comp_stats.py 2>&1 | head -8
