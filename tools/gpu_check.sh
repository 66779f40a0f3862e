#!/bin/bash
# GPU-box check: parity suite, a bench line, and a kernel-trace profile of a short bench run.
# Usage (from the repo root, via gpurun):  bash tools/gpu_check.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -m gpu -x -q "$@" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
cat $OUT/bench.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv || true
echo done
