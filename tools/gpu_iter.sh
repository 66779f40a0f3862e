#!/bin/bash
# GPU-box iteration: parity suite, bench line, strip timings, kernel-trace summary of a short bench.
# Usage (via gpurun, from the repo root):  bash tools/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-it}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread "${KARG[@]}" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('fps',d['fps'],'ms',d['ms_per_step'],d['stages_ms'])"
GS=1,8 TIMING=2 timeout -k 10 200 python3 tools/strip_bench.py > $OUT/strips.log 2>&1 || { tail -30 $OUT/strips.log; exit 1; }
cat $OUT/strips.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv || true
echo done
