#!/bin/bash
# GPU box: selected tests (pytest -k), the default bench line and the 50 M / 4K line.
# Usage: bash tools/gpu_quick.sh TAG "pytest -k expr"
set -o pipefail
TAG=${1:-q}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('fps',d['fps'],'orbit',d['orbit']['fps'],'cold',d.get('cold'))"
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench4.log 2>&1 || { tail -30 $OUT/bench4.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench4.log').read().strip().splitlines()[-1]);print('cfg4 fps',d['fps'],'orbit',d['orbit']['fps'],'cold',d.get('cold'))"
echo done
