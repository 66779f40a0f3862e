#!/bin/bash
# GPU box: cold-path A/B (GS_SEED=0: a cold frame is one chunk; default: seeded), 6.1 M/1080p and 50 M/4K.
set -o pipefail
TAG=${1:-cold}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for S in 0 1; do
  GS_SEED=$S timeout -k 10 200 python bench.py --steps 60 --warmup 10 --no-cpu-baseline > $OUT/bench_s$S.log 2>&1 || { tail -30 $OUT/bench_s$S.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_s$S.log').read().strip().splitlines()[-1]);print('seed $S fps',d['fps'],'orbit',d['orbit']['fps'],'cold',d.get('cold'))"
done
for S in 0 1; do
  GS_SEED=$S timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench4_s$S.log 2>&1 || { tail -30 $OUT/bench4_s$S.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench4_s$S.log').read().strip().splitlines()[-1]);print('cfg4 seed $S fps',d['fps'],'orbit',d['orbit']['fps'],'cold',d.get('cold'))"
done
echo done
