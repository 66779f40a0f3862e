#!/bin/bash
# GPU box: moving-camera frames seeded from their own view (GS_SEED_MOVING=1) against the
# history threshold: bench lines at 1080p and 50 M / 4K (orbit, cold).
set -o pipefail
TAG=${1:-sm}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
for v in 0 1; do
  GS_SEED_MOVING=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('seedmov%s 1080p fps %.1f orbit %.1f cold %.1f sparse %.1f' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), d['orbit'])"
done
done
for v in 0 1; do
  GS_SEED_MOVING=$v timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --steps 30 --warmup 3 > $OUT/c4_${v}.log 2>&1 || { tail -5 $OUT/c4_${v}.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_${v}.log').read().strip().splitlines()[-1]); print('seedmov%s 4k fps %.1f orbit %.1f cold %.1f' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps']), d['orbit'])"
done
echo done
