#!/bin/bash
# GPU box: -m gpu suite on the working tree, then bench lines alternating between the working tree
# (base) and lib/ab variants, same box.  Usage: bash tools/r05/ab2.sh TAG "prev b4" [reps]
set -o pipefail
TAG=${1:-ab2}; VARS=${2:-prev}; REPS=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
for r in $(seq $REPS); do
for v in base $VARS; do
  if [ "$v" = base ]; then L=$B; else L=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so; fi
  GSPLAT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 $BENCH_ARGS > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
done
echo done
