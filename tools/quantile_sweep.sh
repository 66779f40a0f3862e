#!/bin/bash
# GPU box: the bench line (static and orbit fps) at several saturation quantiles of the chunk
# controller (GS_SAT_QUANTILE).  Usage: bash tools/quantile_sweep.sh OUTDIR "0.9 0.98 1" [bench args]
set -o pipefail
OUT=$1; QS=$2; shift 2
mkdir -p $OUT
for q in $QS; do
  GS_SAT_QUANTILE=$q timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $OUT/q$q.log 2>&1 || { tail -20 $OUT/q$q.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/q$q.log').read().strip().splitlines()[-1]); print('q=$q fps %.1f orbit %.1f chunk_frac %.3f unsat %d k1 %d' % (d['fps'], d['orbit']['fps'], d['chunk_fraction'], d['tiles_unsaturated'], d['orbit']['k_chunk1_last']))"
done
