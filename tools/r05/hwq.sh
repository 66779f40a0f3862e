#!/bin/bash
# GPU box: bench and the 1080p G=8 strip bound under GPU_MAX_HW_QUEUES = 4 (the box default), 5, 6, 8
# (how the context's streams -- the caller's, three frame-set streams, a copy stream -- map onto
# hardware queues), REPS rounds.
set -o pipefail
TAG=${1:-hwq}; REPS=${2:-2}; QS=${3:-"4 5 6 8"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq $REPS); do
for q in $QS; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${q}_$r.log 2>&1 || { tail -5 $OUT/b_${q}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${q}_$r.log').read().strip().splitlines()[-1]); print('q%-3s fps %.1f orbit %.1f cold %.1f sparse %.1f' % ('$q', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  GPU_MAX_HW_QUEUES=$q GS=1,8 TIMING=0 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | sed -e "s/^/q$q 1080p /" | grep -v "^$" | cut -c1-60
done
done
echo done
