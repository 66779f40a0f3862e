#!/bin/bash
# GPU box: bench.py (with its orbit / cold / sparse lines) under environment variants, interleaved.
# Usage: bash tools/ab_env.sh TAG REPS "NAME=VAL,NAME2=VAL2" ...   ("-" = no variables)
set -o pipefail
OUT=gpurun_out/${1:-abe}; REPS=${2:-2}; shift 2
mkdir -p $OUT
for rep in $(seq $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env=""; [ "$v" != "-" ] && env=$(echo $v | tr ',' ' ')
    env $env timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps ${STEPS:-200} ${BENCH_ARGS:-} > $OUT/v${i}_$rep.log 2>&1 || { tail -5 $OUT/v${i}_$rep.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/v${i}_$rep.log').read().strip().splitlines()[-1]); s=d['stages_ms']
print('%-36s %d  %.1f fps  orbit %.1f cold %.1f sparse %.1f | project %.1f bin %.1f tsort %.1f comp %.1f us' % ('$v', $rep, d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], s['ms_project']*1e3, s['ms_bin']*1e3, s['ms_tile_sort']*1e3, s['ms_composite']*1e3))"
  done
done
