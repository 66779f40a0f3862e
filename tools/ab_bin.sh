#!/bin/bash
# GPU box: the bench frame's stage times (bench.py --no-extra, timing=1 stages) with the per-tile
# cut off (GS_TILE_CUT=0), for the committed build and lib/ab/libgsplat_X.so variants, interleaved.
# Usage: bash tools/ab_bin.sh TAG REPS V...   (V = cur or X)
set -o pipefail
OUT=gpurun_out/${1:-abb}; REPS=${2:-2}; shift 2
mkdir -p $OUT
for rep in $(seq $REPS); do
  for v in "$@"; do
    env="GS_TILE_CUT=0"
    [ $v != cur ] && env="$env GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so"
    env $env timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extra --steps 100 > $OUT/${v}_$rep.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads(open('$OUT/${v}_$rep.log').read().strip().splitlines()[-1]); s=d['stages_ms']
print('%-20s %d fps %.2f  project %.1f bin %.1f tsort %.1f comp %.1f us' % ('$v', $rep, d['fps'], s['ms_project']*1e3, s['ms_bin']*1e3, s['ms_tile_sort']*1e3, s['ms_composite']*1e3))"
  done
done
