#!/bin/bash
# GPU box: bench.py (with its orbit / cold / sparse lines unless EXTRA=0) for the committed build
# and lib/ab/libgsplat_X.so variants, interleaved REPS times.
# Usage: bash tools/ab_libs.sh TAG REPS V...   (V = cur or X)
set -o pipefail
OUT=gpurun_out/${1:-abl}; REPS=${2:-2}; shift 2
mkdir -p $OUT
extra=""; [ "${EXTRA:-1}" = 0 ] && extra="--no-extra"
for rep in $(seq $REPS); do
  for v in "$@"; do
    env=""
    [ $v != cur ] && env="GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so"
    env $env timeout -k 10 200 python3 bench.py --no-cpu-baseline $extra --steps 200 > $OUT/${v}_$rep.log 2>&1 || { tail -5 $OUT/${v}_$rep.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/${v}_$rep.log').read().strip().splitlines()[-1]); s=d['stages_ms']
x=lambda k: d[k]['fps'] if k in d else 0
print('%-10s %d  %.1f fps  orbit %.1f cold %.1f sparse %.1f | project %.1f bin %.1f tsort %.1f comp %.1f us' % ('$v', $rep, d['fps'], x('orbit'), x('cold'), x('sparse'), s['ms_project']*1e3, s['ms_bin']*1e3, s['ms_tile_sort']*1e3, s['ms_composite']*1e3))"
  done
done
