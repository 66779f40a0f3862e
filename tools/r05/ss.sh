#!/bin/bash
# GPU box: frame-set streams (GS_SET_STREAMS builds lib/ab/libgsplat_ss1/ss2) against the default
# (one stream per frame set): bench and the 1080p / 4K G=8 strip bounds, REPS rounds.
set -o pipefail
TAG=${1:-ss}; REPS=${2:-2}; VARS=${3:-"ss1 ss2"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
lib() { if [ "$1" = base ]; then echo $R/gaussian-splatting-web_amd/lib/libgsplat.so; else echo $R/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
for r in $(seq $REPS); do
for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-5s fps %.1f orbit %.1f cold %.1f sparse %.1f' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  GSPLAT_LIB=$(lib $v) GS=1,8 TIMING=0 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | sed -e "s/^/$v 1080p /" | grep -v "^$" | cut -c1-60
done
done
for r in $(seq $REPS); do for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=0 WARMUP=10 timeout -k 10 400 python -u tools/strip_bench.py 2>&1 | sed -e "s/^/$v 4k /" | grep -v "^$" | cut -c1-60
done; done
echo done
