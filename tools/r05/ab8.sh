#!/bin/bash
# GPU box: -m gpu suite, bench A/B (working tree vs lib/ab variants), and the G = 1/8 strip
# bounds at 1080p and 50 M / 4K with the small binning partition count on (default) and off
# (GS_BIN_SMALL=0), plus the per-strip stage times.
set -o pipefail
TAG=${1:-ab8}; VARS=${2:-prev}; REPS=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
lib() { if [ "$1" = base ]; then echo $B; else echo $PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
for r in $(seq $REPS); do
for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
done
for bs in 1500000 0; do
  GS_BIN_SMALL=$bs GS=1,8 TIMING=2 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | grep "G=" | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g;s/^/binsmall$bs 1080p /"
  GS_BIN_SMALL=$bs N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=2 WARMUP=10 timeout -k 10 400 python -u tools/strip_bench.py 2>&1 | grep "G=" | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g;s/^/binsmall$bs 4k /"
done
for v in $VARS; do
  GSPLAT_LIB=$(lib $v) GS=1,8 TIMING=2 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | grep "G=" | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g;s/^/$v 1080p /"
  GSPLAT_LIB=$(lib $v) N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=2 WARMUP=10 timeout -k 10 400 python -u tools/strip_bench.py 2>&1 | grep "G=" | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g;s/^/$v 4k /"
done
GS=8 timeout -k 10 300 python -u tools/diag/strip_stages.py 2>&1 | tee $OUT/stages1080.txt | head -3
N=50000000 W=3840 H=2160 SEED=50 GS=8 timeout -k 10 500 python -u tools/diag/strip_stages.py 2>&1 | tee $OUT/stages4k.txt | head -3
echo done
