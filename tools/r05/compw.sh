#!/bin/bash
# GPU box: wave-per-tile composite A/B. -m gpu suite with it on (default), then the bench with
# GS_COMP_W=0 (k_composite) / 1 (k_composite_w, 5 waves/SIMD) / the 4-wave build (lib/ab w4),
# REPS rounds, and a kernel-trace of each.
set -o pipefail
TAG=${1:-compw}; REPS=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
fi
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
W4=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_w4.so
run() {  # name, lib, GS_COMP_W
  GS_COMP_W=$3 GSPLAT_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_$1_$r.log 2>&1 || { tail -5 $OUT/b_$1_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_$1_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$1', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
}
for r in $(seq $REPS); do
  run old $B 0
  run w5 $B 1
  run w4 $W4 1
  run w5all $B 2
done
for v in "old $B 0" "w5 $B 1" "w4 $W4 1"; do
  set -- $v
  mkdir -p $OUT/k_$1
  GS_COMP_W=$3 GSPLAT_LIB=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k_$1 -o run -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $OUT/k_$1.log 2>&1 || { tail -5 $OUT/k_$1.log; exit 1; }
  f=$(ls $OUT/k_$1/*/run_kernel_stats.csv $OUT/k_$1/run_kernel_stats.csv 2>/dev/null | head -n 1)
  echo "== $1"; grep -i "composite" $f | cut -d, -f1-5 | head -n 6
done
echo done
