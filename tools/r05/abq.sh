#!/bin/bash
# GPU box: -m gpu suite on the working tree, then bench A/B against lib/ab variants (REPS rounds;
# fps of every sequence + the bench stages) and each library's bench kernel statistics.
set -o pipefail
TAG=${1:-abq}; VARS=${2:-prev}; REPS=${3:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
lib() { if [ "$1" = base ]; then echo $B; else echo $R/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
fi
for r in $(seq $REPS); do
for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
done
for v in base $VARS; do
  (cd /tmp && GSPLAT_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 60 --warmup 5 > $R/$OUT/k_$v.log 2>&1) || { tail -20 $OUT/k_$v.log; exit 1; }
  echo "== $v"; python3 tools/kstats.py $OUT/k_$v/run_kernel_stats.csv 1 > $OUT/k_$v.txt; head -n 12 $OUT/k_$v.txt
done
echo done
