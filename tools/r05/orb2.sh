#!/bin/bash
# GPU box: bench A/B (working tree vs lib/ab variants; orbit fps in each line) and the orbit
# frames' kernel statistics for the working tree.
set -o pipefail
TAG=${1:-orb}; VARS=${2:-prev}; REPS=${3:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
lib() { if [ "$1" = base ]; then echo $B; else echo $PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
if [ -n "$TESTS" ]; then
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for r in $(seq $REPS); do
for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3))"
done
done
(cd /tmp && MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k.log 2>&1) || { tail -20 $OUT/k.log; exit 1; }
python3 tools/kstats.py $OUT/k/run_kernel_stats.csv 65 | head -24
echo done
