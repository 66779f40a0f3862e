#!/bin/bash
# GPU box: stream priority experiment (GS_PRIO 0/1/2) on the bench lines and G=8 strips;
# then orbit kernel statistics (working tree, GS_PRIO=${KP:-0}).
set -o pipefail
TAG=${1:-prio}; REPS=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
for r in $(seq $REPS); do
for v in 0 1 2; do
  GS_PRIO=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('prio%s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3))"
done
done
for v in 0 1 2; do
  GS_PRIO=$v GS=8 TIMING=2 timeout -k 10 200 python -u tools/strip_bench.py 2>&1 | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g;s/^/prio$v 1080p /"
done
(cd /tmp && GS_PRIO=${KP:-0} MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k.log 2>&1) || { tail -20 $OUT/k.log; exit 1; }
python3 tools/kstats.py $OUT/k/run_kernel_stats.csv 65 | head -20
echo done
