#!/bin/bash
# GPU box: bench lines with the list split off / on (orbit: chunk 1's long lists split over four
# wave pairs), and the orbit frames' kernel statistics with it on.
set -o pipefail
TAG=${1:-so}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
for r in 1 2; do
for ls in 0 1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --list-split $ls > $OUT/b_${ls}_$r.log 2>&1 || { tail -5 $OUT/b_${ls}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${ls}_$r.log').read().strip().splitlines()[-1]); print('split%s fps %.1f orbit %.1f cold %.1f sparse %.1f' % ('$ls', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']))"
done
done
(cd /tmp && LIST_SPLIT=1 MODE=adaptive_staged timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k.log 2>&1) || { tail -20 $OUT/k.log; exit 1; }
python3 tools/kstats.py $OUT/k/run_kernel_stats.csv 65 > $OUT/k.txt; grep -E "composite|c1_|frame_end" $OUT/k.txt
echo done
