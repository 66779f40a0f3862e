#!/bin/bash
# GPU box: full -m gpu suite, bench, strips (1080p + 4K), orbit kernel stats.
set -o pipefail
TAG=${1:-s5}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print('fps %.1f orbit %.1f cold %.1f sparse %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
TIMING=2 timeout -k 10 200 python -u tools/strip_bench.py > $OUT/strips.txt 2>&1 || { tail -20 $OUT/strips.txt; exit 1; }
cat $OUT/strips.txt
N=50000000 W=3840 H=2160 SEED=50 TIMING=2 WARMUP=10 timeout -k 10 400 python -u tools/strip_bench.py > $OUT/strips_cfg4.txt 2>&1 || { tail -20 $OUT/strips_cfg4.txt; exit 1; }
cat $OUT/strips_cfg4.txt
(cd /tmp && MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/ko -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/ko.log 2>&1) || { tail -20 $OUT/ko.log; exit 1; }
grep adaptive $OUT/ko.log; python3 tools/kstats.py $OUT/ko/run_kernel_stats.csv 65 > $OUT/ko.txt; head -16 $OUT/ko.txt
echo done
