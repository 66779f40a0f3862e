#!/bin/bash
# GPU box: chunk-1 / split / order tests, orbit kernel stats, bench line.
set -o pipefail
TAG=${1:-s4}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_order.py tests/test_gpu_parity.py tests/test_gpu_bench_sequences.py -m gpu -x -q --timeout 500 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
(cd /tmp && LIST_SPLIT=0 MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k1 -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k1.log 2>&1) || { tail -20 $OUT/k1.log; exit 1; }
cat $OUT/k1.log | grep adaptive
python3 tools/kstats.py $OUT/k1/run_kernel_stats.csv 65 > $OUT/k1.txt; head -22 $OUT/k1.txt
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); print('fps %.1f orbit %.1f cold %.1f sparse %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
(cd /tmp && LIST_SPLIT=1 MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/k2 -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/k2.log 2>&1) || { tail -20 $OUT/k2.log; exit 1; }
python3 tools/kstats.py $OUT/k2/run_kernel_stats.csv 65 > $OUT/k2.txt; grep adaptive $OUT/k2.log; head -12 $OUT/k2.txt
echo done
