#!/bin/bash
# GPU box: the 50 M / 3840x2160 configuration (BASELINE configs[4]) on one GPU: bench line and a
# kernel trace summary of the same command.  Usage: bash tools/cfg4_prof.sh TAG
set -o pipefail
TAG=${1:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]);print('fps',d['fps'],'ms',d['ms_per_step'],d['stages_ms'],'orbit',d.get('orbit',{}).get('fps'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
python3 tools/kstats.py $OUT/prof/run_kernel_stats.csv || true
echo done
