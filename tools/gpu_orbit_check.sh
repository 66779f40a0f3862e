#!/bin/bash
# GPU box: the GPU suite, a bench line and the orbit's per-kernel times (rocprofv3 over
# tools/orbit_probe.py, the adaptive mode).  Usage: bash tools/gpu_orbit_check.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-orb}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
python3 -c "
import json
d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1])
print('bench %.1f fps  orbit %.1f  cold %.1f  sparse %.1f  stages %s' % (d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['stages_ms']))"
MODE=adaptive timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/orb -o run -- python3 tools/orbit_probe.py > $OUT/orb.log 2>&1 || { tail -20 $OUT/orb.log; exit 1; }
grep adaptive $OUT/orb.log
python3 tools/kstats.py $OUT/orb/run_kernel_stats.csv > $OUT/orb_k.txt || true
head -20 $OUT/orb_k.txt
