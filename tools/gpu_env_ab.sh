#!/bin/bash
# GPU box: bench line + strip bound under an environment switch.  Usage: bash tools/gpu_env_ab.sh VAR "v1 v2" [tests]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/env
VAR=$1
if [ "$3" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/env/tests.log 2>&1 || { tail -40 gpurun_out/env/tests.log; exit 1; }
  tail -2 gpurun_out/env/tests.log
fi
for v in $2; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/env/b$v.log 2>&1 || { tail -5 gpurun_out/env/b$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/env/b$v.log').read().strip().splitlines()[-1]); print('$VAR=$v fps %.1f orbit %.1f cold %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  env $VAR=$v GS=1,2,4,8 TIMING=2 timeout -k 10 200 python tools/strip_bench.py 2>&1 | cut -c1-60
done
