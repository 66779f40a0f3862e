#!/bin/bash
# GPU box: GPU tests, then bench line + strip bound with frame graphs on and off (GSPLAT_GRAPHS).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gr
if [ "$1" != notests ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gr/tests.log 2>&1 || { tail -40 gpurun_out/gr/tests.log; exit 1; }
tail -2 gpurun_out/gr/tests.log
fi
for g in 1 0; do
  GSPLAT_GRAPHS=$g timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/gr/b$g.log 2>&1 || { tail -5 gpurun_out/gr/b$g.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/gr/b$g.log').read().strip().splitlines()[-1]); print('graphs=$g fps %.1f orbit %.1f cold %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  GSPLAT_GRAPHS=$g GS=1,2,4,8 TIMING=2 timeout -k 10 200 python tools/strip_bench.py 2>&1 | cut -c1-60
  GSPLAT_GRAPHS=$g GS=8 STRIP=1 timeout -k 10 200 python tools/diag/host_time.py 2>&1 | tail -1
done
