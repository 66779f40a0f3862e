#!/bin/bash
# GPU box: the driver's bench command (--steps 20 --warmup 5) with and without the prewarm.
set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
for pw in 0.2 0; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 --prewarm $pw > gpurun_out/pw.log 2>&1 || { tail -5 gpurun_out/pw.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/pw.log').read().strip().splitlines()[-1]); print('prewarm $pw: fps %.1f ms_per_step %.4f' % (d['fps'], d['ms_per_step']), d['config']['prewarm'])"
done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/pw_full.log 2>&1 || { tail -5 gpurun_out/pw_full.log; exit 1; }
tail -n 1 gpurun_out/pw_full.log | cut -c1-400
echo done
