#!/bin/bash
# GPU box: the bench line's value against the timed window (the driver runs --steps 20 --warmup 5).
set -o pipefail
export TMPDIR=/tmp
for sw in "20 5" "20 50" "100 5" "200 20"; do
  set -- $sw
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps $1 --warmup $2 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('steps $1 warmup $2: fps %.1f ms_per_step %.4f' % (d['fps'], d['ms_per_step']))"
done
echo done
