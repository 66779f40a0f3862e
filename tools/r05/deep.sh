#!/bin/bash
# GPU box: three frames in flight at the bench size (GS_DEEP_TILES) against two: bench lines.
set -o pipefail
export TMPDIR=/tmp
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
D=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_deep3.so
for r in 1 2 3; do
for v in base deep3; do
  L=$B; [ $v = deep3 ] && L=$D
  GSPLAT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/dp.log 2>&1 || { tail -5 gpurun_out/dp.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dp.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']))"
done
done
echo done
