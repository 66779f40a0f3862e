#!/bin/bash
# GPU box: 50 M / 4K bench line (and the 1080p headline) for the default library and each lib/ab
# variant.  Usage: bash tools/ab_cfg4.sh "base v1 v2"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in $1; do
  if [ "$v" = base ]; then L=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so; else L=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so; fi
  GSPLAT_LIB=$L timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/c4_$v.log 2>&1 || { tail -5 gpurun_out/ab/c4_$v.log; exit 1; }
  GSPLAT_LIB=$L timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-extra > gpurun_out/ab/h_$v.log 2>&1 || { tail -5 gpurun_out/ab/h_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/c4_$v.log').read().strip().splitlines()[-1]); h=json.loads(open('gpurun_out/ab/h_$v.log').read().strip().splitlines()[-1]); print('$v 4K fps %.1f orbit %.1f' % (d['fps'], d['orbit']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()}, '1080p fps %.1f' % h['fps'])"
done
