#!/bin/bash
# GPU box: bench line (static + orbit) and G=8 strip bound for the default library and each
# lib/ab variant.  Usage: bash tools/ab_run.sh "base g1 g4" [tests]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ "$2" = tests ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; tail -2 gpurun_out/ab/tests.log
fi
for v in $1; do
  if [ "$v" = base ]; then L=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so; else L=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so; fi
  GSPLAT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab/$v.log 2>&1 || { tail -5 gpurun_out/ab/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); print('$v fps %.1f orbit %.1f' % (d['fps'], d['orbit']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
  GSPLAT_LIB=$L GS=1,8 TIMING=2 timeout -k 10 200 python tools/strip_bench.py 2>&1 | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g"
done
