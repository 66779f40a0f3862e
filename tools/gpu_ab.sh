#!/bin/bash
# GPU box: A/B of the default library against lib/ab/<variant>.so on the bench line (fps only),
# alternating runs.  Usage: bash tools/gpu_ab.sh VARIANT [rounds] [bench args...]
set -o pipefail
V=$1; R=${2:-3}; shift 2
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for lib in default $V; do
    if [ $lib = default ]; then unset GSPLAT_LIB; else export GSPLAT_LIB=gaussian-splatting-web_amd/lib/ab/$lib.so; fi
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extra "$@" > gpurun_out/ab/$lib.$i.json 2>gpurun_out/ab/$lib.$i.err || { tail -5 gpurun_out/ab/$lib.$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-16s fps %8.1f  composite %s' % (sys.argv[2], d['fps'], d.get('roofline',{}).get('achieved')))" gpurun_out/ab/$lib.$i.json $lib
  done
done
unset GSPLAT_LIB
