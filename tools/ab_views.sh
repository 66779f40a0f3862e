#!/bin/bash
# GPU box: stage times of cold views 1 and 3 (tools/diag/view_probe.py) and the bench line for the
# default library and each lib/ab variant.  Usage: bash tools/ab_views.sh "base v1 v2"
set -o pipefail
mkdir -p gpurun_out/abv
for v in $1; do
  if [ "$v" = base ]; then L=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so; else L=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so; fi
  for V in 1 3; do
    GSPLAT_LIB=$L VIEW=$V timeout -k 10 120 python3 tools/diag/view_probe.py > gpurun_out/abv/${v}_v$V.txt 2>&1 || { tail -5 gpurun_out/abv/${v}_v$V.txt; exit 1; }
    python3 -c "import ast,sys; d=ast.literal_eval([l for l in open('gpurun_out/abv/${v}_v$V.txt') if l.startswith('{')][-1]); print('$v view $V total %.3f proj %.3f bin %.3f tsort %.3f comp %.3f c1 %.3f wide %d' % (d['ms_total'], d['ms_project'], d['ms_bin'], d['ms_tile_sort'], d['ms_composite'], d['ms_sort'], d['wide_chunk0']))"
  done
  GSPLAT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/abv/$v.log 2>&1 || { tail -5 gpurun_out/abv/$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abv/$v.log').read().strip().splitlines()[-1]); print('$v fps %.1f orbit %.1f cold %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps']), {k: round(x*1e3,1) for k,x in d['stages_ms'].items()})"
done
