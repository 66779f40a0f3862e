#!/bin/bash
# GPU box: bench (list split on / off) and the G=8 strip bound for base and the lib/ab variants.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab1; mkdir -p $OUT
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
for ls in 0 1; do
  GSPLAT_LIB=$B timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --list-split $ls > $OUT/bench_ls$ls.log 2>&1 || { tail -5 $OUT/bench_ls$ls.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_ls$ls.log').read().strip().splitlines()[-1]); print('list_split $ls fps %.1f orbit %.1f cold %.1f sparse %.1f' % (d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps']), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
for v in base b4 q2k; do
  if [ "$v" = base ]; then L=$B; else L=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so; fi
  echo "== $v"
  LIST_SPLIT=0 GSPLAT_LIB=$L GS=1,8 TIMING=2 timeout -k 10 200 python tools/strip_bench.py 2>&1 | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g"
done
echo done
