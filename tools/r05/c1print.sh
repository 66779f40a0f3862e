#!/bin/bash
set -o pipefail
OUT=gpurun_out/c1p; mkdir -p $OUT
export TMPDIR=/tmp
STEPS=12 MODE=adaptive GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_c1p.so timeout -k 10 200 python -u tools/orbit_probe.py > $OUT/probe.txt 2>&1 || { tail -20 $OUT/probe.txt; exit 1; }
grep -c C1T $OUT/probe.txt; grep C1F $OUT/probe.txt | tail -12
python3 - <<'PY'
import collections
L=[l.split() for l in open('gpurun_out/c1p/probe.txt') if l.startswith('C1T')]
n=[int(x[2]) for x in L]
print('C1T tiles', len(n), 'entries', sum(n), 'max', max(n) if n else 0, 'zero', sum(1 for x in n if x==0), '>=256', sum(1 for x in n if x>=256))
PY
echo done
