#!/bin/bash
# GPU box: k_cull changes: the GPU suite (or TESTS), bench A/B against lib/ab variants, and
# kernel stats of one-chunk frames (sparse, 50 M / 4K) for each library.
set -o pipefail
TAG=${1:-cull}; VARS=${2:-prev}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
B=$R/gaussian-splatting-web_amd/lib/libgsplat.so
lib() { if [ "$1" = base ]; then echo $B; else echo $R/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
for v in base $VARS; do
  GSPLAT_LIB=$(lib $v) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > $OUT/b_${v}_$r.log 2>&1 || { tail -5 $OUT/b_${v}_$r.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.log').read().strip().splitlines()[-1]); print('%-6s fps %.1f orbit %.1f cold %.1f sparse %.1f (comp %.1f)' % ('$v', d['fps'], d['orbit']['fps'], d['cold']['fps'], d['sparse']['fps'], d['sparse']['ms_composite']*1e3), {k: round(v*1e3,1) for k,v in d['stages_ms'].items()})"
done
done
for v in base $VARS; do
for w in sparse cfg4; do
  (cd /tmp && GSPLAT_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/${v}_$w -o run -- python3 $R/tools/diag/onechunk_probe.py $w 5 > $R/$OUT/${v}_$w.log 2>&1) || { tail -30 $OUT/${v}_$w.log; exit 1; }
  echo "$v $(grep 'one-chunk' $OUT/${v}_$w.log | cut -c1-60)"
  python3 tools/kstats.py $OUT/${v}_$w/run_kernel_stats.csv 6 | grep -E "k_tile_sort|k_bin_emit" | sed -e "s/^/   /"
done
done
echo done
