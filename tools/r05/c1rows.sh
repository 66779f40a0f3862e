#!/bin/bash
# GPU box: k_c1_rows alone (orbit frames, stages serialised) for the working tree and variants.
set -o pipefail
TAG=${1:-c1r}; VARS=${2:-c1e c1g}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
B=$PWD/gaussian-splatting-web_amd/lib/libgsplat.so
lib() { if [ "$1" = base ]; then echo $B; else echo $R/gaussian-splatting-web_amd/lib/ab/libgsplat_$1.so; fi; }
for v in base $VARS; do
(cd /tmp && GSPLAT_LIB=$(lib $v) MODE=adaptive_staged timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/$v -o run -- python3 $R/tools/orbit_probe.py > $R/$OUT/$v.log 2>&1) || { tail -20 $OUT/$v.log; exit 1; }
python3 tools/kstats.py $OUT/$v/run_kernel_stats.csv 65 > $OUT/$v.txt
echo "$v: $(grep -E 'k_c1_rows|k_c1_parts ' $OUT/$v.txt | tr -s ' ' | tr '\n' ';')"
done
echo done
