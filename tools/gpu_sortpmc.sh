#!/bin/bash
# GPU box: PMC passes over one-chunk frames (tools/diag/onechunk_probe.py), for the long-list
# per-tile sort.  Usage: bash tools/gpu_sortpmc.sh TAG [cfg4|sparse] [kernel]
set -o pipefail
TAG=${1:-sp}
W=${2:-cfg4}
K=${3:-k_tile_sort_huge}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="python3 tools/diag/onechunk_probe.py $W 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $P > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
grep "one-chunk" $OUT/stats.log
python3 tools/kstats.py $OUT/stats/run_kernel_stats.csv 4 > $OUT/kstats.txt || true
cat $OUT/kstats.txt
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- $P \
      > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
python3 tools/pmc_summary.py $OUT > $OUT/pmc.txt
grep -A 18 "^$K\$" $OUT/pmc.txt || true
echo done
