#!/bin/bash
# GPU box: the profile set committed under profiles/ for a round.
#   1. rocprofv3 --kernel-trace --stats over the default bench command (short)
#   2. PMC passes (SQ, FETCH_SIZE, WRITE_SIZE) over the same command, one group per run
# Usage: bash tools/collect_profiles.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $BENCH \
    > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 $BENCH \
      > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run fetch FETCH_SIZE
run write WRITE_SIZE
echo profiles done
