#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, kernel trace only).
# Usage (GPU box): bash tools/pmc.sh TAG [command...]   (default: a short bench run)
set -o pipefail
TAG=${1:-pmc}; shift
CMD=("$@")
[ ${#CMD[@]} -eq 0 ] && CMD=(python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline)
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
      "${CMD[@]}" > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc done
