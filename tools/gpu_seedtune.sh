#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-seedtune}
mkdir -p $OUT
for TAU in 9.21 6 4 2.5; do
  for C in 3 4; do
    GS_SEED_TAU=$TAU timeout -k 10 300 python tools/cold_probe.py $C > $OUT/c${C}_t$TAU.log 2>&1 || { tail -20 $OUT/c${C}_t$TAU.log; exit 1; }
    echo "cfg $C: $(tail -1 $OUT/c${C}_t$TAU.log)"
  done
done
