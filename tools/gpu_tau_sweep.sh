#!/bin/bash
# GPU box: seeded (cold) frame times of tools/cold_probe.py at several GS_SEED_TAU values.
# Usage: bash tools/gpu_tau_sweep.sh "6 9.21 12"
set -o pipefail
export TMPDIR=/tmp
for c in 3 4; do
  for t in $1; do
    echo "== config $c tau $t"
    GS_SEED_TAU=$t timeout -k 10 200 python3 tools/cold_probe.py $c 2>&1 | grep -E "^v[0-9]+ (cold|warm)" | cut -c1-150 || exit 1
  done
done
