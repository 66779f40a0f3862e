#!/bin/bash
# GPU box: orbit frame time (tools/orbit_probe.py, adaptive chunks) at several saturation quantiles
# of the chunk controller, 1080p and 4K.  Usage: bash tools/gpu_qsweep_orbit.sh "0.5 0.8 0.95"
set -o pipefail
export TMPDIR=/tmp
for c in 3 4; do
  for q in $1; do
    echo -n "config $c q=$q: "
    GS_SAT_QUANTILE=$q CONFIG=$c STEPS=60 MODE=adaptive timeout -k 10 200 python3 tools/orbit_probe.py 2>&1 | cut -c1-120 || exit 1
  done
done
