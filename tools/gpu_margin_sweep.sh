#!/bin/bash
# GPU box: orbit frame time (tools/orbit_probe.py, adaptive chunks) of lib/ab/libgsplat_m<margin>.so
# builds (GS_MOVING_MARGIN) against the default library, 1080p and 4K.
# Usage: bash tools/gpu_margin_sweep.sh "1.00 1.20"
set -o pipefail
export TMPDIR=/tmp
for c in 3 4; do
  for m in default $1; do
    if [ $m = default ]; then unset GSPLAT_LIB; else export GSPLAT_LIB=gaussian-splatting-web_amd/lib/ab/libgsplat_m$m.so; fi
    echo -n "config $c margin $m: "
    CONFIG=$c STEPS=60 MODE=adaptive timeout -k 10 200 python3 tools/orbit_probe.py 2>&1 | cut -c1-110 || exit 1
  done
done
unset GSPLAT_LIB
