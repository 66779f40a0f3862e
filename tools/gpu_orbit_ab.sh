#!/bin/bash
# GPU box: orbit and cold frame times (tools/orbit_probe.py adaptive, tools/cold_probe.py) of the
# default library against lib/ab/<variant>.so, alternating.  Usage: bash tools/gpu_orbit_ab.sh VARIANT [rounds]
set -o pipefail
export TMPDIR=/tmp
V=$1; R=${2:-2}
for i in $(seq 1 $R); do
  for c in 3 4; do
    for lib in default $V; do
      if [ $lib = default ]; then unset GSPLAT_LIB; else export GSPLAT_LIB=gaussian-splatting-web_amd/lib/ab/$lib.so; fi
      echo -n "config $c $lib: "
      CONFIG=$c STEPS=60 MODE=adaptive timeout -k 10 200 python3 tools/orbit_probe.py 2>&1 | cut -c1-100 || exit 1
    done
  done
done
unset GSPLAT_LIB
