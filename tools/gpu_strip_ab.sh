#!/bin/bash
# GPU box: G=1,8 strip bound with and without an environment switch (A/B), twice each, plus the
# device-group host time.  Usage: bash tools/gpu_strip_ab.sh VAR
set -o pipefail
export TMPDIR=/tmp
V=${1:-GS_NO_FUSE_PARTS}
for r in 1 2; do
  for e in 0 1; do
    echo "== $V=$e"
    env $V=$e GS=1,8 TIMING=2 timeout -k 10 200 python3 tools/strip_bench.py 2>&1 | sed -e "s/(p0.000 s0.000 b0.000 t0.000 /(/g" | cut -c1-60 || exit 1
  done
done
timeout -k 10 300 python3 tools/diag/group_host_time.py || exit 1
