#!/bin/bash
# GPU box: the strip bound with and without stage events (TIMING 0 / 2), 200 timed frames per strip.
set -o pipefail
export TMPDIR=/tmp
for t in 0 2; do
  GS=1,8 TIMING=$t FRAMES=200 timeout -k 10 300 python -u tools/strip_bench.py 2>&1 | grep "G=" | cut -c1-60 | sed -e "s/^/timing$t 1080p /"
  N=50000000 W=3840 H=2160 SEED=50 GS=1,8 TIMING=$t FRAMES=200 WARMUP=10 timeout -k 10 500 python -u tools/strip_bench.py 2>&1 | grep "G=" | cut -c1-60 | sed -e "s/^/timing$t 4k /"
done
echo done
