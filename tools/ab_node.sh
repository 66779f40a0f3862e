#!/bin/bash
# GPU box: Node drop-in fps (tools/node_fps.js, 200 frames) and the bench line for lib/ab variants,
# each variant copied over lib/libgsplat.so in turn (the addon loads that file), two alternating passes.
# Usage: bash tools/ab_node.sh "v1 v2"
set -o pipefail
L=gaussian-splatting-web_amd/lib
for pass in 1 2; do
  for v in $1; do
    cp $L/ab/libgsplat_$v.so $L/libgsplat.so
    n=$(timeout -k 10 200 node tools/node_fps.js 6100000 6 1920 1080 200) || exit 1
    b=$(timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-extra) || exit 1
    python3 -c "import json,sys; n=json.loads(sys.argv[1]); b=json.loads(sys.argv[2].strip().splitlines()[-1]); print('$v pass $pass node %.0f / %.0f  bench %.0f' % (n['device_resident_fps'], n['host_readback_fps'], b['fps']))" "$n" "$b"
  done
done
