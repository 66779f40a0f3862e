#!/bin/bash
# GPU box: tools/gpu_iter.sh, then the 50 M / 4K bench line.  Usage: bash tools/gpu_iter4.sh TAG
set -o pipefail
bash tools/gpu_iter.sh $1 || exit 1
timeout -k 10 400 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$1/bench4.log 2>&1 || { tail -30 gpurun_out/$1/bench4.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/$1/bench4.log').read().strip().splitlines()[-1]);print('cfg4 fps',d['fps'],'ms',d['ms_per_step'],d['stages_ms'],'orbit',d.get('orbit',{}).get('fps'))"
