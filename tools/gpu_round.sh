#!/bin/bash
# GPU box: full parity suite, the default bench line, the 50 M / 4K bench line, and a torchrun
# N=1 launch of the same bench (the driver's launcher).  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_cfg4.log 2>&1 || { tail -30 $OUT/bench_cfg4.log; exit 1; }
tail -1 $OUT/bench_cfg4.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline > $OUT/bench_torchrun.log 2>&1 || { tail -30 $OUT/bench_torchrun.log; exit 1; }
tail -1 $OUT/bench_torchrun.log
echo done
