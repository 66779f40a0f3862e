set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t8.log 2>&1; tail -3 gpurun_out/t8.log
timeout -k 10 300 python tools/chunk_sweep.py --fractions 0.1,0.14,0.2,1.0,0
