set -o pipefail
timeout -k 10 300 python tools/chunk_sweep.py --fractions 0.14,0.2,0 --frames 30
