set -o pipefail
bash tools/gpu_check.sh r1q || exit 1
timeout -k 10 400 python tools/strip_bench.py
