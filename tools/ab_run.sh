set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; tail -2 gpurun_out/ab/tests.log
for v in base nohist base nohist; do
  GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 100 > gpurun_out/ab/$v.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v.log').read().strip().splitlines()[-1]); print('$v', d['fps'], d['stages_ms']['ms_chunk1'], d['stages_ms']['ms_composite'])"
done
