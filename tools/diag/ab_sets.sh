# A/B of library variants in lib/ab (G=1 throughput with frames in flight, G=4/8 strips)
set -o pipefail
for v in ${VARIANTS:-D2 D3 D2 D3}; do
  GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so timeout -k 10 120 python3 -u tools/diag/host_time.py > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo $v $(head -1 gpurun_out/ab_$v.log | cut -c1-90)
  GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so GS=${GSL:-4,8} TIMING=2 timeout -k 10 120 python3 -u tools/strip_bench.py 2>&1 | cut -c1-50 || exit 1
done
