set -o pipefail
for v in S2 S3; do
  GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so timeout -k 10 120 python3 -u tools/diag/host_time.py > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo $v $(head -1 gpurun_out/ab_$v.log)
  GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/ab/libgsplat_$v.so GS=1,4,8 TIMING=2 timeout -k 10 120 python3 -u tools/strip_bench.py 2>&1 | cut -c1-60 || exit 1
done
