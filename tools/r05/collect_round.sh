#!/bin/bash
# Here (CPU): turn a tools/round_profiles_r05.sh run (gpurun_out/round_TAG, gpurun_out/prof_TAG)
# into the committed profiles/r05_* set.   bash tools/r05/collect_round.sh TAG
set -e
T=${1:?tag}; R=gpurun_out/round_$T; P=profiles
python3 tools/profile_summary.py gpurun_out/prof_$T r05
tail -n 1 $R/bench.log > $P/r05_bench.json
tail -n 1 $R/bench_cfg4.log > $P/r05_bench_cfg4.json
cp $R/c4/run_kernel_stats.csv $P/r05_cfg4_kernel_stats.csv
python3 tools/trace_median.py $R/c4s/run_kernel_trace.csv > $P/r05_cfg4_serialised.txt
cp $R/strips.log $P/r05_strips.txt
cp $R/strips_cfg4.log $P/r05_strips_cfg4.txt
cp $R/strip8_timeline.txt $P/r05_strip8_timeline.txt
cp $R/onechunk.txt $P/r05_onechunk.txt
cp $R/group_host_time.txt $P/r05_group_host_time.txt
cp $R/orbit.txt $P/r05_orbit.txt
echo collected $T
