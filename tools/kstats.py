#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel summary (run_kernel_stats.csv) as per-frame microseconds:
    python tools/kstats.py gpurun_out/<tag>/prof/run_kernel_stats.csv [frames]
Average duration and calls per frame (frames = calls of k_composite by default)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else max(
    (int(r["Calls"]) for r in rows if "k_composite" in r["Name"]), default=1)
tot = 0.0
for r in rows:
    name = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("gs::", "")
    per = float(r["TotalDurationNs"]) / frames / 1e3
    tot += per
    print("%-36s avg %9.2f us  calls/frame %5.2f  per-frame %9.2f us" % (name, float(r["AverageNs"]) / 1e3,
                                                                        int(r["Calls"]) / frames, per))
print("%-36s %40.2f us" % ("total per frame", tot))
