#!/usr/bin/env python3
"""Median / min duration and launch count per kernel from a rocprofv3 kernel trace CSV:
    python tools/trace_median.py run_kernel_trace.csv"""
import collections
import csv
import re
import statistics
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("gs::", "")
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
frames = max((len(v) for k, v in d.items() if k.startswith("k_composite")), default=1)
for n, v in sorted(d.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print("%-34s median %8.2f us  min %8.2f  launches/frame %5.2f" % (n, statistics.median(v), min(v), len(v) / frames))
