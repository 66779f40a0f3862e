#!/usr/bin/env python3
"""From a rocprofv3 --kernel-trace --hip-trace run: for each launch of a kernel (default
k_part_list, the first of a frame's chain), when the host called hipLaunchKernel and when the
kernel started (us, relative to the first such call), i.e. whether the chain waited for the host
or for the GPU.   python tools/diag/enqueue_lag.py OUT_DIR/run [kernel]"""
import csv
import re
import sys

base = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_part_list"
kt = list(csv.DictReader(open(base + "_kernel_trace.csv")))
ht = list(csv.DictReader(open(base + "_hip_api_trace.csv")))
kernels = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"]))
                 for r in kt if name in r["Kernel_Name"])
api = {int(r["Correlation_Id"]): (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in ht}
rows = [(api[c][0], s, e) for s, e, c in kernels if c in api][-12:]
t0 = rows[0][0]
for call, s, e in rows:
    print("host call %9.1f  kernel start %9.1f  lag %7.1f us" % ((call - t0) / 1e3, (s - t0) / 1e3, (s - call) / 1e3))
