#!/usr/bin/env python3
"""Kernel timeline window from a rocprofv3 kernel-trace CSV: every launch that starts in
[t, t + span) of the run's last part (start / end in us relative to the window, queue id), to see
how the launches of frames in flight overlap.   python tools/timeline.py run_kernel_trace.csv [span_us]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
span = float(sys.argv[2]) if len(sys.argv) > 2 else 400.0
t_end = int(rows[-1]["End_Timestamp"])
t0 = t_end - int(span * 2e3)
qcol = next((c for c in ("Queue_Id", "Stream_Id", "Queue_ID") if c in rows[0]), None)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s >= t0 + span * 1e3:
        continue
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("gs::", "")
    print("%8.1f %8.1f %7.1f  q%-4s %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, r.get(qcol, "?") if qcol else "?", n))
