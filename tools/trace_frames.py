#!/usr/bin/env python3
"""Per-frame kernel sequence from a rocprofv3 kernel-trace CSV: the last FRAMES frames (a frame
starts at the kernel named --start), each kernel's duration and the idle gap before it."""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("void ", "")
    return n.replace("gs::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--start", default="k_cull")
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == a.start]
    for f0, f1 in list(zip(idx, idx[1:]))[-a.frames:]:
        t0 = int(rows[f0]["Start_Timestamp"])
        print("frame span %.1f us" % ((int(rows[f1]["Start_Timestamp"]) - t0) / 1e3))
        prev = int(rows[f0 - 1]["End_Timestamp"]) if f0 else t0
        for r in rows[f0:f1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print("  gap %6.1f  dur %7.1f  %s" % ((s - prev) / 1e3, (e - s) / 1e3, short(r["Kernel_Name"])))
            prev = e


if __name__ == "__main__":
    main()
