#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace database (rocpd SQLite): per-kernel stats and the
launch sequence of the last frame with the idle gap before each kernel.

    python tools/trace_summary.py gpurun_out/TAG/prof/run_results.db [--frame-start k_project]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name.replace("gs::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--frame-start", default="k_project")
    ap.add_argument("--seq", action="store_true", help="print the last frame's launch sequence")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, "
                          "lds_size from kernels order by start"))
    stats = defaultdict(list)
    for r in rows:
        stats[short(r[0])].append((r[2] - r[1]) / 1e3)
    tot = sum(sum(v) for v in stats.values())
    print("%-44s %6s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "max_us", "pct"))
    for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
        print("%-44s %6d %10.1f %10.2f %10.2f %6.2f" % (k, len(v), sum(v), sum(v) / len(v), max(v),
                                                        100 * sum(v) / tot))
    starts = [i for i, r in enumerate(rows) if a.frame_start in r[0]]
    if a.seq and len(starts) >= 2:
        i0, i1 = starts[-2], starts[-1]
        print("\nframe (second to last), %d kernels, span %.1f us:" % (i1 - i0, (rows[i1][1] - rows[i0][1]) / 1e3))
        prev_end = rows[i0 - 1][2] if i0 else rows[i0][1]
        for r in rows[i0:i1]:
            print("  gap %7.2f  dur %8.2f  grid %8d x %4d  vgpr %3d/%3d lds %6d  %s" % (
                (r[1] - prev_end) / 1e3, (r[2] - r[1]) / 1e3, r[3], r[4], r[5], r[6], r[7], short(r[0])))
            prev_end = r[2]


if __name__ == "__main__":
    main()
