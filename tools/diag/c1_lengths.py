#!/usr/bin/env python3
"""Chunk-1 list lengths per frame from a GS_C1_PRINT diagnostics build's device printf lines
("C1T tile len" per chunk-1 tile, then the frame end's "C1F not_done n c1_parts m").

    GSPLAT_LIB=lib/libgsplat_c1print.so MODE=adaptive STEPS=8 python tools/orbit_probe.py > log
    python tools/diag/c1_lengths.py log
"""
import sys

import numpy as np


def main():
    frames, cur = [], []
    for line in open(sys.argv[1]):
        p = line.split()
        if p[:1] == ["C1T"]:
            cur.append(int(p[2]))
        elif p[:1] == ["C1F"]:
            frames.append((int(p[2]), int(p[4]), cur))
            cur = []
    for nd, parts, L in frames[-6:]:
        a = np.array(L) if L else np.zeros(1)
        print("not_done %5d c1_parts %6d  tiles %5d entries %7d  len p50 %5d p90 %5d p99 %5d max %5d  top10 %s"
              % (nd, parts, len(L), a.sum(), np.percentile(a, 50), np.percentile(a, 90), np.percentile(a, 99),
                 a.max(), sorted(L)[-10:]))


if __name__ == "__main__":
    main()
