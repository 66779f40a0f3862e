#!/usr/bin/env python3
"""Diagnostic: per-stage frame times and per-chunk work at fixed first-chunk fractions
(bench workload).  python tools/chunk_sweep.py [--n 6100000] [--fractions 0.05,0.1,...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=6_100_000)
    ap.add_argument("--fractions", default="0.02,0.04,0.06,0.08,0.1,0.14,0.2,0.3,0.5,1.0,0")
    ap.add_argument("--frames", type=int, default=20)
    a = ap.parse_args()
    W, H = 1920, 1080
    aos = gs.synth_aos(a.n, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, a.n, 16)
    buf = gs.DeviceBuffer(H * W * 16)
    keys = ("ms_total", "ms_project", "ms_sort", "ms_bin", "ms_tile_sort", "ms_ranges", "ms_composite")
    print("f      " + " ".join("%9s" % k[3:] for k in keys) + "   k_chunk0  k_chunk1 unsat wide0 wide1 f_used")
    for f in [float(x) for x in a.fractions.split(",")]:
        o = gs.make_opts(timing=1, chunk_fraction=f)
        for _ in range(5):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        ctx.timings_reset()
        for _ in range(a.frames):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        st = ctx.timings()
        print("%-6g " % f + " ".join("%9.4f" % st[k] for k in keys) +
              " %10d %9d %5d %5d %5d %.3f" % (st["k_chunk0"], st["k_chunk1"], st["tiles_unsaturated"],
                                            st["wide_chunk0"], st["wide_chunk1"], st["chunk_fraction"]),
              flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
