#!/usr/bin/env python3
"""Per-rank frame time of the row-strip split, measured one strip at a time on one GPU (the
8-GPU run itself is the driver's): for G in 1, 2, 4, 8, every strip's mean frame time and stage
times; the slowest strip bounds the G-GPU frame (plus the all-gather).  Env: N, W, H, SEED, GS,
STRIP, TIMING (0: no events; 1: every stage; 2: the composite only), WARMUP, FRAMES (timed)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402
from gsplat_amd.strips import strip_geometry  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    aos = gs.synth_aos(N, int(os.environ.get("SEED", 6)), W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    base = 0.0
    sc = gs.Scene(ctx, aos, N, 16)
    gl = tuple(int(x) for x in os.environ.get("GS", "1,2,4,8").split(","))
    only = int(os.environ["STRIP"]) if "STRIP" in os.environ else None
    for G in gl:
        rows = strip_geometry(H, 0, G)[1]
        buf = gs.DeviceBuffer((rows if G > 1 else H) * W * 16)
        worst = 0.0
        line = []
        for g in range(G):
            if only is not None and g != only:
                continue
            o = gs.make_opts(strip_index=g, strip_count=G, timing=int(os.environ.get("TIMING", "1")),
                             out_format=gs.GS_OUT_RGBA_F16, list_split=int(os.environ.get("LIST_SPLIT", "0")))
            # warm-up: the scene's chunk controller was last fed another strip's statistics,
            # which reach the host up to 8 frames late
            for _ in range(int(os.environ.get("WARMUP", 20))):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            ctx.timings_reset()
            nf = int(os.environ.get("FRAMES", 30))
            t0 = time.perf_counter()
            for _ in range(nf):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            ms = (time.perf_counter() - t0) / nf * 1e3
            st = ctx.timings()
            worst = max(worst, ms)
            line.append("%d:%.3f(p%.3f s%.3f b%.3f t%.3f c%.3f)" % (g, ms, st["ms_project"], st["ms_sort"],
                                                                  st["ms_bin"], st["ms_tile_sort"], st["ms_composite"]))
        base = worst if G == 1 else base
        print("G=%d worst %.3f ms  speedup-bound %.2f  | %s" % (G, worst, base / worst if worst else 0.0,
                                                            " ".join(line)), flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
