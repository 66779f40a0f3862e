#!/usr/bin/env python3
"""Host-side cost of enqueuing bench frames: wall time of N render_device calls (no sync) vs the
time until the GPU drains, at timing levels 0 and 2 (env GS / STRIP: one row strip of GS)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), 1920, 1080
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    buf = gs.DeviceBuffer(H * W * 8)
    G, S = int(os.environ.get("GS", "1")), int(os.environ.get("STRIP", "0"))
    for lvl in (0, 2, 0):
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=lvl, strip_index=S, strip_count=G)
        for _ in range(10):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        F = 200
        t0 = time.perf_counter()
        per = []
        for _ in range(F):
            a = time.perf_counter()
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            per.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        ctx.sync()
        t2 = time.perf_counter()
        per.sort()
        print("timing=%d: enqueue %.1f us/frame (p50 %.1f p90 %.1f max %.1f), total %.1f us/frame" %
              (lvl, (t1 - t0) / F * 1e6, per[F // 2] * 1e6, per[int(F * 0.9)] * 1e6, per[-1] * 1e6,
               (t2 - t0) / F * 1e6), flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
