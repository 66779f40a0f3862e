#!/usr/bin/env python3
"""Frame statistics (ctx.timings(): visible splats, chunk split, entries, stage times) of every
row strip of G (env GS, default 1,8) at the bench configuration, frames serialised (timing=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402
from gsplat_amd.strips import strip_geometry  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), 1920, 1080
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    for G in (int(x) for x in os.environ.get("GS", "1,8").split(",")):
        rows = strip_geometry(H, 0, G)[1]
        buf = gs.DeviceBuffer((rows if G > 1 else H) * W * 16)
        for g in range(G):
            o = gs.make_opts(strip_index=g, strip_count=G, timing=1, out_format=gs.GS_OUT_RGBA_F16)
            for _ in range(8):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            ctx.timings_reset()
            for _ in range(20):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            st = ctx.timings()
            print("G=%d g=%d" % (G, g), {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()},
                  flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
