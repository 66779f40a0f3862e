"""Seeded (cold) frames against the steady state of the same view: per view of gsplat_amd.COLD_VIEWS,
one frame right after a cut (seeded) and the 8th frame on that view (the controller's history),
each serialised with stage timing.  Usage: python tools/cold_probe.py [cfg 3|4]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N, W, H, seed = {3: (6_100_000, 1920, 1080, 6), 4: (50_000_000, 3840, 2160, 50)}[cfg]
ctx = gs.Context(0)
sc = gs.Scene(ctx, gs.synth_aos(N, seed, W, H), N, 16)
buf = gs.DeviceBuffer(W * H * 8)
o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=1)


def frame(u):
    ctx.timings_reset()
    sc.render_device(u, W, H, buf.ptr.value, W * H * 8, None, o)
    ctx.sync()
    return ctx.timings()


def show(tag, st):
    print("%-10s %6.3f ms  proj %.3f bin %.3f tsort %.3f comp %.3f c1 %.3f | chunk0 %.4f T %.3f unsat %5d k0 %8d k1 %8d"
          % (tag, st["ms_total"], st["ms_project"], st["ms_bin"], st["ms_tile_sort"], st["ms_composite"],
             st["ms_sort"], st["chunk_fraction"], st["chunk_depth"], st["tiles_unsaturated"], st["k_chunk0"], st["k_chunk1"]), flush=True)


tot = {"cold": 0.0, "warm": 0.0}
for rep in range(2):
    for v in range(len(gs.COLD_VIEWS)):
        u = gs.cold_uniforms(W, H, v)
        st = frame(u)
        show("v%d cold" % v, st)
        tot["cold"] += st["ms_total"] * (rep == 1)
        for _ in range(6):
            frame(u)
        st = frame(u)
        show("v%d warm" % v, st)
        tot["warm"] += st["ms_total"] * (rep == 1)
print("TOTAL cold %.3f warm %.3f (4 views, serialised, %s)" % (tot["cold"], tot["warm"], os.environ.get("GS_SEED_TAU", "")))
one = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=1, chunk_fraction=1.0)
for v in range(len(gs.COLD_VIEWS) if os.environ.get("ONECHUNK") else 0):
    ctx.timings_reset()
    sc.render_device(gs.cold_uniforms(W, H, v), W, H, buf.ptr.value, W * H * 8, None, one)
    ctx.sync()
    show("v%d 1chunk" % v, ctx.timings())
