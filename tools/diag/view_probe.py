#!/usr/bin/env python3
"""One view of gsplat_amd.COLD_VIEWS rendered repeatedly (warm, stage timing): frame statistics
incl. wide splats, for profiling a single view under rocprofv3.   VIEW=3 python tools/diag/view_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402

N, W, H, seed = 6_100_000, 1920, 1080, 6
v = int(os.environ.get("VIEW", "3"))
ctx = gs.Context(0)
sc = gs.Scene(ctx, gs.synth_aos(N, seed, W, H), N, 16)
buf = gs.DeviceBuffer(W * H * 8)
o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=1)
u = gs.cold_uniforms(W, H, v)
for k in range(12):
    ctx.timings_reset()
    sc.render_device(u, W, H, buf.ptr.value, W * H * 8, None, o)
    ctx.sync()
st = ctx.timings()
print({k: (round(x, 4) if isinstance(x, float) else x) for k, x in st.items()})
