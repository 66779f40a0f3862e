import os, sys, time
sys.path.insert(0, "gaussian-splatting-web_amd")
import gsplat_amd as gs
N, W, H = 6_100_000, 1920, 1080
aos = gs.synth_aos(N, 6, W, H); u = gs.bench_uniforms(W, H)
ctx = gs.Context(0); sc = gs.Scene(ctx, aos, N, 16)
for G in (1, 8):
    buf = gs.DeviceBuffer(H * W * 16)
    o = gs.make_opts(strip_index=3 if G > 1 else 0, strip_count=G, timing=1)
    for _ in range(5): sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync(); ctx.timings_reset()
    for _ in range(30): sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync(); st = ctx.timings()
    print(os.environ.get("GS_PDBG", "0"), G, "project %.4f sort %.4f nvis %d" % (st["ms_project"], st["ms_sort"], st["n_vis"]), flush=True)
