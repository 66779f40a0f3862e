import os, sys, time
sys.path.insert(0, "gaussian-splatting-web_amd")
import gsplat_amd as gs
N, W, H = 6_100_000, 1920, 1080
aos = gs.synth_aos(N, 6, W, H); u = gs.bench_uniforms(W, H)
buf = gs.DeviceBuffer(H * W * 8)
with gs.Context([0] * 8) as gc:
    sc = gs.Scene(gc, aos, N, 16)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
    for _ in range(30):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    gc.sync()
    print("---- isolated", flush=True)
    sys.stderr.flush()
    for _ in range(20):
        gc.sync()
        a = time.perf_counter()
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        print("call %.1f us" % ((time.perf_counter() - a) * 1e6), flush=True)
    gc.sync()
