#!/usr/bin/env python3
"""Host readback rates through the C ABI (1920x1080, 6.1 M scene, f16 or f32 framebuffers):
copies alone (gs_readback_start/wait into page-locked arrays), frames alone (device-resident),
and frames with their readback pipelined two deep (the Node Renderer's host-readback loop)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = 6_100_000, 1920, 1080
    f16 = os.environ.get("F16", "1") == "1"
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    L, c = gs.lib(), ctx.handle
    nb = W * H * (8 if f16 else 16)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16 if f16 else gs.GS_OUT_RGBA_F32)
    devs = [ctypes.c_void_p(), ctypes.c_void_p()]
    for d in devs:
        assert L.gs_framebuffer_alloc(c, nb, ctypes.byref(d)) == 0
    hosts = [np.zeros(nb, np.uint8) for _ in range(3)]
    reg = os.environ.get("REG", "1") == "1"
    if reg:
        for h in hosts:
            assert L.gs_host_register(c, h.ctypes.data_as(ctypes.c_void_p), nb) == 0
    F = 100
    for _ in range(10):
        sc.render_device(u, W, H, devs[0].value, nb, None, o)
    ctx.sync()
    # copies alone
    t0 = time.perf_counter()
    tk = []
    for k in range(F):
        t = ctypes.c_uint32()
        assert L.gs_readback_start(c, devs[k % 2], hosts[k % 3].ctypes.data_as(ctypes.c_void_p), nb, ctypes.byref(t)) == 0
        tk.append(t.value)
        if k >= 1:
            L.gs_readback_wait(c, tk[k - 1])
    L.gs_readback_wait(c, tk[-1])
    cp = (time.perf_counter() - t0) / F
    # frames alone
    t0 = time.perf_counter()
    for k in range(F):
        sc.render_device(u, W, H, devs[k % 2].value, nb, None, o)
    ctx.sync()
    fr = (time.perf_counter() - t0) / F
    # frames + readback, two in flight
    t0 = time.perf_counter()
    tk = []
    for k in range(F):
        if k >= 2:
            L.gs_readback_wait(c, tk[k - 2])
        sc.render_device(u, W, H, devs[k % 2].value, nb, None, o)
        t = ctypes.c_uint32()
        assert L.gs_readback_start(c, devs[k % 2], hosts[k % 3].ctypes.data_as(ctypes.c_void_p), nb, ctypes.byref(t)) == 0
        tk.append(t.value)
    for t in tk[-2:]:
        L.gs_readback_wait(c, t)
    both = (time.perf_counter() - t0) / F
    print("%s %s: copy %.3f ms (%.1f GB/s)  frame %.3f ms  frame+readback %.3f ms (%.0f fps)" % (
        "f16" if f16 else "f32", "registered" if reg else "pageable", cp * 1e3, nb / cp / 1e9, fr * 1e3,
        both * 1e3, 1 / both), flush=True)
    if reg:
        for h in hosts:
            L.gs_host_unregister(c, h.ctypes.data_as(ctypes.c_void_p))
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
