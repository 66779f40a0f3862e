#!/usr/bin/env python3
"""Chunk 1's composite per listed tile under the orbit camera (diagnostics build with
-DGS_CQ_TIME, GSPLAT_LIB=.../libgsplat_cqtime.so): per frame, the kernel's span, and each tile's
list length, start and duration (wall clock, 10 ns ticks), the longest tiles and when they started.

    GSPLAT_LIB=$PWD/gaussian-splatting-web_amd/lib/libgsplat_cqtime.so python tools/diag/cq_time.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, ROOT)
import gsplat_amd as gs  # noqa: E402
from bench import CONFIGS, orbit_uniforms  # noqa: E402


def main():
    N, W, H, seed = CONFIGS[int(os.environ.get("CONFIG", 3))]
    aos = gs.synth_aos(N, seed, W, H)
    L = ctypes.CDLL(gs.LIB_PATH)
    buf = gs.DeviceBuffer(H * W * 8)
    out = np.zeros((16384, 3), np.uint64)
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, N, 16)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
        for k in range(int(os.environ.get("FRAMES", 12))):
            sc.render_device(orbit_uniforms(W, H, k), W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            L.gs_diag_cq_times(out.ctypes.data_as(ctypes.c_void_p), 16384)
            m = out[:, 1] > 0
            if not m.any() or k < 4:
                continue
            t = out[m]
            t0 = t[:, 1].min()
            st, en = (t[:, 1] - t0) * 0.01, (t[:, 2] - t0) * 0.01   # us
            n = (t[:, 0] >> np.uint64(32)).astype(np.int64)
            d = en - st
            top = np.argsort(d)[::-1][:6]
            ph = np.zeros((16384, 4, 4), np.uint64)
            L.gs_diag_cq_phase(ph.ctypes.data_as(ctypes.c_void_p))
            tl = (t[top[0], 0] & np.uint64(0xFFFFFFFF)).astype(np.int64)
            w = ph[tl].astype(np.float64)   # the longest tile's waves: walk, park, barrier (shader cycles)
            print("  longest tile %d: per wave walk / park / barrier cycles %s" % (tl, [tuple(int(x) for x in w[q, 1:]) for q in range(4)]))
            print("frame %d: %d tiles, span %.1f us; duration p50 %.2f p90 %.2f max %.1f us; n p50 %d max %d; "
                  "longest (n, start, dur): %s; last start %.1f" %
                  (k, m.sum(), en.max(), np.percentile(d, 50), np.percentile(d, 90), d.max(), np.percentile(n, 50),
                   n.max(), [(int(n[i]), round(float(st[i]), 1), round(float(d[i]), 1)) for i in top], st.max()),
                  flush=True)
        sc.close()


if __name__ == "__main__":
    main()
