#!/usr/bin/env python3
"""Composite tile order study (diagnostics build, GSPLAT_LIB=.../libgsplat_diag.so): per-tile
wall-clock durations and blend counts of two consecutive bench frames; how well frame f predicts
frame f+1; and a list-scheduling simulation of the XCD bands (320 workgroup slots per XCD) under
the current order, longest-first by the previous frame's blends, and light-last."""
import ctypes
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def grab(L, ntile):
    tm = np.zeros((16384, 3), dtype=np.uint64)
    L.gs_diag_comp_times(tm.ctypes.data_as(ctypes.c_void_p), 16384)
    tm = tm[:ntile]
    b = (tm[:, 0].astype(np.int64) & 0xFFFFFFFFFF)
    e = (tm[:, 1].astype(np.int64) & 0xFFFFFFFFFF)
    blends = (tm[:, 1] >> np.uint64(40)).astype(np.int64)
    return b, e, blends


def simulate(order, dur, slots):
    """List scheduling: tiles start in `order` on the first free slot; returns the makespan."""
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for t in order:
        s = heapq.heappop(h)
        f = s + dur[t]
        end = max(end, f)
        heapq.heappush(h, f)
    return end


def main():
    N, W, H = 6_100_000, 1920, 1080
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    L = ctypes.CDLL(gs.LIB_PATH)
    buf = gs.DeviceBuffer(H * W * 8)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
    ntile = ((W + 15) // 16) * ((H + 15) // 16)
    frames = []
    for k in range(12):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        if k >= 9:
            frames.append(grab(L, ntile))
    (b0, e0, n0), (b1, e1, n1) = frames[0], frames[1]
    d0, d1 = (e0 - b0) / 100.0, (e1 - b1) / 100.0
    print("tile us: mean %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f" % (d1.mean(), *np.percentile(d1, [10, 50, 90]), d1.max()))
    print("corr(dur f, dur f+1) %.3f  corr(blends f, dur f+1) %.3f  corr(blends f, blends f+1) %.3f" %
          (np.corrcoef(d0, d1)[0, 1], np.corrcoef(n0, d1)[0, 1], np.corrcoef(n0, n1)[0, 1]))
    span = (e1.max() - b1.min()) / 100.0
    print("measured span %.1f us" % span)
    per = (ntile + 7) // 8
    slots = 320
    res = {}
    for name in ("measured_start", "raster", "lpt_prev_blends", "lpt_prev_dur", "light_last", "oracle_lpt"):
        mk = []
        for x in range(8):
            band = np.arange(x * per, min(ntile, (x + 1) * per))
            if name == "measured_start":
                order = band[np.argsort(b1[band])]
            elif name == "raster":
                order = band
            elif name == "lpt_prev_blends":
                order = band[np.argsort(-n0[band], kind="stable")]
            elif name == "lpt_prev_dur":
                order = band[np.argsort(-d0[band], kind="stable")]
            elif name == "light_last":
                m = d0[band].mean()
                light = d0[band] < 0.8 * m
                order = np.concatenate([band[~light], band[light]])
            else:
                order = band[np.argsort(-d1[band], kind="stable")]
            mk.append(simulate(order, d1, slots))
        res[name] = max(mk)
    print("simulated makespan (us, slowest XCD):", {k: round(v, 1) for k, v in res.items()})
    print("lower bound (mean load per slot): %.1f" % max(d1[x * per:(x + 1) * per].sum() / slots for x in range(8)))
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
