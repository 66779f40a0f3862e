#!/usr/bin/env python3
"""Composite blend counters on the bench frame (diagnostics build: `make -C
gaussian-splatting-web_amd diag`, run with GSPLAT_LIB=.../lib/libgsplat_diag.so).  Prints, per
frame: wave-level blends, live and hit pixel evaluations, blends with no hit, blends whose hits
are only in rows 0-7 or only in rows 8-15 of the wave's 8x16 half tile, and list entries."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    aos = gs.synth_aos(N, int(os.environ.get("SEED", 6)), W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    L = ctypes.CDLL(gs.LIB_PATH)
    import numpy as np
    buf = gs.DeviceBuffer(H * W * 8)
    G, g = int(os.environ.get("G", 1)), int(os.environ.get("STRIP", 0))
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=2, strip_index=g, strip_count=G,
                     list_split=int(os.environ.get("LIST_SPLIT", "0")))
    for _ in range(4):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync()
    ctx.timings_reset()
    F = 10
    for _ in range(F):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync()
    print("composite (HIP events) %.1f us per frame" % (ctx.timings()["ms_composite"] * 1e3))
    ntile = ((W + 15) // 16) * ((H + 15) // 16)
    if G > 1:  # the strip's tiles (local tile ids)
        from gsplat_amd.strips import strip_geometry
        ntile = ((W + 15) // 16) * (strip_geometry(H, g, G)[1] // 16)
        H = strip_geometry(H, g, G)[1]
    cn = np.zeros((16384, 2, 8), dtype=np.uint64)
    L.gs_diag_comp_counters(cn.ctypes.data_as(ctypes.c_void_p), 16384)
    ntile = min(ntile, 16384)
    c = cn[:ntile].sum(axis=(0, 1)).astype(np.float64)  # the last frame
    if os.environ.get("PHASE"):  # GS_COMP_PHASE build: per-wave shader cycles by phase
        ph = cn[:ntile, :, :5].astype(np.float64)
        tot = ph.sum(axis=2)
        names = ["first batch", "walks", "parks", "barriers", "gathers"]
        print("phase kcycles per wave (mean over waves): " +
              "  ".join("%s %.2f (%.0f%%)" % (nm, ph[:, :, i].mean() / 1e3, 100 * ph[:, :, i].sum() / tot.sum())
                        for i, nm in enumerate(names)) + "  total %.2f" % (tot.mean() / 1e3))
        c[0] = 0  # (the counters are not blend statistics)
    if c[0] > 0:
        px = 64 * 2 * c[0]
        print("wave blends/frame %.4g  pixel evals %.4g" % (c[0], px))
        print("live pixel evals %.4g (%.3f)  hits %.4g (%.3f of evals, %.3f of live)" %
              (c[1], c[1] / px, c[2], c[2] / px, c[2] / max(1, c[1])))
        print("blends with no hit %.3f  hits only rows 0-7 %.3f  only rows 8-15 %.3f" %
              (c[3] / c[0], c[4] / c[0], c[5] / c[0]))
        print("pixel evals inside the alpha disc (pair best) %.4g  list entries (tiles) %.4g" % (c[6], c[7]))
        # the two waves of a tile: steps of each; a wave done early waits at the batch barriers
        s = cn[:ntile, :, 0].astype(np.float64)
        print("wave steps: sum %.4g  sum of per-tile max x2 %.4g (idle share %.3f)  tiles with one wave "
              "at 0 steps %d" % (s.sum(), 2 * s.max(axis=1).sum(), 1 - s.sum() / max(1, 2 * s.max(axis=1).sum()),
                                 int(((s[:, 0] == 0) ^ (s[:, 1] == 0)).sum())))
    # per-tile wall-clock spans of the last frame (100 MHz clock)
    tm = np.zeros((16384, 3), dtype=np.uint64)
    L.gs_diag_comp_times(tm.ctypes.data_as(ctypes.c_void_p), 16384)
    tm = tm[:ntile]
    b = tm[:, 0].astype(np.int64) & 0xFFFFFFFFFF
    e = tm[:, 1].astype(np.int64) & 0xFFFFFFFFFF
    blends = (tm[:, 1] >> np.uint64(40)).astype(np.int64)
    hw = tm[:, 2].astype(np.int64) & 0xFFFFFFFF
    xcc = (tm[:, 2] >> np.uint64(32)).astype(np.int64) & 0xF
    cu = ((hw >> 8) & 15) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5)
    nl = (tm[:, 0] >> np.uint64(40)).astype(np.int64)
    t0 = b.min()
    b, e = (b - t0) / 100.0, (e - t0) / 100.0  # us
    d_ = e - b
    print("kernel span %.1f us; tile us: mean %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f" %
          (e.max(), d_.mean(), *np.percentile(d_, [50, 90, 99]), d_.max()))
    for x in range(8):
        m = xcc == x
        if m.any():
            cus, cnts = np.unique(cu[m], return_counts=True)
            print("  xcc %d: tiles %d busy-sum %.0f  first start %.1f last end %.1f  blends %d  CUs %d (tiles/CU %d..%d)" %
                  (x, m.sum(), d_[m].sum(), b[m].min(), e[m].max(), blends[m].sum(), len(cus), cnts.min(), cnts.max()))
    ts = np.linspace(0, e.max(), 21)
    act = [int(((b <= t) & (e > t)).sum()) for t in ts]
    print("active tiles over time:", act)
    print("list length: mean %.0f p50 %.0f p90 %.0f max %d; corr(len, dur) %.3f" %
          (nl.mean(), np.median(nl), np.percentile(nl, 90), nl.max(), np.corrcoef(nl, d_)[0, 1]))
    rows = (H + 15) // 16
    TXn = (W + 15) // 16
    print("per tile row: mean dur / mean len:",
          " ".join("%d:%.0f/%.0f" % (r, d_[r * TXn:(r + 1) * TXn].mean(), nl[r * TXn:(r + 1) * TXn].mean())
                   for r in range(0, rows, 3)))
    order = np.argsort(-e)[:10]
    TX = (W + 15) // 16
    print("last to finish (tile, tx, ty, start, dur):",
          [(int(t), int(t % TX), int(t // TX), round(float(b[t]), 1), round(float(d_[t]), 1)) for t in order])
    heavy = np.argsort(-d_)[:10]
    print("longest (tile, tx, ty, start, dur):",
          [(int(t), int(t % TX), int(t // TX), round(float(b[t]), 1), round(float(d_[t]), 1), int(nl[t])) for t in heavy])
    if os.environ.get("SAVE"):  # per-tile arrays for offline scheduling studies
        np.savez(os.environ["SAVE"], start=b, end=e, n=nl, blends=blends, xcc=xcc, cu=cu)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
