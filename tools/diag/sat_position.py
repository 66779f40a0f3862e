#!/usr/bin/env python3
"""How much of a chunked frame's chunk-0 tile lists does the composite use?  Per tile of the bench
view: the position at which the tile saturates in its one-chunk list (every pixel's T < t_min,
alpha and box test as k_composite, evaluated here in numpy from the frame's slot records), against
the tile's chunk-0 entries of the steady-state chunked frame (the entries with key < the chunk
threshold, found as the key that leaves the frame's measured chunk-0 entry count).  The difference
is what per-tile chunk thresholds would stop binning, sorting and gathering."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = 6_100_000, 1920, 1080
    view = sys.argv[1] if len(sys.argv) > 1 else "bench"
    TX = (W + 15) // 16
    aos = gs.synth_aos(N, 6, W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    u = gs.bench_uniforms(W, H) if view == "bench" else gs.orbit_uniforms(W, H, int(view))
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
    for _ in range(20):  # the controller's steady state
        sc.render(u, W, H, o)
    ctx.timings_reset()
    sc.render(u, W, H, o)
    st = ctx.timings()
    k0 = st["k_chunk0"]
    sc.render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=1.0))
    rg, en = sc.tile_lists()
    sl = sc.last_slots()
    rec = np.zeros((N, 7), np.float32)
    rec[sl["index"]] = np.concatenate([sl["r0"], sl["r1"][:, :3]], axis=1)
    keys = en[:, 0].astype(np.uint64)
    T0 = np.sort(keys)[min(k0, len(keys) - 1)]
    L = 2.0 * np.sqrt(np.log2(np.e))
    tot0 = tot_sat = tot_all = 0
    frac = []
    ys, xs = np.mgrid[0:16, 0:16]
    for t in range(len(rg)):
        b, e = int(rg[t, 0]), int(rg[t, 1])
        if e <= b:
            continue
        tx, ty = t % TX, t // TX
        px = (xs + tx * 16 + 0.5).ravel().astype(np.float32)
        py = (ys + ty * 16 + 0.5).ravel().astype(np.float32)
        r = rec[en[b:e, 1]]
        dx = px[None, :] - r[:, 0:1]
        dy = py[None, :] - r[:, 1:2]
        uu = dx * r[:, 2:3] + dy * r[:, 3:4]
        vv = dx * r[:, 4:5] + dy * r[:, 5:6]
        a = np.exp2(r[:, 6:7] - (uu * uu + vv * vv))
        a = np.where((np.maximum(np.abs(uu), np.abs(vv)) <= L) & (a >= 1 / 255), a, 0.0)
        Tc = np.cumprod(1.0 - a, axis=0)
        done = np.all(Tc < 1e-4, axis=1)
        s = int(np.argmax(done)) + 1 if done.any() else e - b
        c0 = int((keys[b:e] < T0).sum())
        tot0 += c0
        tot_sat += min(s, c0)
        tot_all += e - b
        frac.append(s / max(c0, 1))
    frac = np.array(frac)
    print("view %s: chunk-0 entries %d (measured k_chunk0 %d), one-chunk entries %d" % (view, tot0, k0, tot_all))
    print("entries up to each tile's saturation point (within chunk 0): %d = %.3f of chunk 0" % (tot_sat, tot_sat / tot0))
    print("saturation position / chunk-0 list: p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(frac, [10, 50, 90, 100])))


if __name__ == "__main__":
    main()
