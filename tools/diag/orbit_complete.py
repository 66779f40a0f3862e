#!/usr/bin/env python3
"""Moving-camera diagnostic: which tiles never saturate (the one-chunk image's alpha), and how
well the tiles that never saturated one or two frames earlier (dilated by r tiles) predict them.
A tile predicted "complete" would take every splat in chunk 0; a miss would still need chunk 1.

    python tools/diag/orbit_complete.py          (CONFIG=3 STEPS=60 by default)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, ROOT)
import gsplat_amd as gs  # noqa: E402
from bench import CONFIGS, orbit_uniforms  # noqa: E402


def dilate(m, r):
    """Tiles within r tiles (Chebyshev) of a set tile."""
    H, W = m.shape
    p = np.zeros((H + 2 * r, W + 2 * r), bool)
    p[r:r + H, r:r + W] = m
    out = np.zeros_like(m)
    for dy in range(2 * r + 1):
        for dx in range(2 * r + 1):
            out |= p[dy:dy + H, dx:dx + W]
    return out


def main():
    cfg = int(os.environ.get("CONFIG", "3"))
    N, W, H, seed = CONFIGS[cfg]
    steps = int(os.environ.get("STEPS", "60"))
    aos = gs.synth_aos(N, seed, W, H)
    TX, TY = (W + 15) // 16, (H + 15) // 16
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, N, 16)
        o1 = gs.make_opts(chunk_fraction=1.0)
        ns = []
        for k in range(steps):
            img = sc.render(orbit_uniforms(W, H, k), W, H, o1)
            a = img[..., 3].astype(np.float64)
            pad = np.zeros((TY * 16, TX * 16))
            pad[:H, :W] = 1.0 - a                       # transmittance; padding counts as saturated
            t = pad.reshape(TY, 16, TX, 16).max(axis=(1, 3))
            ns.append(t >= 1e-4)
        # the adaptive orbit's chunk-1 tiles (mean per frame)
        oa = gs.make_opts()
        for k in range(steps):
            sc.render(orbit_uniforms(W, H, k), W, H, oa)
        ctx.timings_reset()
        for k in range(steps):
            sc.render(orbit_uniforms(W, H, k), W, H, oa)
        st = ctx.timings()
        print("config %d %dx%d: %d tiles; never-saturating tiles per frame: mean %.0f min %d max %d" %
              (cfg, W, H, TX * TY, np.mean([m.sum() for m in ns]), min(m.sum() for m in ns), max(m.sum() for m in ns)))
        print("adaptive orbit: " + " ".join("%s=%.4g" % (k, v) for k, v in st.items()
                                            if k in ("tiles_unsaturated", "k_chunk0", "k_chunk1", "chunk_fraction")))
        for lag in (1, 2):
            for r in (0, 1, 2, 3, 4):
                miss, extra = [], []
                for k in range(lag, steps):
                    pred = dilate(ns[k - lag], r)
                    miss.append(int((ns[k] & ~pred).sum()))
                    extra.append(int((pred & ~ns[k]).sum()))
                print("lag %d dilate %d: missed never-saturating tiles per frame mean %.1f max %d; "
                      "predicted but saturating mean %.1f max %d" %
                      (lag, r, np.mean(miss), max(miss), np.mean(extra), max(extra)))
        sc.close()


if __name__ == "__main__":
    main()
