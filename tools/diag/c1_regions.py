#!/usr/bin/env python3
"""How much shorter would a long tile's composite chain be with finer per-region lists?  For the
longest one-chunk tile lists of orbit frames (the tiles chunk 1 walks thousands of entries in), the
number of splats whose pixel box reaches each 8x8 quarter (k_composite_q's per-wave lists) and each
4x4 region, over the deepest `DEEP` share of each list (the chunk-1 part).

    python tools/diag/c1_regions.py        (FRAMES="3 6 40", TOP=20, DEEP=0.7)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, ROOT)
import gsplat_amd as gs  # noqa: E402
from bench import CONFIGS, orbit_uniforms  # noqa: E402


def counts(x0, x1, y0, y1, tx0, ty0, cell):
    """Splats (pixel boxes) reaching each cell x cell region of the tile at (tx0, ty0)."""
    n = 16 // cell
    out = np.zeros((n, n), np.int64)
    for ry in range(n):
        for rx in range(n):
            ax, ay = tx0 + rx * cell, ty0 + ry * cell
            out[ry, rx] = ((x0 <= ax + cell - 1) & (x1 >= ax) & (y0 <= ay + cell - 1) & (y1 >= ay)).sum()
    return out


def main():
    N, W, H, seed = CONFIGS[3]
    top, deep = int(os.environ.get("TOP", 20)), float(os.environ.get("DEEP", 0.7))
    aos = gs.synth_aos(N, seed, W, H)
    TX = (W + 15) // 16
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, N, 16)
        o1 = gs.make_opts(chunk_fraction=1.0)
        for k in (int(v) for v in os.environ.get("FRAMES", "3 6 40").split()):
            sc.render(orbit_uniforms(W, H, k), W, H, o1)
            rg, en = sc.tile_lists()
            rec = sc.last_records()
            bx = rec[:, 14].view(np.uint32)
            by = rec[:, 15].view(np.uint32)
            ln = rg[:, 1] - rg[:, 0]
            tiles = np.argsort(ln)[::-1][:top]
            rq, rr, rl = [], [], []
            for t in tiles:
                b, e = int(rg[t, 0]), int(rg[t, 1])
                b = b + int((e - b) * (1.0 - deep))
                g = en[b:e, 1]
                x0, x1, y0, y1 = bx[g] & 0xFFFF, bx[g] >> 16, by[g] & 0xFFFF, by[g] >> 16
                tx0, ty0 = (t % TX) * 16, (t // TX) * 16
                q = counts(x0, x1, y0, y1, tx0, ty0, 8)
                r = counts(x0, x1, y0, y1, tx0, ty0, 4)
                rl.append(e - b)
                rq.append(q.max())
                rr.append(r.max())
            rl, rq, rr = np.array(rl), np.array(rq), np.array(rr)
            print("frame %d: top %d tiles, deep part %d..%d entries; chain 8x8 quarters / list %.3f, 4x4 regions / "
                  "list %.3f, 4x4 / 8x8 %.3f (max tile: list %d, quarter %d, region %d)" %
                  (k, top, rl.min(), rl.max(), (rq / rl).mean(), (rr / rl).mean(), (rr / rq).mean(), rl.max(),
                   rq[rl.argmax()], rr[rl.argmax()]), flush=True)
        sc.close()


if __name__ == "__main__":
    main()
