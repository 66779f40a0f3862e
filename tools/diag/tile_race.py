#!/usr/bin/env python3
"""The open one-tile difference: cold view 3 of the bench scene rendered again and
again with forced chunk fractions; for every render whose image differs from the one-chunk render,
is the tile's sorted list (gs_debug_tile_lists) different too, or only the composite's result?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = 6_100_000, 1920, 1080
    TX, tile = (W + 15) // 16, 47 * 120 + 26
    aos = gs.synth_aos(N, 6, W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    u = gs.cold_uniforms(W, H, 3)
    o = dict(out_format=gs.GS_OUT_RGBA_F16)
    one = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, **o)).view(np.uint16)
    rg, en = sc.tile_lists()
    full = en[rg[tile, 0]:rg[tile, 1]].copy()
    print("one-chunk list of tile %d: %d entries, keys unique %s" % (tile, len(full), len(np.unique(full[:, 0])) == len(full)))
    # the one-chunk render itself, again and again: image and the tile's list against the first
    for rep in range(40):
        img = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, **o)).view(np.uint16)
        rg, en = sc.tile_lists()
        lst = en[rg[tile, 0]:rg[tile, 1]]
        d = int(np.any(img != one, axis=-1).sum())
        if d or not np.array_equal(lst, full):
            a = set(map(tuple, full.tolist()))
            b = set(map(tuple, lst.tolist()))
            order_ok = bool(np.all(np.diff(lst[:, 0].astype(np.int64)) > 0)) if len(lst) > 1 else True
            print("one-chunk rep %d: %d px differ; list %d vs %d entries, missing %d extra %d, ascending keys %s; "
                  "missing %s extra %s" % (rep, d, len(lst), len(full), len(a - b), len(b - a), order_ok,
                                           sorted(a - b)[:4], sorted(b - a)[:4]), flush=True)
    # forced splits: image only (tile lists exist for one-chunk frames only)
    for rep in range(3):
        for f in np.linspace(0.05, 0.95, 19):
            img = sc.render(u, W, H, gs.make_opts(chunk_fraction=float(f), **o)).view(np.uint16)
            d = np.any(img != one, axis=-1)
            if d.any():
                ys, xs = np.nonzero(d)
                print("rep %d f %.2f: %d px differ (rows %d-%d cols %d-%d)" % (rep, f, d.sum(), ys.min(), ys.max(), xs.min(), xs.max()), flush=True)
    print("done")


if __name__ == "__main__":
    main()
