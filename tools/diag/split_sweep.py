#!/usr/bin/env python3
"""Chunk-split sweep: render one view of the bench scene with forced chunk fractions (and after a
history of other views) and compare every image bit for bit with the one-chunk render; prints the
splits that differ.   Env: VIEW (cold view index, default 3), N, W, H, SEED."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    v = int(os.environ.get("VIEW", 3))
    aos = gs.synth_aos(N, int(os.environ.get("SEED", 6)), W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    u = gs.cold_uniforms(W, H, v)
    o16 = dict(out_format=gs.GS_OUT_RGBA_F16)
    one = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, **o16)).view(np.uint16)
    bad = 0
    for f in np.linspace(0.01, 0.99, 99):
        img = sc.render(u, W, H, gs.make_opts(chunk_fraction=float(f), timing=1, **o16)).view(np.uint16)
        st = ctx.timings()
        if not np.array_equal(img, one):
            d = np.any(img != one, axis=-1)
            ys, xs = np.nonzero(d)
            bad += 1
            print("fraction %.2f: %d pixels differ, rows %d-%d cols %d-%d; k_chunk0 %d k_chunk1 %d unsat %d" %
                  (f, d.sum(), ys.min(), ys.max(), xs.min(), xs.max(), st["k_chunk0"], st["k_chunk1"],
                   st["tiles_unsaturated"]), flush=True)
    # adaptive frames after the other cold views (the test's sequence), each against one chunk
    views = [gs.cold_uniforms(W, H, k) for k in range(12)]
    ones = {k: sc.render(views[k], W, H, gs.make_opts(chunk_fraction=1.0, **o16)).view(np.uint16) for k in range(4)}
    for rep in range(int(os.environ.get("REPS", 5))):
        for k in range(12):
            img = sc.render(views[k], W, H, gs.make_opts(**o16)).view(np.uint16)
            if not np.array_equal(img, ones[k % 4]):
                bad += 1
                print("adaptive rep %d frame %d (view %d) differs: %d pixels" % (rep, k, k % 4, np.any(img != ones[k % 4], axis=-1).sum()), flush=True)
    print("sweep done, %d differing renders" % bad)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
