#!/usr/bin/env python3
"""Round-6 A/B of the tile-list bug: the bench scene's cold views (view 3 is the one
round 5 caught), each rendered as one chunk again and again, with the binning invariant
(kErrBinning: k_bin_emit's entries against k_bin_count's checksums) and the host's structural
check of every tile list (gs_debug_tile_list_check) after each render, plus the round-5 tile's
list (tile column 26, row 47: 1791 entries before 2071db7, 1792 with the bug).

Run it once per library (GSPLAT_LIB selects one): the committed build and the diagnostics build
made with -DGS_BIN_CONTRACT_FAST (the binning's ellipse math compiled with contraction as in
round 5).  Prints one line per render that is not clean and a summary line."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    N, W, H = 6_100_000, 1920, 1080
    tile = 47 * ((W + 15) // 16) + 26
    print("lib", os.path.basename(gs.LIB_PATH), flush=True)
    aos = gs.synth_aos(N, 6, W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=1.0)
    bad_renders = errors = 0
    lens = {}
    for view in (3, 0, 1, 2):
        u = gs.cold_uniforms(W, H, view)
        first = None
        for rep in range(reps):
            try:
                img = sc.render(u, W, H, o).view(np.uint16)
            except gs.GsError as e:
                errors += 1
                print("view %d rep %d: %s" % (view, rep, e), flush=True)
                continue
            chk = sc.tile_list_check()
            rg, en = sc.tile_lists()
            lst = en[rg[tile, 0]:rg[tile, 1]]
            lens.setdefault(view, set()).add(len(lst))
            same = first is None or np.array_equal(img, first)
            if first is None:
                first = img
            if chk["dup"] or chk["order"] or chk["gaps"] or chk["bad"] or not same:
                bad_renders += 1
                print("view %d rep %d: %s, image %s, tile %d list %d entries" %
                      (view, rep, chk, "same" if same else "DIFFERS", tile, len(lst)), flush=True)
        print("view %d done: tile %d list lengths %s" % (view, tile, sorted(lens.get(view, ()))), flush=True)
    print("SUMMARY lib %s renders %d kErrBinning %d structural/image failures %d" %
          (os.path.basename(gs.LIB_PATH), 4 * reps, errors, bad_renders), flush=True)


if __name__ == "__main__":
    main()
