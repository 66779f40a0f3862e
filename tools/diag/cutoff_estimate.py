#!/usr/bin/env python3
"""CPU estimate (oracle): how many chunk-0 (tile, splat) entries a per-tile depth cutoff would
drop.  Per 16x16 tile: its list in the reference's depth order (quad-box tiles, as or_tile_stats),
the entry at which every pixel saturates (T < t_min), the global chunk threshold the controller
sets (1.15 x the deepest saturation depth), and the entries below a per-tile cutoff of m x the
tile's own saturation depth.  python tools/diag/cutoff_estimate.py [N] [W] [H]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gsplat_amd as gs  # noqa: E402
import oracle_py as orc  # noqa: E402


def key_to_depth(k):
    k = k.astype(np.uint32)
    neg = (k & 0x80000000) == 0
    fu = np.where(neg, k ^ 0x80000001, k ^ 0x80000000).astype(np.uint32)
    return np.abs(fu.view(np.float32))


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 6_100_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    sp = orc.project(aos.view(np.uint8), N, 16, u, W, H)
    vis = np.nonzero(sp["visible"] == 1)[0].astype(np.uint32)
    _, order = orc.stable_sort_pairs(sp["key"][vis], vis)
    TX, TY = (W + 15) // 16, (H + 15) // 16
    ln = np.zeros(TX * TY, np.uint32)
    used = np.zeros(TX * TY, np.uint32)
    qp = ctypes.c_uint64()
    L = orc.lib()
    L.or_tile_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.or_tile_stats(sp.ctypes.data, order.ctypes.data, order.size, W, H, 1e-4, ln.ctypes.data, used.ctypes.data,
                    ctypes.byref(qp))
    # entries (tile, key) in depth order, tile-major
    s = sp[order]
    r = s["rect"]
    x0, y0, x1, y1 = r[:, 0] // 16, r[:, 1] // 16, r[:, 2] // 16, r[:, 3] // 16
    nt = (x1 - x0 + 1) * (y1 - y0 + 1)
    rep = np.repeat(np.arange(s.size), nt)
    off = np.arange(rep.size) - np.repeat(np.cumsum(nt) - nt, nt)
    w = (x1 - x0 + 1)[rep]
    tile = (y0[rep] + off // w) * TX + (x0[rep] + off % w)
    key = s["key"][rep]
    o = np.argsort(tile, kind="stable")  # keeps depth order within a tile
    tile, key = tile[o], key[o]
    start = np.searchsorted(tile, np.arange(TX * TY))
    sat = used < ln  # saturated before the list ended
    satkey = np.full(TX * TY, 0xFFFFFFFF, np.uint32)
    idx = start[sat] + used[sat] - 1
    satkey[sat] = key[idx]
    dsat = key_to_depth(satkey[sat])
    T = 1.15 * dsat.max()
    dkey = key_to_depth(key)
    c0 = int((dkey < T).sum())
    print("N %d  %dx%d  visible %d  entries (quad-box tiles) %d  tiles saturated %d / %d" %
          (N, W, H, vis.size, key.size, int(sat.sum()), TX * TY))
    print("global T (1.15 x deepest saturation depth %.3f): chunk-0 entries %d, used (blended) entries %d" %
          (dsat.max(), c0, int(used.sum())))
    for m in (1.02, 1.05, 1.1, 1.15, 1.3):
        cut = np.full(TX * TY, T, np.float64)
        cut[sat] = np.minimum(m * key_to_depth(satkey[sat]), T)
        n = int((dkey < cut[tile]).sum())
        print("per-tile cutoff %.2f x own saturation depth: entries %d (%.1f %% of chunk 0)" % (m, n, 100.0 * n / c0))


if __name__ == "__main__":
    main()
