#!/usr/bin/env python3
"""Per-tile list statistics of a one-chunk frame, for the long-list per-tile sort (ts_long):
list lengths, and per tile the 256-bucket split ts_long makes over [kmin, kmax] of the 64-bit
(depth key, index) keys -- how many entries land in buckets of more than Cap (TsBig: 2048), the
part ts_rounds sorts in O(L^2 / Cap).
    python tools/diag/tile_list_stats.py cfg4|sparse|bench"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402

CAP, BB = 2048, 8


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    if which == "cfg4":
        n, W, H = 50_000_000, 3840, 2160
        aos = gs.synth_aos(n, 50, W, H)
    elif which == "sparse":
        n, W, H = 6_100_000, 1920, 1080
        aos = gs.synth_aos_sparse(n, 6, W, H)
    else:
        n, W, H = 6_100_000, 1920, 1080
        aos = gs.synth_aos(n, 6, W, H)
    u = gs.bench_uniforms(W, H)
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, n, 16)
        del aos
        buf = gs.DeviceBuffer(W * H * 8)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=1.0)
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        rg, en = sc.tile_lists()
        buf.free()
        sc.close()
    L = (rg[:, 1] - rg[:, 0]).astype(np.int64)
    K = int(L.sum())
    print("%s: tiles %d entries %d mean %.0f" % (which, len(L), K, K / max(1, len(L))))
    for q in (50, 90, 99, 99.9, 100):
        print("  list length p%-5s %d" % (q, int(np.percentile(L, q))))
    long_ = np.nonzero(L > CAP)[0]
    print("  tiles > Cap: %d holding %d entries (%.1f %%)" % (len(long_), int(L[long_].sum()),
                                                             100.0 * L[long_].sum() / max(1, K)))
    heavy_tiles = heavy_entries = 0
    rounds_cost = 0  # entries re-read by ts_rounds: sum over heavy buckets of len * ceil(len / Cap)
    worst = []
    key64 = (en[:, 0].astype(np.uint64) << np.uint64(32)) | en[:, 1].astype(np.uint64)
    for t in long_:
        k = key64[rg[t, 0]:rg[t, 1]]
        kmin, kmax = int(k.min()), int(k.max())
        span = kmax - kmin
        sh = 0 if span == 0 else max(0, span.bit_length() - BB)
        b = ((k - np.uint64(kmin)) >> np.uint64(sh)).astype(np.int64)
        cnt = np.bincount(b, minlength=1 << BB)
        hv = cnt[cnt > CAP]
        if len(hv):
            heavy_tiles += 1
            heavy_entries += int(hv.sum())
            rounds_cost += int((hv * ((hv + CAP - 1) // CAP)).sum())
            worst.append((int(hv.max()), int(L[t]), int(t)))
    worst.sort(reverse=True)
    print("  tiles with a heavy bucket: %d; entries in heavy buckets %d; ts_rounds entry reads %d (%.2f x K)" %
          (heavy_tiles, heavy_entries, rounds_cost, rounds_cost / max(1, K)))
    print("  largest heavy buckets (bucket, list, tile):", worst[:8])
    # the 1024-thread shape's count ranking (lists <= 8192, 4096 buckets of equal width over the
    # tile's key range): element i = j * 1024 + t is ranked by a loop over its bucket, so a wave's
    # step j costs the largest bucket among its 64 lanes
    samp = long_[:: max(1, len(long_) // 400)]
    mean_b, mean_wmax = [], []
    for t in samp:
        k = key64[rg[t, 0]:rg[t, 1]]
        if len(k) > 8192:
            continue
        kmin, kmax = int(k.min()), int(k.max())
        span = kmax - kmin
        sh = 0 if span == 0 else max(0, span.bit_length() - 12)
        b = ((k - np.uint64(kmin)) >> np.uint64(sh)).astype(np.int64)
        cnt = np.bincount(b, minlength=4096)
        sz = cnt[b]
        mean_b.append(sz.mean())
        pad = np.zeros(8192, np.int64)
        pad[:len(sz)] = sz
        mean_wmax.append(pad.reshape(8, 16, 64).max(axis=2).sum() / (8 * 16))
    if mean_b:
        print("  1024-thread ranking over %d tiles: mean bucket of an element %.2f; mean wave-step cost %.2f" %
              (len(mean_b), float(np.mean(mean_b)), float(np.mean(mean_wmax))))
    # per-tile work if one workgroup streams ~ 6 reads per entry: the longest lists
    top = np.argsort(L)[::-1][:8]
    print("  longest lists (tile, L):", [(int(t), int(L[t])) for t in top])


if __name__ == "__main__":
    main()
