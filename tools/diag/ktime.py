#!/usr/bin/env python3
"""Per-workgroup wall-clock stamps of k_cull and k_project (diagnostics build with -DGS_KTIME,
selected with GSPLAT_LIB) on the bench scene: the full frame and strip 1 of 8, frames serialised.
Prints, per kernel: workgroups, span, start spread, entry -> first item and first item -> exit
percentiles, items per workgroup."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402
from gsplat_amd.strips import strip_geometry  # noqa: E402


def report(name, a):
    t = a.astype(np.int64) & 0xFFFFFFFFFF
    x = (a >> np.uint64(40)).astype(np.int64)
    ok = (t[:, 0] > 0) & (t[:, 2] > 0)
    t, x = t[ok], x[ok]
    if not len(t):
        print(name, "no stamps")
        return
    t0 = t[:, 0].min()
    s, m, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0
    busy = x[:, 2] > 0
    pc = lambda v: "p10 %.1f p50 %.1f p90 %.1f max %.1f" % (*np.percentile(v, [10, 50, 90]), v.max())
    print("%s: workgroups %d (with items %d), span %.1f us; start %s" % (name, len(t), busy.sum(), e.max(), pc(s)))
    if busy.any():
        print("   entry->first item %s" % pc((m - s)[busy]))
        print("   first item->exit  %s" % pc((e - m)[busy]))
        if a.shape[1] > 3 and (t[:, 3] > 0).any():
            for k, lab in ((3, "geometry in (first unit)"), (4, "projected"), (5, "SH in")):
                v = (t[:, k] - t0) / 100.0
                okk = busy & (t[:, k] > 0)
                if okk.any():
                    print("   entry->%s %s" % (lab, pc((v - s)[okk])))
        print("   items/wg %s ; idle wgs exit %s" % (pc(x[busy, 2].astype(float)), pc((e - s)[~busy]) if (~busy).any() else "-"))


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), 1920, 1080
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    L = ctypes.CDLL(gs.LIB_PATH)
    for G, g in ((1, 0), (8, 1)):
        rows = strip_geometry(H, g, G)[1]
        buf = gs.DeviceBuffer((rows if G > 1 else H) * W * 16)
        o = gs.make_opts(strip_index=g, strip_count=G, timing=1, out_format=gs.GS_OUT_RGBA_F16)
        for _ in range(10):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        kt = np.zeros((2, 8192, 6), dtype=np.uint64)
        L.gs_diag_kt(kt.ctypes.data_as(ctypes.c_void_p))
        print("== G=%d strip %d" % (G, g))
        fe = np.zeros(8, dtype=np.uint64)
        L.gs_diag_fe(fe.ctypes.data_as(ctypes.c_void_p))
        f = fe.astype(np.int64)
        print("frame end (us from k_chunk1 entry): start %.2f  shards in %.2f  reduced %.2f  host copy done %.2f  end %.2f" %
              tuple((f[k] - f[5]) / 100.0 for k in range(5)), " ctl word %.2f shard word %.2f" % ((f[6] - f[5]) / 100.0, (f[7] - f[5]) / 100.0))
        report("k_cull", kt[0])
        report("k_project", kt[1])
        # clear for the next configuration: render with stamps zeroed is not possible from here,
        # so stamps of workgroups that did not run in this frame keep old values (filtered by start)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
