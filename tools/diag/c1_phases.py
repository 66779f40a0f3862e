#!/usr/bin/env python3
"""k_chunk1 phase times (diagnostics build: `make -C gaussian-splatting-web_amd diag
DIAGFLAGS=-DGS_C1_TIME`, run with GSPLAT_LIB=.../lib/libgsplat_diag.so): workgroup 0's wall clock
after each grid barrier, averaged over the frames with chunk-1 work, for the static bench camera
and bench.py's orbit camera."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, ROOT)
import gsplat_amd as gs  # noqa: E402
from bench import CONFIGS, orbit_uniforms  # noqa: E402

PHASES = ["unsat rows", "partition list", "records", "bin count", "col scan", "tile scan", "emit",
          "tile sort", "composite"]


def main():
    N, W, H, seed = CONFIGS[int(os.environ.get("CONFIG", "3"))]
    aos = gs.synth_aos(N, seed, W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    L = ctypes.CDLL(gs.LIB_PATH)
    buf = gs.DeviceBuffer(H * W * 8)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
    for name, cams in (("static", [gs.bench_uniforms(W, H)] * 60), ("orbit", [orbit_uniforms(W, H, k) for k in range(60)])):
        acc, nf, last = np.zeros(9), 0, None
        for k, u in enumerate(cams):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            t = np.zeros(16, np.uint64)
            L.gs_diag_c1_times(t.ctypes.data_as(ctypes.c_void_p))
            if k >= 5 and last is not None and t[0] != last[0]:
                acc += np.diff(t[:10].astype(np.float64)) * 0.01  # 100 MHz -> us
                nf += 1
            last = t.copy()
        st = ctx.timings()
        print("%s: %d frames with chunk-1 work, last frame tiles_unsaturated %d k_chunk1 %d" %
              (name, nf, st["tiles_unsaturated"], st["k_chunk1"]))
        if nf:
            print("   " + "  ".join("%s %.1f" % (p, v / nf) for p, v in zip(PHASES, acc)) + "  total %.1f us" % (acc.sum() / nf))
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
