#!/usr/bin/env python3
"""Moving-camera diagnostics: frame times of the bench scene under bench.py's orbit camera with
the adaptive chunk split, with one chunk forced, and the stage times of orbit frames (timing=1)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
sys.path.insert(0, ROOT)
import gsplat_amd as gs  # noqa: E402
from bench import CONFIGS, orbit_uniforms  # noqa: E402


def main():
    cfg = int(os.environ.get("CONFIG", "3"))
    N, W, H, seed = CONFIGS[cfg]
    steps = int(os.environ.get("STEPS", "60"))
    aos = gs.synth_aos(N, seed, W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    buf = gs.DeviceBuffer(H * W * 8)
    uo = [orbit_uniforms(W, H, k) for k in range(steps)]
    modes = [("adaptive", 0.0, 0), ("one_chunk", 1.0, 0), ("adaptive_staged", 0.0, 1), ("one_chunk_staged", 1.0, 1)]
    only = os.environ.get("MODE")  # one mode only (e.g. under rocprofv3)
    for name, cf, timing in [m for m in modes if not only or m[0] == only]:
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=cf, timing=timing,
                         list_split=int(os.environ.get("LIST_SPLIT", "0")))
        for k in range(5):
            sc.render_device(uo[k], W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        ctx.timings_reset()
        t0 = time.perf_counter()
        for k in range(steps):
            sc.render_device(uo[k], W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        ms = (time.perf_counter() - t0) / steps * 1e3
        st = ctx.timings()
        print("%-18s %.3f ms/frame  %s" % (name, ms, " ".join("%s=%.4g" % (k, v) for k, v in st.items()
                                                               if k.startswith("ms_") or k in ("tiles_unsaturated",
                                                               "k_chunk0", "k_chunk1", "chunk_fraction", "n_vis"))),
              flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
