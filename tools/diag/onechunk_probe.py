#!/usr/bin/env python3
"""One-chunk frames (every visible splat binned, sorted and composited: chunk_fraction = 1) of a
configuration, each waited for, for a rocprofv3 kernel trace of the non-saturated path:
    python tools/diag/onechunk_probe.py cfg4|sparse|bench [frames]
cfg4 = 50 M at 3840x2160 (seed 50); sparse = bench.py's sparse scene (6.1 M, opacity logit ~ N(-4, 2))
at 1920x1080; bench = the bench scene at 1920x1080.  Prints the mean wall time per frame."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    if which == "cfg4":
        n, W, H, aos = 50_000_000, 3840, 2160, None
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
        t = []
        for _ in range(frames):
            t0 = time.perf_counter()
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            t.append(time.perf_counter() - t0)
        st = ctx.timings()
        print("%s one-chunk frame: mean %.3f ms min %.3f ms; n_vis %d k_binned %d; longest list %d, "
              "tiles to the long-list pass %d" % (which, 1e3 * sum(t) / len(t), 1e3 * min(t), st["n_vis"],
                                                  st["k_entries"], st["list_max"], st["tiles_long"]), flush=True)
        buf.free()
        sc.close()


if __name__ == "__main__":
    main()
