#!/usr/bin/env python3
"""Per-strip stage times and frame statistics (gs_opts.timing = 1: every stage between events,
frames serialised) for G row strips of one scene, against the full frame (G = 1).

Env: N, W, H, SEED (scene; 50 M / 3840x2160 / seed 50 is config 4), GS (comma list of G),
FRAMES (timed frames per strip)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    aos = gs.synth_aos(N, int(os.environ.get("SEED", 6)), W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    F = int(os.environ.get("FRAMES", 20))
    buf = gs.DeviceBuffer(H * W * 8)
    keys = ("ms_total", "ms_project", "ms_bin", "ms_tile_sort", "ms_composite", "ms_other")
    for G in [int(x) for x in os.environ.get("GS", "1,8").split(",")]:
        for g in range(G):
            sc = gs.Scene(ctx, aos, N, 16)  # a context of its own per strip, as on G GPUs
            o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, timing=1, strip_index=g, strip_count=G)
            for _ in range(10):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            ctx.timings_reset()
            for _ in range(F):
                sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
            ctx.sync()
            t = ctx.timings()
            print("G=%d strip %d  " % (G, g) + " ".join("%s %.1f" % (k[3:], t[k] * 1e3) for k in keys) +
                  "  | n_vis %d k_total %d k0 %d k1 %d chunk %.3f unsat %d" %
                  (t["n_vis"], t["k_total"], t["k_chunk0"], t["k_chunk1"], t["chunk_fraction"],
                   t["tiles_unsaturated"]), flush=True)
            sc.close()


if __name__ == "__main__":
    main()
