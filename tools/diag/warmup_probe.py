#!/usr/bin/env python3
"""The first frames after a scene upload (and, REPS > 1, after IDLE seconds with the GPU idle) (the bench scene, frames in flight as in bench.py): the
host time of each frame's call and, every few frames, the mean frame time since the last report
with the chunk controller's state (chunk fraction, chunk-0 entries, seeded frames).

Env: N, W, H, SEED, FRAMES, EVERY."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), int(os.environ.get("W", 1920)), int(os.environ.get("H", 1080))
    F, E = int(os.environ.get("FRAMES", 60)), int(os.environ.get("EVERY", 5))
    aos = gs.synth_aos(N, int(os.environ.get("SEED", 6)), W, H)
    u = gs.bench_uniforms(W, H)
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, N, 16)
    buf = gs.DeviceBuffer(H * W * 8)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
    for rep in range(int(os.environ.get("REPS", 1))):
        if rep:
            time.sleep(float(os.environ.get("IDLE", 2.0)))  # the GPU idle between repeats
            print("-- after %.1f s idle" % float(os.environ.get("IDLE", 2.0)), flush=True)
        run(ctx, sc, u, W, H, buf, o, F, E)


def run(ctx, sc, u, W, H, buf, o, F, E):
    ctx.sync()
    ctx.timings_reset()
    t0 = time.perf_counter()
    for i in range(1, F + 1):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        if i % E == 0:
            ctx.sync()
            t = time.perf_counter()
            st = ctx.timings()
            print("frames %3d-%3d: %.3f ms/frame  chunk_fraction %.3f k_chunk0 %d seeded %d chunked %d" %
                  (i - E + 1, i, (t - t0) / E * 1e3, st["chunk_fraction"], st["k_chunk0"], st["frames_seeded"],
                   st["frames_chunked"]), flush=True)
            ctx.timings_reset()
            t0 = time.perf_counter()


if __name__ == "__main__":
    main()
