#!/usr/bin/env python3
"""Host time of one device-group frame against one row strip's.

A G-member group (gs_ctx_create with a device list; here the list repeats device 0, as a one-GPU
box allows) enqueues member g's strip from member g's own host thread.  This prints, for the bench
scene at 1920x1080 with f16 output and frames in flight:
  * strip s of G rendered by a plain context (opts.strip_index/strip_count): the host time of one
    gs_render_device call (p50 / p90 over F frames);
  * the G-member group: the host time of one gs_render_device call, and the frame rate.
The group's p50 over the single strip's p50 is the ratio the verdict asks to be <= 1.5.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402


def isolated_times(sc, ctx, u, W, H, buf, o, F):
    """Host time of one call with the GPU idle (a sync before each): the enqueue cost alone."""
    for _ in range(10):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync()
    per = []
    for _ in range(F):
        ctx.sync()
        a = time.perf_counter()
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        per.append(time.perf_counter() - a)
    ctx.sync()
    per.sort()
    return per[F // 2] * 1e6, per[int(F * 0.9)] * 1e6


def enqueue_times(sc, ctx, u, W, H, buf, o, F):
    for _ in range(20):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    ctx.sync()
    per = []
    t0 = time.perf_counter()
    for _ in range(F):
        a = time.perf_counter()
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        per.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    per.sort()
    return per[F // 2] * 1e6, per[int(F * 0.9)] * 1e6, (t1 - t0) / F * 1e6, (t2 - t0) / F * 1e6


def main():
    N, W, H = int(os.environ.get("N", 6_100_000)), 1920, 1080
    G, F = int(os.environ.get("G", "8")), int(os.environ.get("F", "300"))
    aos = gs.synth_aos(N, 6, W, H)
    u = gs.bench_uniforms(W, H)
    buf = gs.DeviceBuffer(H * W * 8)
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, N, 16)
        strip = []
        for s in (0, G // 2):
            o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, strip_index=s, strip_count=G)
            p50, p90, mean, tot = enqueue_times(sc, ctx, u, W, H, buf, o, F)
            i50, i90 = isolated_times(sc, ctx, u, W, H, buf, o, F // 2)
            strip.append(i50)
            print("strip %d/%d (one context): enqueue p50 %.1f us p90 %.1f mean %.1f; %.1f us/frame; "
                  "alone (GPU idle) p50 %.1f p90 %.1f" % (s, G, p50, p90, mean, tot, i50, i90), flush=True)
        sc.close()
    with gs.Context([0] * G) as gc:
        sc = gs.Scene(gc, aos, N, 16)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
        for rep in range(2):
            p50, p90, mean, tot = enqueue_times(sc, gc, u, W, H, buf, o, F)
            i50, i90 = isolated_times(sc, gc, u, W, H, buf, o, F // 2)
            print("group of %d (device 0 repeated, peer copies): call p50 %.1f us p90 %.1f mean %.1f; "
                  "%.1f us/frame (%.0f fps, all strips on one GPU); alone (GPU idle) p50 %.1f p90 %.1f" %
                  (G, p50, p90, mean, tot, 1e6 / tot, i50, i90), flush=True)
        print("ratio group / strip host time, GPU idle (p50) = %.2f%s" %
              (i50 / max(strip), " (GS_GROUP_SERIAL=1)" if os.environ.get("GS_GROUP_SERIAL") == "1" else ""),
              flush=True)
        sc.close()
    buf.free()


if __name__ == "__main__":
    main()
