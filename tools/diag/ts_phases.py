#!/usr/bin/env python3
"""Phase split of the long-list per-tile sort (ts_long) in one-chunk frames.  Needs the
diagnostics library built with the phase timers:
    make -C gaussian-splatting-web_amd diag DIAGFLAGS=-DGS_TS_TIME
    GSPLAT_LIB=gaussian-splatting-web_amd/lib/libgsplat_diag.so python tools/diag/ts_phases.py cfg4|sparse
Prints, per phase, the cycles (s_memtime) summed over the tiles as a share of the total."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402

PHASES = ("minmax", "histogram", "scan", "scatter", "rounds", "heavy buckets")
# the 1024-thread shape (k_tile_sort_huge) on lists of one round
PHASES_HUGE = ("load + gather", "minmax", "count", "scan + scatter", "rank + write", "-")


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if which == "cfg4":
        n, W, H = 50_000_000, 3840, 2160
        aos = gs.synth_aos(n, 50, W, H)
    else:
        n, W, H = 6_100_000, 1920, 1080
        aos = gs.synth_aos_sparse(n, 6, W, H) if which == "sparse" else gs.synth_aos(n, 6, W, H)
    L = gs.lib()
    L.gs_diag_ts_time.argtypes = [ctypes.c_void_p]
    cnt = (ctypes.c_ulonglong * 8)()
    u = gs.bench_uniforms(W, H)
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, n, 16)
        del aos
        buf = gs.DeviceBuffer(W * H * 8)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=1.0)
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        L.gs_diag_ts_time(cnt)
        for _ in range(frames):
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        ctx.sync()
        assert L.gs_diag_ts_time(cnt) == 0
        buf.free()
        sc.close()
    tot = sum(cnt[:6])
    print("%s: %d long lists, %d entries over %d frames; %.0f cycles per tile" %
          (which, cnt[6], cnt[7], frames, tot / max(1, cnt[6])))
    names = PHASES_HUGE if os.environ.get("HUGE") == "1" else PHASES
    for i, name in enumerate(names):
        print("  %-14s %5.1f %%  %8.0f cycles/tile  %6.2f cycles/entry" %
              (name, 100.0 * cnt[i] / max(1, tot), cnt[i] / max(1, cnt[6]), cnt[i] / max(1, cnt[7])))


if __name__ == "__main__":
    main()
