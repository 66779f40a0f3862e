import sys, os, numpy as np
sys.path.insert(0, "gaussian-splatting-web_amd")
import gsplat_amd as gs
W, H, n = 640, 360, 150_000
aos = gs.synth_aos(n, 23, W, H).reshape(n, 80)
right = np.nonzero(aos[:, 0] > 0)[0]
aos[right[np.arange(right.size) % 50 != 0], 2] = 5.0
aos = aos.reshape(-1)
u = gs.bench_uniforms(W, H)
ctx = gs.Context(0)
sc = gs.Scene(ctx, aos, n, 16)
for accum in (0, 1):
    t_min = 0.0 if accum else 1e-4
    ref = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=1.0))
    st0 = ctx.timings()
    for f in (0.5, 0.25, 0.1, 0.02):
        sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=1.0))
        img = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=f))
        st = ctx.timings()
        d = np.abs(img - ref).max(-1)
        ys, xs = np.nonzero(d > 0)
        tiles = sorted(set(zip((ys // 16).tolist(), (xs // 16).tolist())))
        print("accum", accum, "f", f, "diffpx", len(ys), "maxdiff", float(d.max()), "tiles", tiles[:8],
              "nvis", st["n_vis"], "k0", st["k_chunk0"], "k1", st["k_chunk1"], "unsat", st["tiles_unsaturated"],
              "cf", round(st["chunk_fraction"], 4))
        if len(ys):
            y, x = ys[0], xs[0]
            print("   px", (y, x), "img", img[y, x], "ref", ref[y, x])
