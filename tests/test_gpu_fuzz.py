"""Seeded randomized parity: frame sizes that are not whole tiles, scene sizes from one splat up,
every SH degree, sparse and dense opacities, moving cameras (so the chunk controller predicts from
a different view than the one drawn), row strips, forced chunk splits and the list split -- each
case against the fp32 oracle (test_gpu_parity.image_close_fp32: MSE < 1e-8, max-abs <= 1e-3
outside <= 0.01 % pixels), with strips and chunk splits bit-identical to the one-pass frame and
every render deterministic. Fixed seeds: a failure names its case and reproduces."""
import numpy as np
import pytest

import oracle_py as orc
from test_gpu_parity import image_close_fp32

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")

N_CASES = 40


def draw_case(i):
    rng = np.random.default_rng(9000 + i)
    W = int(rng.integers(16, 2600))
    H = int(rng.integers(8, 1500))
    n = int(rng.choice([1, 2, 37, 1000, 20_000, 150_000, 1_000_000]))
    nsh = int(rng.choice([1, 4, 9, 16]))
    shift = float(rng.choice([0.0, -2.0, -4.0]))
    cam = str(rng.choice(["bench", "orbit", "cold"]))
    k = int(rng.integers(0, 60))
    G = int(rng.integers(2, 7))
    frac = float(rng.choice([0.0, 0.3, 0.7]))
    return W, H, n, nsh, shift, cam, k, G, frac


def uniforms(cam, W, H, k):
    if cam == "orbit":
        return gs.orbit_uniforms(W, H, k)
    if cam == "cold":
        return gs.cold_uniforms(W, H, k)
    return gs.bench_uniforms(W, H)


@pytest.mark.parametrize("case", range(N_CASES))
def test_randomized_frames(gpu_ctx, case):
    W, H, n, nsh, shift, cam, k, G, frac = draw_case(case)
    tag = "fuzz%d_%dx%d_n%d_sh%d_s%g_%s%d" % (case, W, H, n, nsh, shift, cam, k)
    full = gs.synth_aos(n, 100 + case, W, H).reshape(n, 80)
    full[:, 12] += np.float32(shift)
    rec = np.ascontiguousarray(full[:, : 16 + 4 * nsh]).reshape(-1)
    sc = gs.Scene(gpu_ctx, rec, n, nsh)
    # two earlier views first: the adaptive chunk split of the checked frame is predicted from them
    for j in (k + 7, k + 3):
        sc.render(uniforms(cam, W, H, j), W, H)
    u = uniforms(cam, W, H, k)
    img = sc.render(u, W, H)
    ref, _ = orc.render(rec.view(np.uint8), n, nsh, u, W, H, accum=0, t_min=1e-4)
    r = image_close_fp32(img, ref, name=tag)
    assert r[2], (tag, r)

    one = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    assert np.array_equal(one, img), (tag, "adaptive chunk split differs from one pass")
    if frac > 0:
        split = sc.render(u, W, H, gs.make_opts(chunk_fraction=frac))
        assert np.array_equal(split, one), (tag, "chunk_fraction", frac)
    parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G, chunk_fraction=frac))
             for g in range(G)]
    assert np.array_equal(np.concatenate(parts, axis=0)[:H], one), (tag, "strips", G, frac)

    ls = sc.render(u, W, H, gs.make_opts(list_split=1))
    r = image_close_fp32(ls, ref, name=tag + "_ls")
    assert r[2], (tag, "list_split", r)
    assert np.array_equal(sc.render(u, W, H, gs.make_opts(list_split=1)), ls), (tag, "list_split determinism")


@pytest.mark.parametrize("case", range(12))
def test_randomized_fp16_modes(gpu_ctx, case):
    """The rgba16float-target accumulation (the reference's blend, rounded after every splat)
    against the oracle's fp16-target mode (image_close_fp16), with strips bit-identical to the
    full frame; and the bench's mode (fp32 accumulation, t_min 1e-4, f16 out) against the WebGPU
    stand-in's bar (webgpu_bar)."""
    from test_gpu_parity import image_close_fp16, webgpu_bar
    W, H, n, nsh, shift, cam, k, G, frac = draw_case(500 + case)
    tag = "fuzz16_%d_%dx%d_n%d_sh%d_s%g_%s%d" % (case, W, H, n, nsh, shift, cam, k)
    full = gs.synth_aos(n, 700 + case, W, H).reshape(n, 80)
    full[:, 12] += np.float32(shift)
    rec = np.ascontiguousarray(full[:, : 16 + 4 * nsh]).reshape(-1)
    sc = gs.Scene(gpu_ctx, rec, n, nsh)
    u = uniforms(cam, W, H, k)
    o16 = dict(accum=gs.GS_ACCUM_FP16_TARGET, t_min=0.0)
    img = sc.render(u, W, H, gs.make_opts(**o16))
    ref, st = orc.render(rec.view(np.uint8), n, nsh, u, W, H, accum=1, t_min=0.0)
    r = image_close_fp16(img, ref)
    assert r[2], (tag, r)
    parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G, **o16)) for g in range(G)]
    assert np.array_equal(np.concatenate(parts, axis=0)[:H], img), (tag, "fp16-target strips", G)
    # the visible set, exact (one pass over every rank: a chunked frame projects only the ranks
    # that can still reach an unsaturated tile)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, timing=1))
    assert gpu_ctx.timings()["n_vis"] == st["n_vis"], tag
    bench_mode = sc.render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16))
    webgpu_bar(bench_mode, rec, n, nsh, u, W, H, name=tag)
