"""The list split (gs_opts.list_split = 1, composite_tile's SEG wave pairs), against the oracle.

With list_split = 1 a frame with fewer tiles than the device holds at once (a row strip, a small
image, chunk 1's unsaturated tiles) cuts each long tile list into up to 4 contiguous segments,
blends each from (C = 0, T = 1) on its own wave pair and merges them in list order.  The invariant
this mode keeps ("next round" 1) is the fp32 oracle's bar plus run-to-run
determinism, not bit-identity with the one-chain walk (list_split = 0, which the other test files
hold bit for bit across chunk splits, strips and device groups):

  * fp32 oracle (src/simple_render.ts:169-200 blend, t_min cutoff): MSE < 1e-8, max-abs <= 1e-3
    outside <= 0.01 % pixels (image_close_fp32);
  * the WebGPU stand-in (fp16-target oracle, no cutoff): MSE < 1e-5, >= 99.9 % within 2e-2;
  * the same inputs twice: the same bits.
"""
import numpy as np
import pytest

import oracle_py as orc
from test_gpu_parity import image_close_fp32, webgpu_bar

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")


def _scene(n, seed, W, H, shift):
    aos = gs.synth_aos(n, seed, W, H).reshape(n, 80)
    aos[:, 12] += shift  # opacity logit: faint scenes keep long lists unsaturated
    return np.ascontiguousarray(aos.reshape(-1))


@pytest.mark.parametrize("shift,t_min", [(-4.0, 0.0), (-4.0, 1e-4), (0.0, 1e-4), (-1.5, 1e-4)])
def test_split_small_frame_matches_oracle(gpu_ctx, shift, t_min):
    """320x240 (300 tiles: 4 pairs per tile) with lists of several hundred to thousands of
    entries; saturating (shift 0, -1.5) and not (-4).  Split vs oracle, vs the one-chain walk
    (close, not identical: the split happened), twice (identical)."""
    W, H, n = 320, 240, 300_000
    aos = _scene(n, 91, W, H, shift)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    o_split = gs.make_opts(chunk_fraction=1.0, t_min=t_min, list_split=1)
    a = sc.render(u, W, H, o_split)
    b = sc.render(u, W, H, o_split)
    assert np.array_equal(a, b), "list split: not deterministic"
    exact = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, t_min=t_min))
    rg, _ = sc.tile_lists()
    assert (rg[:, 1] - rg[:, 0]).max() >= 4 * 96  # lists long enough for 4 segments
    assert not np.array_equal(a, exact)
    assert np.abs(a.astype(np.float64) - exact).max() < 2e-3
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=t_min)
    r = image_close_fp32(a, ref, name="split_small_%g_%g" % (shift, t_min))
    assert r[2], r
    if t_min > 0:
        webgpu_bar(a.astype(np.float16), aos, n, 16, u, W, H, name="split_small_webgpu")


def test_split_chunked_frame(gpu_ctx):
    """A two-chunk frame (fixed split) with both chunks split: chunk 1 resumes each tile from
    chunk 0's merged state and splits its own list (k_composite<false, 4> on the compact list of
    unsaturated tiles)."""
    W, H, n = 320, 240, 300_000
    aos = _scene(n, 93, W, H, -1.5)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    imgs = []
    for k in range(3):  # the first: chunk 1 in k_chunk1; then (tiles left unsaturated) its split launches
        gpu_ctx.timings_reset()
        imgs.append(sc.render(u, W, H, gs.make_opts(chunk_fraction=0.1, list_split=1, timing=1)))
        st = gpu_ctx.timings()
        assert st["frames_chunked"] == 1 and st["tiles_unsaturated"] > 0 and st["k_chunk1"] > 0, st
        r = image_close_fp32(imgs[-1], ref, name="split_chunked_%d" % k)
        assert r[2], (k, r)
    assert np.array_equal(imgs[1], imgs[2])


@pytest.mark.parametrize("G", [4, 8])
def test_split_strips_1080p(gpu_ctx, G):
    """1 M Gaussians at 1920x1080 as G row strips (1020 / 2040 tiles per strip: 2 or 1 pairs per
    tile); the assembled strips against the oracle's full frame."""
    W, H, n = 1920, 1080, 1_000_000
    aos = gs.synth_aos(n, 3, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G, list_split=1)) for g in range(G)]
    img = np.concatenate(parts, axis=0)[:H]
    again = np.concatenate([sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G, list_split=1, chunk_fraction=1.0))
                            for g in range(G)], axis=0)[:H]
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    for name, im in (("chunked", img), ("one_chunk", again)):
        r = image_close_fp32(im, ref, name="split_strips_%d_%s" % (G, name))
        assert r[2], (name, r)


@pytest.mark.parametrize("accum", [0, 1])
def test_row_bands_do_not_change_the_image(gpu_ctx, accum):
    """CompositeParams::bands: a frame after one whose tiles mostly did not saturate walks 8x4 row
    bands (4 per wave) instead of 8x8 quarters.  Each pixel still sees its list in order and a
    splat left off its band's list adds exactly zero, so the image is bit-identical: the first
    frame (no history: 2 bands) against the next ones (4 bands), in both accumulation modes."""
    W, H, n = 320, 240, 300_000
    aos = _scene(n, 95, W, H, -4.0)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    o = gs.make_opts(accum=accum, t_min=1e-4 if accum == 0 else 0.0)
    imgs = [sc.render(u, W, H, o) for _ in range(3)]
    assert np.array_equal(imgs[0], imgs[1]) and np.array_equal(imgs[1], imgs[2])
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=accum, t_min=1e-4 if accum == 0 else 0.0)
    from test_gpu_parity import image_close_fp16
    r = image_close_fp32(imgs[2], ref, name="bands4") if accum == 0 else image_close_fp16(imgs[2], ref)
    assert r[2], r
