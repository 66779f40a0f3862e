"""GPU parity tests: the HIP renderer (through the C ABI) against the CPU oracle.

Tolerances:
  * depth keys and the visible set: bit-exact (per-tile draw order: test_gpu_order.py);
  * projected floats: <= 1e-5 relative (colour/opacity) and <= 1e-3 px absolute (centre);
  * image vs the fp32 oracle: MSE < 1e-8 and max-abs <= 1e-3 outside <= 0.01 % pixels
    (pixels whose quad-edge / alpha-threshold test flips under last-ulp differences);
  * image vs the fp16-target oracle: MSE < 1e-5 and >= 99.9 % pixels within 2e-2.
"""
import os

import numpy as np
import pytest

import oracle_py as orc
from conftest import camera, load_scene

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")

SMALL_SCENES = ["simple", "pc_short", "m3splat"]
SMALL_CAMS = ["app", "close", "behind"]


def dump(name, **arrays):
    """On failure, keep the arrays for offline diffing (GS_DUMP_DIR, e.g. gpurun_out/)."""
    d = os.environ.get("GS_DUMP_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        np.savez_compressed(os.path.join(d, name + ".npz"), **arrays)


def image_close_fp32(img, ref, frac_out=1e-4, tol=1e-3, name=None):
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    mse = float((d ** 2).mean())
    bad = float((d.max(axis=-1) > tol).mean())
    ok = mse < 1e-8 and bad <= frac_out
    if not ok and name:
        dump(name, img=img, ref=ref)
    return mse, bad, ok


def image_close_fp16(img, ref):
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    mse = float((d ** 2).mean())
    good = float((d.max(axis=-1) <= 2e-2).mean())
    return mse, good, mse < 1e-5 and good >= 0.999


def webgpu_bar(img16, aos, n, nsh, u, W, H, name=None):
    """The north star's bar for the mode bench.py times (fp32 accumulation, t_min 1e-4, f16 out)
    against the declared WebGPU stand-in: the oracle's rgba16float-target mode with no cutoff
    (src/simple_render.ts:455-471 "under" blend, :499-505 rgba16float target): per-pixel MSE < 1e-5
    over RGBA and >= 99.9 % of pixels within 2e-2 (image_close_fp16)."""
    ref16, _ = orc.render(np.ascontiguousarray(aos).view(np.uint8), n, nsh, u, W, H, accum=1, t_min=0.0)
    r = image_close_fp16(np.asarray(img16).astype(np.float32), ref16)
    assert r[2], (name, r)
    return r


# ------------------------------------------------------------------------------- sort
@pytest.mark.parametrize("n", [1, 7, 100, 4095, 4096, 4097, 65536 + 13, 1_000_003])
def test_sort_pairs_exact(gpu_ctx, n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    keys[::3] = keys[0]  # many ties: stability matters
    vals = np.arange(n, dtype=np.uint32)
    k, v = gpu_ctx.sort_pairs(keys, vals)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(k, keys[order])
    assert np.array_equal(v, vals[order])


@pytest.mark.parametrize("bits", [(0, 8), (0, 13), (0, 16), (8, 24), (3, 30)])
def test_sort_partial_bits(gpu_ctx, bits):
    b0, b1 = bits
    n = 300_001
    rng = np.random.default_rng(b0 * 31 + b1)
    keys = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    vals = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    k, v = gpu_ctx.sort_pairs(keys, vals, b0, b1)
    digit = (keys >> np.uint32(b0)) & np.uint32((1 << (b1 - b0)) - 1) if b1 - b0 < 32 else keys
    order = np.argsort(digit, kind="stable")
    assert np.array_equal(k, keys[order])
    assert np.array_equal(v, vals[order])


def test_sort_matches_oracle(gpu_ctx):
    rng = np.random.default_rng(5)
    n = 200_000
    keys = (rng.integers(0, 64, n) * 1000003).astype(np.uint32)
    vals = rng.permutation(n).astype(np.uint32)
    k, v = gpu_ctx.sort_pairs(keys, vals)
    ko, vo = orc.stable_sort_pairs(keys, vals)
    assert np.array_equal(k, ko) and np.array_equal(v, vo)


# ------------------------------------------------------------------------------- projection + order
@pytest.mark.parametrize("scene", SMALL_SCENES)
@pytest.mark.parametrize("cam", SMALL_CAMS)
def test_projection_and_order(gpu_ctx, scene, cam):
    aos, n, nsh = load_scene(scene)
    W, H = 256, 256
    u, _ = camera(scene + "_" + cam, W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    sc.render(u, W, H)
    sp = orc.project(aos, n, nsh, u, W, H)
    vis = sp["visible"] == 1
    keys, idx = sc.last_order()
    # visible set and keys are bit-exact (last_order sorts the slots on the host; the order the
    # composite used is checked per tile in test_gpu_order.py, and the slot records there too)
    ok_, ov_ = orc.stable_sort_pairs(sp["key"][vis], np.nonzero(vis)[0].astype(np.uint32))
    assert np.array_equal(idx, ov_)
    assert np.array_equal(keys, ok_)
    rec = sc.last_records()[vis]
    o = sp[vis]
    np.testing.assert_allclose(rec[:, 0], o["c"][:, 0], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(rec[:, 1], o["c"][:, 1], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(np.exp2(rec[:, 6].astype(np.float64)), o["op"], rtol=2e-6)
    binned = rec[:, 13].view(np.uint32) > 0  # colour is in the composite records of binned splats
    assert binned.mean() > 0.5
    # SH colour: one thread per splat in the reference's expression order, bit-exact
    assert np.array_equal(rec[binned, 8:11].view(np.uint32), o["col"][binned].astype(np.float32).view(np.uint32))
    e1n = (o["e1"] ** 2).sum(1, keepdims=True)
    e2n = (o["e2"] ** 2).sum(1, keepdims=True)
    sq = np.sqrt(np.log2(np.e))  # records hold the axes prescaled by sqrt(log2 e)
    g1, g2 = rec[:, 2:4].astype(np.float64) / sq, rec[:, 4:6].astype(np.float64) / sq
    r1, r2 = (o["e1"] / e1n).astype(np.float64), (o["e2"] / e2n).astype(np.float64)
    # u^2+v^2 = d^T (e1^ e1^T + e2^ e2^T) d: rotation-invariant conic, tight tolerance
    conic_g = g1[:, :, None] * g1[:, None, :] + g2[:, :, None] * g2[:, None, :]
    conic_r = r1[:, :, None] * r1[:, None, :] + r2[:, :, None] * r2[:, None, :]
    scale = np.abs(conic_r).reshape(len(r1), -1).max(1)[:, None, None]
    assert np.all(np.abs(conic_g - conic_r) <= 2e-5 * scale)
    # the axes themselves: the eigenvector direction is ill-conditioned when lambda1 ~ lambda2
    np.testing.assert_allclose(g1, r1, rtol=2e-3, atol=1e-5)
    np.testing.assert_allclose(g2, r2, rtol=2e-3, atol=1e-5)
    assert np.array_equal(rec[:, 12].view(np.uint32), o["key"])


# ------------------------------------------------------------------------------- images
@pytest.mark.parametrize("scene", SMALL_SCENES)
@pytest.mark.parametrize("cam", SMALL_CAMS)
@pytest.mark.parametrize("size", [(256, 256), (96, 64)])
def test_image_small_fp32(gpu_ctx, scene, cam, size):
    W, H = size
    aos, n, nsh = load_scene(scene)
    u, _ = camera(scene + "_" + cam, W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    img = sc.render(u, W, H, gs.make_opts(t_min=1e-4))
    ref, st = orc.render(aos, n, nsh, u, W, H, accum=0, t_min=1e-4)
    mse, bad, ok = image_close_fp32(img, ref)
    assert ok, (mse, bad)
    assert gpu_ctx.timings()["n_vis"] == st["n_vis"]


@pytest.mark.parametrize("scene", SMALL_SCENES)
def test_image_small_fp16_target(gpu_ctx, scene):
    W, H = 256, 256
    aos, n, nsh = load_scene(scene)
    u, _ = camera(scene + "_behind", W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    img = sc.render(u, W, H, gs.make_opts(accum=gs.GS_ACCUM_FP16_TARGET, t_min=0.0))
    ref, _ = orc.render(aos, n, nsh, u, W, H, accum=1, t_min=0.0)
    mse, good, ok = image_close_fp16(img, ref)
    assert ok, (mse, good)


def test_image_no_early_stop(gpu_ctx):
    W, H = 256, 256
    aos, n, nsh = load_scene("pc_short")
    u, _ = camera("pc_short_behind", W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    img = sc.render(u, W, H, gs.make_opts(t_min=0.0))
    ref, _ = orc.render(aos, n, nsh, u, W, H, accum=0, t_min=0.0)
    assert image_close_fp32(img, ref)[2]


def test_synthetic_1m_1080p(gpu_ctx):
    """Config 3 (synthetic 1 M @ 1920x1080) against the full oracle."""
    W, H = 1920, 1080
    aos = gs.synth_aos(1_000_000, 1, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 1_000_000, 16)
    img = sc.render(u, W, H, gs.make_opts(timing=1))
    st_gpu = gpu_ctx.timings()
    ref, st = orc.render(aos.view(np.uint8), 1_000_000, 16, u, W, H, accum=0, t_min=1e-4)
    assert st_gpu["n_vis"] == st["n_vis"]
    # the oracle counts every tile of each binning box; the GPU bins each splat's alpha >= 1/255
    # ellipse row by row (a subset), and the image check below shows no contributing tile is lost
    assert 0.4 * st["k_tiles"] <= st_gpu["k_entries"] <= st["k_tiles"]
    mse, bad, ok = image_close_fp32(img, ref, name="synth1m")
    assert ok, (mse, bad)


def test_strips_match_full_image(gpu_ctx):
    W, H = 1920, 1080
    aos = gs.synth_aos(200_000, 3, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 200_000, 16)
    full = sc.render(u, W, H)
    for G in (2, 3, 8):
        parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G)) for g in range(G)]
        img = np.concatenate(parts, axis=0)
        assert np.array_equal(img[:H], full), G
        assert not img[H:].any(), G  # padding rows past the image: zero


def test_deterministic(gpu_ctx):
    W, H = 640, 480
    aos = gs.synth_aos(300_000, 9, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 300_000, 16)
    a = sc.render(u, W, H)
    b = sc.render(u, W, H)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_f16_output(gpu_ctx):
    W, H = 320, 200
    aos = gs.synth_aos(50_000, 4, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 50_000, 16)
    a = sc.render(u, W, H)
    h = sc.render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16))
    assert np.array_equal(a.astype(np.float16), h)


# ------------------------------------------------------------------------------- edge cases
def test_empty_scene(gpu_ctx):
    sc = gs.Scene(gpu_ctx, np.zeros(0, np.uint8), 0, 16)
    img = sc.render(gs.bench_uniforms(64, 48), 64, 48)
    assert img.shape == (48, 64, 4) and not img.any()


def test_all_culled(gpu_ctx):
    W, H = 200, 100
    aos = gs.synth_aos(10_000, 2, W, H)
    view = gs.look_at((0.0, 0.0, 0.0), (0.0, 0.0, 1.0))  # looking away from every splat
    u = gs.pack_uniforms(view, gs.perspective(1.04719755, W / H, 0.03, 1000.0))
    sc = gs.Scene(gpu_ctx, aos, 10_000, 16)
    img = sc.render(u, W, H)
    assert not img.any()
    assert gpu_ctx.timings()["n_vis"] == 0


@pytest.mark.parametrize("size", [(1, 1), (17, 33), (16, 16), (1023, 7)])
def test_odd_sizes(gpu_ctx, size):
    W, H = size
    aos = gs.synth_aos(20_000, 11, max(W, 2), max(H, 2))
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 20_000, 16)
    img = sc.render(u, W, H)
    ref, _ = orc.render(aos.view(np.uint8), 20_000, 16, u, W, H)
    r = image_close_fp32(img, ref, name="odd_%dx%d" % (W, H))
    assert r[2], r


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_thin_rotated_splats_binning(gpu_ctx, seed):
    """Ellipse binning is conservative: sparse, thin, rotated, mostly opaque splats on an empty
    background with no early termination, so a tile dropped from a splat's list would change
    pixels at T ~ 1; at most 2 pixels may differ by more than 1e-3 (alpha-threshold rounding)."""
    W, H = 512, 384
    n = 400
    rng = np.random.default_rng(seed)
    aos = np.zeros((n, 80), np.float32)
    z = rng.uniform(3.0, 8.0, n)
    aos[:, 0] = rng.uniform(-0.6, 0.6, n) * z
    aos[:, 1] = rng.uniform(-0.45, 0.45, n) * z
    aos[:, 2] = -z
    aos[:, 4] = rng.uniform(0.2, 0.9, n)
    aos[:, 5] = rng.uniform(0.005, 0.04, n)
    aos[:, 6] = rng.uniform(0.005, 0.04, n)
    q = rng.normal(size=(n, 4))
    aos[:, 8:12] = q / np.linalg.norm(q, axis=1, keepdims=True)
    aos[:, 12] = rng.uniform(-2.0, 6.0, n)
    aos[:, 16:19] = rng.uniform(0.5, 2.0, (n, 3))
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H, gs.make_opts(t_min=0.0))
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64)).max(axis=-1)
    assert st["n_vis"] > n // 2
    assert int((d > 1e-3).sum()) <= 2, (int((d > 1e-3).sum()), float(d.max()))


def test_huge_splats(gpu_ctx):
    """Splats clamped by the 4096-px cap (full-screen quads) and a Gaussian at the camera."""
    W, H = 320, 240
    n = 64
    aos = gs.synth_aos(n, 21, W, H).reshape(n, 80)
    aos[:, 4:7] = 0.5  # large scales
    aos[0, 0:3] = (0.0, 0.0, -0.0301)  # just past the near plane
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H)
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H)
    r = image_close_fp32(img, ref, name="huge_splats")
    assert r[2], r


@pytest.mark.parametrize("nsh", [1, 4, 9])
def test_lower_sh_degrees(gpu_ctx, nsh):
    W, H = 128, 96
    n = 5000
    full = gs.synth_aos(n, 13, W, H).reshape(n, 80)
    rec = full[:, : 16 + 4 * nsh].copy().reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, rec, n, nsh)
    img = sc.render(u, W, H)
    ref, _ = orc.render(rec.view(np.uint8), n, nsh, u, W, H)
    r = image_close_fp32(img, ref, name="sh%d" % nsh)
    assert r[2], r


def test_scene_turnover_on_one_context(gpu_ctx):
    """Round-5's unexplained fault: test_lower_sh_degrees[1] (n 5000, SH degree 0,
    128x96) died in k_project with a memory aperture violation after 111 tests had run on the
    session context.  This replays the suite's order on one context three times -- a large scene
    rendered as frames in flight (chunked, seeded), a 64-Gaussian scene of full-screen splats,
    then the three low-SH scenes -- each freed before the next is uploaded, and every small frame
    against the oracle.  The frame-state guards (kErrState) turn a count that does not fit its
    list into an error; none may fire."""
    W, H = 128, 96
    n = 5000
    full = gs.synth_aos(n, 13, W, H).reshape(n, 80)
    u = gs.bench_uniforms(W, H)
    refs = {}
    for rnd in range(3):
        big_n = 400_000
        big = gs.Scene(gpu_ctx, gs.synth_aos(big_n, 7 + rnd, 1280, 720), big_n, 16)
        ub = gs.bench_uniforms(1280, 720)
        bufs = [gs.DeviceBuffer(1280 * 720 * 8) for _ in range(4)]
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
        for k in range(8):
            big.render_device(ub if k % 3 else gs.cold_uniforms(1280, 720, k), 1280, 720, bufs[k % 4].ptr.value,
                              1280 * 720 * 8, None, o)
        gpu_ctx.sync()
        for b in bufs:
            b.free()
        big.close()
        hw, hh = 320, 240
        huge = gs.synth_aos(64, 21, hw, hh).reshape(64, 80)
        huge[:, 4:7] = 0.5
        hs = gs.Scene(gpu_ctx, huge.reshape(-1), 64, 16)
        hs.render(gs.bench_uniforms(hw, hh), hw, hh)
        hs.close()
        for nsh in (1, 4, 9):
            rec = full[:, : 16 + 4 * nsh].copy().reshape(-1)
            sc = gs.Scene(gpu_ctx, rec, n, nsh)
            img = sc.render(u, W, H)
            sc.close()
            if nsh not in refs:
                refs[nsh], _ = orc.render(rec.view(np.uint8), n, nsh, u, W, H)
            r = image_close_fp32(img, refs[nsh])
            assert r[2], (rnd, nsh, r)


def test_bad_arguments(gpu_ctx):
    with pytest.raises(gs.GsError):
        gs.Scene(gpu_ctx, np.zeros(112, np.uint8), 1, 3)  # n_sh=3 is not a record size the reference makes


@pytest.mark.parametrize("accum", [0, 1])
def test_chunk_split_is_invisible(gpu_ctx, accum):
    """The saturation-aware two-chunk frame gives the same bits as one pass over every rank,
    for any split (both accumulation modes, with unsaturated tiles present)."""
    W, H = 640, 360
    n = 150_000
    aos = gs.synth_aos(n, 23, W, H).reshape(n, 80)
    # right half of the screen sparse: most of its splats moved behind the camera, so its tiles
    # never saturate and chunk 1 has work
    right = np.nonzero(aos[:, 0] > 0)[0]
    aos[right[np.arange(right.size) % 50 != 0], 2] = 5.0
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    t_min = 0.0 if accum else 1e-4
    ref = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=1.0))
    for f in (0.0, 0.1, 0.3, 0.7, 0.02):  # the last, fixed split leaves unsaturated tiles
        img = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=f))
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f
    st = gpu_ctx.timings()
    assert st["tiles_unsaturated"] > 0


@pytest.mark.parametrize("accum", [0, 1])
def test_wide_splats_chunked(gpu_ctx, accum):
    """Splats binding >= 256 tiles (row-wise emission) in both chunks: near ones in chunk 0,
    faint far ones that reach the unsaturated tiles in chunk 1; identical to one pass and close
    to the oracle."""
    W, H = 640, 360
    n = 150_000
    aos = gs.synth_aos(n, 31, W, H).reshape(n, 80)
    right = np.nonzero(aos[:, 0] > 0)[0]
    aos[right[np.arange(right.size) % 50 != 0], 2] = 5.0
    rng = np.random.default_rng(5)
    wide = rng.choice(n, 600, replace=False)
    aos[wide, 4:7] = rng.uniform(0.05, 0.6, (600, 3)).astype(np.float32) * -aos[wide, 2:3]
    aos[wide[:300], 12] = -3.0  # faint: these do not saturate tiles on their own
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    t_min = 0.0 if accum else 1e-4
    ref = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=1.0))
    for f in (0.0, 0.05, 0.2, 0.01):  # the last, fixed split leaves unsaturated tiles
        img = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min, chunk_fraction=f))
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f
    assert gpu_ctx.timings()["tiles_unsaturated"] > 0
    orc_img, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=accum, t_min=t_min)
    if accum == 0:
        r = image_close_fp32(ref, orc_img, name="wide_chunked")
    else:
        r = image_close_fp16(ref, orc_img)
    assert r[2], r


def test_chunked_strips(gpu_ctx):
    W, H = 800, 600
    aos = gs.synth_aos(100_000, 29, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 100_000, 16)
    full = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=4, chunk_fraction=0.2))
             for g in range(4)]
    assert np.array_equal(np.concatenate(parts, axis=0)[:H], full)


def test_long_tile_lists(gpu_ctx):
    """Every tile's list far longer than one LDS round of k_tile_sort (rounds of consecutive
    keys), faint splats so the composite walks the whole list; against the fp32 oracle."""
    W, H = 64, 64
    n = 10_000
    rng = np.random.default_rng(41)
    aos = gs.synth_aos(n, 41, W, H).reshape(n, 80)
    d = rng.uniform(4.0, 12.0, n).astype(np.float32)
    t = np.float32(np.tan(np.pi / 6))
    aos[:, 0] = rng.uniform(-0.3, 0.3, n) * d * t
    aos[:, 1] = rng.uniform(-0.3, 0.3, n) * d * t
    aos[:, 2] = -d
    aos[:, 4:7] = (1.5 * d * t)[:, None]  # about the image's size
    aos[:, 12] = -3.9  # op ~ 0.02
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H, gs.make_opts(t_min=0.0, chunk_fraction=1.0, timing=1))
    assert gpu_ctx.timings()["k_entries"] >= 16 * 2 * 2048
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    r = image_close_fp32(img, ref, name="long_lists")
    assert r[2], r


def test_skewed_tile_keys(gpu_ctx):
    """Tile (0, 0) holds 1000 near splats and one far splat: its keys crowd a few of
    k_tile_sort's buckets (the bitonic path); the other tiles hold mid-depth splats."""
    W, H = 64, 64
    n = 200_000
    rng = np.random.default_rng(43)
    aos = gs.synth_aos(n, 43, W, H).reshape(n, 80)
    t = np.float32(np.tan(np.pi / 6))
    near = np.arange(1000)
    d = rng.uniform(2.0, 2.5, near.size).astype(np.float32)
    aos[near, 0] = (-1.0 + rng.uniform(0.1, 0.4, near.size)) * d * t
    aos[near, 1] = (1.0 - rng.uniform(0.1, 0.4, near.size)) * d * t
    aos[near, 2] = -d
    aos[near, 4:7] = 0.004
    aos[near, 12] = -3.0
    mid = np.arange(1000, n - 1)
    d = rng.uniform(8.0, 20.0, mid.size).astype(np.float32)
    aos[mid, 0] = rng.uniform(0.1, 0.9, mid.size) * d * t
    aos[mid, 1] = rng.uniform(-0.9, 0.9, mid.size) * d * t
    aos[mid, 2] = -d
    aos[mid, 4:7] = (0.002 * d)[:, None]
    aos[n - 1, 0:3] = (0.0, 0.0, -40.0)
    aos[n - 1, 4:7] = 30.0
    aos[n - 1, 12] = 0.0
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H, gs.make_opts(t_min=0.0, chunk_fraction=1.0))
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    r = image_close_fp32(img, ref, name="skewed_keys")
    assert r[2], r


def _plus_z_uniforms(W, H, fovy=1.0):
    """A +z-forward camera (the reference's JSON-camera convention, src/camera.ts:467-492): view
    flips y and z, projection = 3DGS getProjectionMatrix (src/camera.ts:19-42), column-major."""
    view = np.diag([1.0, -1.0, -1.0, 1.0]).astype(np.float32)
    n, f = 0.2, 100.0
    th = np.tan(fovy / 2)
    tw = th * W / H
    P = np.zeros((4, 4), np.float64)
    P[0, 0] = 1.0 / tw
    P[1, 1] = 1.0 / th
    P[2, 2] = f / (f - n)
    P[2, 3] = -(f * n) / (f - n)
    P[3, 2] = 1.0
    return gs.pack_uniforms(view.T.reshape(-1), P.T.reshape(-1).astype(np.float32))


@pytest.mark.parametrize("cam", ["oblique", "plus_z"])
def test_other_cameras_strips_and_oracle(gpu_ctx, cam):
    """Partition bounds and the per-partition cull under an oblique -z camera and a +z camera:
    the full frame against the fp32 oracle, row strips bit-identical to it."""
    W, H = 640, 480
    n = 200_000
    aos = gs.synth_aos(n, 47, W, H)
    if cam == "oblique":
        view = gs.look_at((3.0, 2.0, 4.0), (0.0, 0.0, -11.0))
        u = gs.pack_uniforms(view, gs.perspective(1.04719755, W / H, 0.03, 1000.0))
    else:
        u = _plus_z_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    full = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, timing=1))
    assert gpu_ctx.timings()["n_vis"] > 1000
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    r = image_close_fp32(full, ref, name="cam_" + cam)
    assert r[2], r
    for G in (3, 8):
        parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=G, chunk_fraction=1.0))
                 for g in range(G)]
        assert np.array_equal(np.concatenate(parts, axis=0)[:H], full), G


def test_non_finite_gaussians(gpu_ctx):
    """NaN / infinite positions, scales and rotations (stored last in Morton order, outside the
    partition bounds): never drawn, the rest of the image unchanged (fp32 oracle)."""
    W, H = 320, 240
    n = 50_000
    aos = gs.synth_aos(n, 53, W, H).reshape(n, 80)
    rng = np.random.default_rng(53)
    bad = rng.choice(n, 600, replace=False)
    aos[bad[:200], 0] = np.nan
    aos[bad[200:300], 1] = np.inf
    aos[bad[300:400], 4:7] = np.inf
    aos[bad[400:500], 8:12] = np.nan
    aos[bad[500:], 12] = np.nan
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H)
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    assert np.isfinite(img).all()
    r = image_close_fp32(img, ref, name="non_finite")
    assert r[2], r


@pytest.mark.parametrize("size", [(640, 480), (1920, 1080)])
def test_pipelined_frames_match_single_frames(gpu_ctx, size):
    """Consecutive frames overlap on the GPU (frame sets with their own streams; three frames in
    flight below 1536 tiles, two above): a burst of frames with alternating cameras, strips, chunk
    splits and two scenes, enqueued without any host wait, must reproduce each frame rendered
    alone, bit for bit."""
    W, H = size
    n = 200_000
    sa = gs.Scene(gpu_ctx, gs.synth_aos(n, 5, W, H), n, 16)
    sb = gs.Scene(gpu_ctx, gs.synth_aos(n // 2, 6, W, H), n // 2, 16)
    ua = gs.bench_uniforms(W, H)
    view = gs.look_at((3.0, 2.0, 4.0), (0.0, 0.0, -11.0))
    ub = gs.pack_uniforms(view, gs.perspective(1.04719755, W / H, 0.03, 1000.0))
    F16 = gs.GS_OUT_RGBA_F16
    seq = [(sa, ua, gs.make_opts(out_format=F16)),
           (sa, ub, gs.make_opts(out_format=F16)),
           (sb, ua, gs.make_opts(out_format=F16)),
           (sa, ua, gs.make_opts(out_format=F16, strip_index=1, strip_count=3)),
           (sa, ub, gs.make_opts(out_format=F16, chunk_fraction=0.25)),
           (sb, ub, gs.make_opts(out_format=F16)),
           (sa, ua, gs.make_opts(out_format=F16)),
           (sa, ub, gs.make_opts(out_format=F16, strip_index=2, strip_count=3))]
    refs = [sc.render(u, W, H, o) for sc, u, o in seq]  # each frame alone (gs_render waits)
    bufs = [gs.DeviceBuffer(H * W * 8) for _ in seq]
    for _ in range(2):
        for (sc, u, o), b in zip(seq, bufs):
            sc.render_device(u, W, H, b.ptr.value, b.nbytes, None, o)
        gpu_ctx.sync()
        for j, ((sc, u, o), b, ref) in enumerate(zip(seq, bufs, refs)):
            got = np.empty(ref.shape, np.float16)
            b.to_host(got)
            # a strip's rows past the image (padding to whole tiles) are written as zero
            row0 = gs.strip_rows(H, o.strip_index, o.strip_count)[0] if o.strip_count > 1 else 0
            valid = min(ref.shape[0], H - row0)
            bad = (got.view(np.uint16) != ref.view(np.uint16)).any(axis=2)
            rows = np.nonzero(bad.any(axis=1))[0]
            assert not bad.any(), (j, int(bad.sum()), rows[:3].tolist(), rows[-3:].tolist(), o.strip_count)
            assert not got[valid:].view(np.uint16).any()
    for b in bufs:
        b.free()
    sa.close()
    sb.close()


def _sparse_right_scene(n, seed, W, H):
    """Right half of the screen sparse (most of its splats moved behind the camera): its tiles
    never saturate, so chunk 1 has work in every frame with a chunk split."""
    aos = gs.synth_aos(n, seed, W, H).reshape(n, 80)
    right = np.nonzero(aos[:, 0] > 0)[0]
    aos[right[np.arange(right.size) % 50 != 0], 2] = 5.0
    return aos.reshape(-1)


def test_chunk1_frames_back_to_back(gpu_ctx):
    """Many two-chunk frames with unsaturated tiles enqueued without host waits (k_chunk1 with its
    grid barriers, then the separate chunk-1 launches once the host has seen unsaturated tiles):
    no device fault is reported and every frame equals the same frame rendered alone."""
    W, H = 640, 360
    n = 150_000
    sc = gs.Scene(gpu_ctx, _sparse_right_scene(n, 23, W, H), n, 16)
    ua = gs.bench_uniforms(W, H)
    ub = gs.pack_uniforms(gs.look_at((0.5, 0.3, 0.0), (0.0, 0.0, -10.0)), gs.perspective(1.04719755, W / H, 0.03, 1000.0))
    F16 = gs.GS_OUT_RGBA_F16
    cases = [(ua, 0.02), (ub, 0.1), (ua, 0.3), (ub, 0.02)]
    refs = [sc.render(u, W, H, gs.make_opts(out_format=F16, chunk_fraction=f)) for u, f in cases]
    bufs = [gs.DeviceBuffer(H * W * 8) for _ in range(24)]
    for k, b in enumerate(bufs):
        u, f = cases[k % len(cases)]
        sc.render_device(u, W, H, b.ptr.value, b.nbytes, None, gs.make_opts(out_format=F16, chunk_fraction=f))
    gpu_ctx.sync()  # raises GsError if any frame's chunk-1 barrier timed out
    assert gpu_ctx.timings()["tiles_unsaturated"] > 0
    for k, b in enumerate(bufs):
        got = np.empty(refs[0].shape, np.float16)
        b.to_host(got)
        assert np.array_equal(got.view(np.uint16), refs[k % len(cases)].view(np.uint16)), k
        b.free()
    sc.close()


def test_device_frame_overflow_reported(gpu_ctx):
    """A device-resident frame whose tile lists exceed the capacity (huge splats covering the
    screen) is reported by a later gs_render_device / gs_sync call, not hidden by the clean frames
    after it; once the capacity has grown, frames equal gs_render's."""
    W, H = 1280, 720
    n = 3000
    aos = gs.synth_aos(n, 41, W, H).reshape(n, 80)
    aos[:, 4:7] = np.abs(aos[:, 2:3]) * 2.0  # every splat's quad covers the screen
    aos[:, 12] = -5.0  # faint: the composite walks whole lists
    aos = aos.reshape(-1)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    u = gs.bench_uniforms(W, H)
    o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, chunk_fraction=1.0)
    buf = gs.DeviceBuffer(H * W * 8)
    errors = []
    for _ in range(6):
        try:
            sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
        except gs.GsError as e:
            errors.append(str(e))
    try:
        gpu_ctx.sync()
    except gs.GsError as e:
        errors.append(str(e))
    assert errors and all("capacity" in e for e in errors), errors
    for _ in range(3):
        sc.render_device(u, W, H, buf.ptr.value, buf.nbytes, None, o)
    gpu_ctx.sync()
    got = np.empty((H, W, 4), np.float16)
    buf.to_host(got)
    ref = sc.render(u, W, H, o)
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))
    buf.free()
    sc.close()
