"""GPU parity of what the product kernels actually wrote, against the CPU oracle:

  * the composite slots k_project / k_chunk1 stored (gs_debug_last_slots) -- not a re-projection;
  * each tile's list in the order the composite consumed it (gs_debug_tile_lists): it must be the
    oracle's stable global draw order (webgpu-radix-sort = stable ascending, src/renderer.ts:175-183,
    :313) restricted to that tile, on scenes with heavy depth-key ties and duplicate Gaussians;
  * the reference's init-sort grid truncation (ref_quirks, src/renderer.ts:306) over consecutive
    frames, against or_render(quirk=1) carrying the same (key, value) state.

Tolerances as in test_gpu_parity.py (keys, sets and orders bit-exact).
"""
import numpy as np
import pytest

import oracle_py as orc
from conftest import camera, load_scene
from test_gpu_parity import image_close_fp16, image_close_fp32

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")

RECT_EMPTY = 0xFFFFFFFE
SQ = np.sqrt(np.log2(np.e))  # the records hold the quad axes prescaled by sqrt(log2 e)


def check_slots(sl, sp):
    """Slots of a one-chunk frame vs the oracle's projection (sp = orc.project output)."""
    vis = sp["visible"] == 1
    idx = sl["index"]
    assert np.unique(idx).size == idx.size, "a Gaussian holds two slots"
    assert np.array_equal(np.sort(idx), np.nonzero(vis)[0]), "visible set"
    o = sp[idx]
    assert np.array_equal(sl["key"], o["key"])
    assert np.array_equal(sl["keybits"][sl["rect"] != RECT_EMPTY], o["key"][sl["rect"] != RECT_EMPTY])
    np.testing.assert_allclose(sl["r0"][:, 0], o["c"][:, 0], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(sl["r0"][:, 1], o["c"][:, 1], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(np.exp2(sl["r1"][:, 2].astype(np.float64)), o["op"], rtol=2e-6)
    binned = sl["rect"] != RECT_EMPTY
    assert np.array_equal(sl["col"][binned].view(np.uint32), o["col"][binned].astype(np.float32).view(np.uint32))
    g1 = sl["r0"][:, 2:4].astype(np.float64) / SQ
    g2 = sl["r1"][:, 0:2].astype(np.float64) / SQ
    e1n = (o["e1"].astype(np.float64) ** 2).sum(1, keepdims=True)
    e2n = (o["e2"].astype(np.float64) ** 2).sum(1, keepdims=True)
    r1, r2 = o["e1"] / e1n, o["e2"] / e2n
    conic_g = g1[:, :, None] * g1[:, None, :] + g2[:, :, None] * g2[:, None, :]
    conic_r = r1[:, :, None] * r1[:, None, :] + r2[:, :, None] * r2[:, None, :]
    scale = np.abs(conic_r).reshape(len(r1), -1).max(1)[:, None, None]
    assert np.all(np.abs(conic_g - conic_r) <= 2e-5 * scale)


def contributing(sp, W, H, margin=0.98):
    """(tile, index) pairs where the oracle's splat clearly reaches a pixel centre of the tile
    (|u|,|v| <= 2 margin, alpha >= 1/255 / margin): every such pair must be in the tile's list."""
    TX = (W + 15) // 16
    pairs = set()
    for i in np.nonzero(sp["visible"] == 1)[0]:
        s = sp[i]
        x0, y0, x1, y1 = s["rect"]
        xs, ys = np.meshgrid(np.arange(x0, x1 + 1) + 0.5, np.arange(y0, y1 + 1) + 0.5)
        dx, dy = xs - s["c"][0], ys - s["c"][1]
        e1, e2 = s["e1"].astype(np.float64), s["e2"].astype(np.float64)
        u = (dx * e1[0] + dy * e1[1]) / (e1 @ e1)
        v = (dx * e2[0] + dy * e2[1]) / (e2 @ e2)
        a = np.exp(-(u * u + v * v)) * s["op"]
        m = (np.abs(u) <= 2 * margin) & (np.abs(v) <= 2 * margin) & (a >= 1.0 / 255 / margin)
        for px, py in zip(xs[m].astype(int), ys[m].astype(int)):
            pairs.add(((py // 16) * TX + px // 16, int(i)))
    return pairs


def check_tile_lists(sc, sp, W, H, full_sets=True):
    rg, en = sc.tile_lists()
    TX, TY = (W + 15) // 16, (H + 15) // 16
    assert rg.shape[0] == TX * TY
    vis = np.nonzero(sp["visible"] == 1)[0].astype(np.uint32)
    _, order = orc.stable_sort_pairs(sp["key"][vis], vis)  # the reference's draw order
    rank = np.full(sp.size, -1, np.int64)
    rank[order] = np.arange(order.size)
    idx = en[:, 1]
    assert np.array_equal(en[:, 0], sp["key"][idx])
    r = rank[idx]
    assert (r >= 0).all(), "an invisible Gaussian in a tile list"
    # inside every tile the ranks ascend strictly: the stable order restricted to the tile
    tile_of = np.zeros(en.shape[0], np.int64)
    for t in range(rg.shape[0]):
        b, e = rg[t]
        assert b <= e
        tile_of[b:e] = t
        if e - b > 1:
            d = np.diff(r[b:e])
            assert (d > 0).all(), (t, int((d <= 0).sum()))
    # every entry's tile meets the splat's pixel rect; every clear contribution is listed
    rect = sp["rect"][idx]
    tx, ty = tile_of % TX, tile_of // TX
    assert ((rect[:, 0] // 16 <= tx) & (tx <= rect[:, 2] // 16) & (rect[:, 1] // 16 <= ty) &
            (ty <= rect[:, 3] // 16)).all()
    if full_sets:
        have = set(zip(tile_of.tolist(), idx.tolist()))
        missing = contributing(sp, W, H) - have
        assert not missing, sorted(missing)[:5]
    return rg, en


# ------------------------------------------------------------------------------- slots
@pytest.mark.parametrize("scene", ["simple", "pc_short", "m3splat"])
@pytest.mark.parametrize("cam", ["app", "close", "behind"])
def test_slots_match_oracle(gpu_ctx, scene, cam):
    aos, n, nsh = load_scene(scene)
    W, H = 256, 256
    u, _ = camera(scene + "_" + cam, W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    sp = orc.project(aos, n, nsh, u, W, H)
    check_slots(sc.last_slots(), sp)
    check_tile_lists(sc, sp, W, H)


def test_slots_synthetic_strip(gpu_ctx):
    """k_project's slots on a 100 k synthetic scene (Morton-ordered storage, many partitions)."""
    W, H, n = 640, 480, 100_000
    aos = gs.synth_aos(n, 71, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    sp = orc.project(aos.view(np.uint8), n, 16, u, W, H)
    check_slots(sc.last_slots(), sp)
    check_tile_lists(sc, sp, W, H, full_sets=False)


def test_chunk1_slots(gpu_ctx):
    """Two-chunk frame: chunk-1 slots (c1_records_body, in k_chunk1 or k_c1_records) carry the same
    records as the oracle, and every slot's chunk agrees with its key against the split."""
    W, H, n = 640, 360, 150_000
    aos = gs.synth_aos(n, 23, W, H).reshape(n, 80)
    right = np.nonzero(aos[:, 0] > 0)[0]
    aos[right[np.arange(right.size) % 50 != 0], 2] = 5.0
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    sc.render(u, W, H, gs.make_opts(chunk_fraction=0.02))
    sl = sc.last_slots()
    assert (sl["chunk"] == 1).any() and (sl["chunk"] == 0).any()
    assert sl["key"][sl["chunk"] == 0].max() < sl["key"][sl["chunk"] == 1].min()
    sp = orc.project(aos.view(np.uint8), n, 16, u, W, H)
    o = sp[sl["index"]]
    assert (o["visible"] == 1).all()
    assert np.array_equal(sl["key"], o["key"])
    binned = sl["rect"] != RECT_EMPTY
    assert np.array_equal(sl["col"][binned].view(np.uint32), o["col"][binned].astype(np.float32).view(np.uint32))
    np.testing.assert_allclose(sl["r0"][:, :2], o["c"], atol=1e-3, rtol=1e-5)


# ------------------------------------------------------------------------------- order with ties
@pytest.mark.parametrize("depths", [1, 4, 32])
def test_tile_order_with_equal_keys(gpu_ctx, depths):
    """Depth keys forced equal (positions on `depths` planes) plus exact duplicate Gaussians: the
    per-tile order must break ties by the reference index, as the reference's stable sort does."""
    W, H, n = 320, 240, 6000
    rng = np.random.default_rng(depths)
    aos = gs.synth_aos(n, 61 + depths, W, H).reshape(n, 80)
    planes = rng.uniform(3.0, 12.0, depths).astype(np.float32)
    z = planes[rng.integers(0, depths, n)]
    t = np.float32(np.tan(np.pi / 6))
    aos[:, 0] = rng.uniform(-1.0, 1.0, n).astype(np.float32) * z * t * np.float32(W / H)
    aos[:, 1] = rng.uniform(-1.0, 1.0, n).astype(np.float32) * z * t
    aos[:, 2] = -z
    aos[:, 12] = rng.uniform(-3.0, 1.0, n)  # semi-transparent: long lists, late saturation
    dup = rng.choice(n, 500, replace=False)
    aos[dup[:250]] = aos[dup[250:]]  # exact duplicates at other indices
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, t_min=0.0))
    sp = orc.project(aos.view(np.uint8), n, 16, u, W, H)
    keys = sp["key"][sp["visible"] == 1]
    assert np.unique(keys).size <= 2 * depths  # ties everywhere (x: a plane's key is one value)
    check_slots(sc.last_slots(), sp)
    check_tile_lists(sc, sp, W, H)
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    r = image_close_fp32(img, ref)
    assert r[2], r


@pytest.mark.parametrize("n,plane_frac", [(800_000, 0.0), (800_000, 0.7), (1_600_000, 0.0), (1_600_000, 0.7),
                                          (3_200_000, 0.0)])
def test_tile_order_long_lists(gpu_ctx, n, plane_frac):
    """Tile lists of thousands of entries (a faint scene: ~2100, ~4100 or ~8300 per tile), longer
    than one sorting round.  The first frame sorts with the 128-thread shape (rounds of 1024:
    ts_long, a bucket scatter then runs of buckets sorted in place); the second with the shape its
    last frame's mean list length picks: the 256-thread shape (mean > 800; ts_long in rounds of
    2048) at 800 K, the huge shape (mean > 3000; a list of <= 7168 sorted whole in LDS, longer
    ones and those with a bucket of more than 64 keys by the long-list launch) at 1.6 M and 3.2 M.  With 70 % of the Gaussians on one
    depth plane, ts_long meets buckets of more than a round of keys, which it hands to ts_rounds.
    Every tile's list must be the stable global order restricted to the tile."""
    W, H = 320, 240
    rng = np.random.default_rng(5)
    aos = gs.synth_aos(n, 81, W, H).reshape(n, 80)
    aos[:, 12] -= 4.0  # faint: long lists, nothing saturates
    if plane_frac:
        m = rng.random(n) < plane_frac
        d = -aos[m, 2]
        aos[m, 0] *= np.float32(8.0) / d
        aos[m, 1] *= np.float32(8.0) / d
        aos[m, 2] = -8.0
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    sp = orc.project(aos.view(np.uint8), n, 16, u, W, H)
    imgs = []
    for _ in range(2):
        imgs.append(sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, t_min=0.0)))
        rg, en = check_tile_lists(sc, sp, W, H, full_sets=False)
        lens = rg[:, 1] - rg[:, 0]
        assert lens.max() > 2048 and np.median(lens) > 1024, (lens.max(), np.median(lens))
        if n >= 3_200_000:
            assert lens.max() > 8192, lens.max()  # lists for the huge shape's long-list launch
    assert np.array_equal(imgs[0], imgs[1])
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    r = image_close_fp32(imgs[0], ref, name="long_lists_%g" % plane_frac)
    assert r[2], r


def test_tile_order_long_tail(gpu_ctx):
    """A few tiles of 20 K+ entries among lists of ~4 K: the
    second frame takes the huge shape (the last frame's mean list > 3000, two 1024-thread
    workgroups per CU), which sorts a list of <= 7168 entries in one LDS round and hands every
    longer one (and any whose keys crowd more than 64 into one bucket) to the linear long-list pass
    (ts_long at 256 threads, FrameCtl::long_n) instead of rounds that each re-read the list.  Orders must equal the stable global order restricted to each tile; the frame's
    statistics report the longest list and the tiles sent to the long-list pass."""
    W, H, n = 320, 240, 1_600_000
    rng = np.random.default_rng(11)
    aos = gs.synth_aos(n, 83, W, H).reshape(n, 80)
    aos[:, 12] -= 4.0  # faint: long lists, nothing saturates
    # a dense cluster: 120 K Gaussians within ~16 px of the image centre at depth 6-10
    m = rng.choice(n, 120_000, replace=False)
    d = rng.uniform(6.0, 10.0, m.size).astype(np.float32)
    t = np.float32(np.tan(np.pi / 6))
    aos[m, 0] = rng.uniform(-0.1, 0.1, m.size).astype(np.float32) * d * t * np.float32(W / H)
    aos[m, 1] = rng.uniform(-0.1, 0.1, m.size).astype(np.float32) * d * t
    aos[m, 2] = -d
    aos = aos.reshape(-1)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    sp = orc.project(aos.view(np.uint8), n, 16, u, W, H)
    imgs = []
    for f in range(3):
        gpu_ctx.timings_reset()
        imgs.append(sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, t_min=0.0)))
        rg, en = check_tile_lists(sc, sp, W, H, full_sets=False)
        lens = (rg[:, 1] - rg[:, 0]).astype(np.int64)
        assert lens.max() > 20_000 and np.median(lens) > 3000, (lens.max(), np.median(lens))
        assert 0 < (lens > 8192).sum() <= 16, (lens > 8192).sum()
        gpu_ctx.sync()
        st = gpu_ctx.timings()
        assert st["list_max"] == lens.max(), (st["list_max"], lens.max())
        if f >= 1:  # the huge shape: every list past one round (7168) went to the long-list pass
            assert (lens > 7168).sum() <= st["tiles_long"] <= (lens > 7168).sum() + lens.size // 64, \
                (st["tiles_long"], (lens > 7168).sum())
    assert np.array_equal(imgs[0], imgs[1]) and np.array_equal(imgs[1], imgs[2])
    ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=0.0)
    r = image_close_fp32(imgs[1], ref, name="long_tail")
    assert r[2], r


# ------------------------------------------------------------------------------- ref_quirks
def test_keyed_slots_rule():
    assert orc.keyed_slots(62) == 62 and orc.keyed_slots(100) == 96 and orc.keyed_slots(1003) == 1000
    assert orc.keyed_slots(524_280) == 524_280


@pytest.mark.parametrize("accum", [0, 1])
def test_ref_quirks_pc_short_1280x720(gpu_ctx, accum):
    """configs[1] (pc_short at 1280x720) as the reference renders it: 96 of 100 slots keyed, the
    tail carrying the previous frame's sorted (key, value); three consecutive frames from three
    cameras against the oracle with the same state."""
    aos, n, nsh = load_scene("pc_short")
    W, H = 1280, 720
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    state = (np.zeros(n, np.uint32), np.zeros(n, np.uint32))
    t_min = 1e-4 if accum == 0 else 0.0
    for f, cam in enumerate(["app", "close", "app", "behind"]):
        u, _ = camera("pc_short_" + cam, W, H)
        img = sc.render(u, W, H, gs.make_opts(ref_quirks=1, accum=accum, t_min=t_min))
        ref, st = orc.render(aos, n, nsh, u, W, H, accum=accum, t_min=t_min, quirk=1, state=state)
        r = image_close_fp32(img, ref, name="quirk_%d_%d" % (accum, f)) if accum == 0 else image_close_fp16(img, ref)
        assert r[2], (f, r)
        # the draw list: (rank, Gaussian) entries per tile, ranks ascending
        rg, en = sc.tile_lists()
        for t in range(rg.shape[0]):
            b, e = rg[t]
            assert (np.diff(en[b:e, 0].astype(np.int64)) > 0).all()
    # frame 1 drew Gaussian 0 four extra times: the quirk changes the image
    plain = sc.render(u, W, H, gs.make_opts(accum=accum, t_min=t_min))
    assert not np.array_equal(plain, img)


def test_ref_quirks_first_frame_draws_gaussian0_extra(gpu_ctx):
    aos, n, nsh = load_scene("pc_short")
    W, H = 256, 256
    u, _ = camera("pc_short_app", W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    sc.render(u, W, H, gs.make_opts(ref_quirks=1, chunk_fraction=1.0))
    keys, idx = sc.last_order()  # (draw rank, Gaussian), sorted by rank
    sp = orc.project(aos, n, nsh, u, W, H)
    if sp["visible"][0]:
        assert (idx == 0).sum() == 5  # its own slot + the 4 untouched (0, 0) slots, drawn first
        assert (idx[:4] == 0).all()
    assert not np.isin(np.arange(96, 100), idx).any()  # never keyed: not drawn on frame 1


def test_ref_quirks_synthetic_tail(gpu_ctx):
    """N = 1003 (1000 keyed, a 3-slot tail) over frames with a moving camera, against the oracle."""
    W, H, n = 320, 240, 1003
    aos = gs.synth_aos(n, 77, W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    state = (np.zeros(n, np.uint32), np.zeros(n, np.uint32))
    for f in range(4):
        view = gs.look_at((0.3 * f, 0.1 * f, 0.5 * f), (0.0, 0.0, -10.0))
        u = gs.pack_uniforms(view, gs.perspective(1.04719755, W / H, 0.03, 1000.0))
        img = sc.render(u, W, H, gs.make_opts(ref_quirks=1))
        ref, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, quirk=1, state=state)
        r = image_close_fp32(img, ref, name="quirk_tail_%d" % f)
        assert r[2], (f, r)


def test_ref_quirks_all_keyed_equals_plain(gpu_ctx):
    """simple.ply (62 <= 64 slots keyed): the quirk changes nothing."""
    aos, n, nsh = load_scene("simple")
    W, H = 256, 256
    u, _ = camera("simple_app", W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    a = sc.render(u, W, H, gs.make_opts(ref_quirks=1))
    b = sc.render(u, W, H)
    assert np.array_equal(a, b)


def test_ref_quirks_size_limit(gpu_ctx):
    n = 524_281
    sc = gs.Scene(gpu_ctx, gs.synth_aos(n, 1, 64, 64), n, 16)
    with pytest.raises(gs.GsError) as e:
        sc.render(gs.bench_uniforms(64, 64), 64, 64, gs.make_opts(ref_quirks=1))
    assert e.value.code == gs.GS_ERR_UNSUPPORTED
