"""The C ABI's device group (gs_ctx_create with a device list): one context drives every device,
strip g of G on devices[g], one gather into devices[0] (RCCL all-gather over distinct devices;
peer copies when the list repeats a device, which is how a one-GPU box exercises the whole group
path).  Every image must equal the single-device frame bit for bit."""
import numpy as np
import pytest

from conftest import camera, load_scene

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")


@pytest.fixture(scope="module")
def scene_data():
    W, H, n = 800, 600, 200_000
    return W, H, n, gs.synth_aos(n, 91, W, H), gs.bench_uniforms(W, H)


@pytest.fixture(scope="module")
def single_images(scene_data):
    W, H, n, aos, u = scene_data
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, n, 16)
        f32 = sc.render(u, W, H)
        f16 = sc.render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, accum=gs.GS_ACCUM_FP16_TARGET))
        n_vis = ctx.timings()["n_vis"]
    return f32, f16, n_vis


@pytest.mark.parametrize("G", [2, 3, 8])
def test_group_host_render_matches_single(scene_data, single_images, G):
    W, H, n, aos, u = scene_data
    with gs.Context([0] * G) as gc:
        assert gc.info() == (G, "peer_copy")
        sc = gs.Scene(gc, aos, n, 16)
        img = sc.render(u, W, H)
        assert np.array_equal(img, single_images[0])
        st = gc.timings()
        assert st["n_vis"] >= single_images[2]  # per-strip visible counts: a splat may reach two strips
        assert st["tile_row_begin"] == 0 and st["tile_row_end"] == (H + 15) // 16


@pytest.mark.parametrize("G", [2, 4])
def test_group_device_frames_in_flight(scene_data, single_images, G):
    """gs_render_device on a group: a burst of frames without host waits, f16 output on device 0."""
    W, H, n, aos, u = scene_data
    with gs.Context([0] * G) as gc:
        sc = gs.Scene(gc, aos, n, 16)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16, accum=gs.GS_ACCUM_FP16_TARGET)
        bufs = [gs.DeviceBuffer(H * W * 8) for _ in range(5)]
        for b in bufs:
            sc.render_device(u, W, H, b.ptr.value, b.nbytes, None, o)
        gc.sync()
        for b in bufs:
            got = np.empty((H, W, 4), np.float16)
            b.to_host(got)
            assert np.array_equal(got.view(np.uint16), single_images[1].view(np.uint16))
            b.free()


def test_group_ref_quirks(scene_data):
    """ref_quirks on a group: every member keeps the same slot state, frame after frame."""
    aos, n, nsh = load_scene("pc_short")
    W, H = 1280, 720
    with gs.Context(0) as ctx, gs.Context([0, 0, 0]) as gc:
        a = gs.Scene(ctx, aos, n, nsh)
        b = gs.Scene(gc, aos, n, nsh)
        for cam in ["app", "close", "behind"]:
            u, _ = camera("pc_short_" + cam, W, H)
            o = gs.make_opts(ref_quirks=1)
            assert np.array_equal(a.render(u, W, H, o), b.render(u, W, H, o))


def test_group_arguments():
    with pytest.raises(gs.GsError) as e:
        gs.Context([0, 4096])
    assert e.value.code == gs.GS_ERR_INVALID
    with gs.Context([0, 0]) as gc:
        sc = gs.Scene(gc, gs.synth_aos(1000, 1, 64, 64), 1000, 16)
        with pytest.raises(gs.GsError) as e:
            sc.render(gs.bench_uniforms(64, 64), 64, 64, gs.make_opts(strip_index=0, strip_count=2))
        assert e.value.code == gs.GS_ERR_INVALID
        with pytest.raises(gs.GsError) as e:
            sc.last_slots()
        assert e.value.code == gs.GS_ERR_UNSUPPORTED


def _group_burst_and_error(devices, gather):
    """A group's render_device burst of 20 frames in flight on a top-heavy scene (two rebalances of
    the strips, both strip buffers of every member alternating), every frame bit-identical to the
    single-device frame; then a frame error (tile-list overflow on huge splats) reported by a later
    call, and clean, bit-identical frames after it.  Each member enqueues from its own host thread."""
    W, H, n = 640, 480, 150_000
    aos = _top_heavy_scene(n, 11, W, H)
    F16 = gs.GS_OUT_RGBA_F16
    views = [gs.orbit_uniforms(W, H, k) for k in range(0, 40, 2)]
    with gs.Context(0) as ctx:
        one = gs.Scene(ctx, aos, n, 16)
        refs = [one.render(u, W, H, gs.make_opts(out_format=F16)) for u in views]
    with gs.Context(devices) as gc:
        assert gc.info() == (len(devices), gather)
        sc = gs.Scene(gc, aos, n, 16)
        bufs = [gs.DeviceBuffer(H * W * 8) for _ in range(len(views))]
        for u, b in zip(views, bufs):
            sc.render_device(u, W, H, b.ptr.value, b.nbytes, None, gs.make_opts(out_format=F16))
        gc.sync()
        assert gc.timings()["frames_rendered"] >= len(views)
        for k, b in enumerate(bufs):
            got = np.empty((H, W, 4), np.float16)
            b.to_host(got)
            assert np.array_equal(got.view(np.uint16), refs[k].view(np.uint16)), (k, gc.strips())
        # an induced frame error: every splat's quad covers the screen, so every member's tile
        # lists overflow (12 000 x 1200 tiles; a member starts with ~1 M entries of capacity)
        m = 12000
        big = gs.synth_aos(m, 41, W, H).reshape(m, 80)
        big[:, 4:7] = np.abs(big[:, 2:3]) * 2.0
        big[:, 12] = 0.0
        bsc = gs.Scene(gc, big.reshape(-1), m, 16)
        u = gs.bench_uniforms(W, H)
        o = gs.make_opts(out_format=F16, chunk_fraction=1.0)
        errors = []
        for _ in range(4):
            try:
                bsc.render_device(u, W, H, bufs[0].ptr.value, bufs[0].nbytes, None, o)
            except gs.GsError as e:
                errors.append(str(e))
        try:
            gc.sync()
        except gs.GsError as e:
            errors.append(str(e))
        assert errors and all("capacity" in e for e in errors), errors
        with gs.Context(0) as ctx:
            want = gs.Scene(ctx, big.reshape(-1), m, 16).render(u, W, H, o)
        for b in bufs[:3]:
            bsc.render_device(u, W, H, b.ptr.value, b.nbytes, None, o)
        gc.sync()
        for b in bufs[:3]:
            got = np.empty((H, W, 4), np.float16)
            b.to_host(got)
            assert np.array_equal(got.view(np.uint16), want.view(np.uint16))
        # and the first scene renders on after the error
        sc.render_device(views[3], W, H, bufs[0].ptr.value, bufs[0].nbytes, None, gs.make_opts(out_format=F16))
        gc.sync()
        got = np.empty((H, W, 4), np.float16)
        bufs[0].to_host(got)
        assert np.array_equal(got.view(np.uint16), refs[3].view(np.uint16))
        for b in bufs:
            b.free()


@pytest.mark.parametrize("peer", [False, True])
def test_group_burst_and_frame_error_one_device(peer, monkeypatch):
    """The burst / frame-error sequence on a group that repeats device 0: its members render
    straight into their rows of the image, or (GS_GROUP_PEER_COPY=1) into strip buffers that are
    peer-copied into it -- the path of members on another device without RCCL."""
    if peer:
        monkeypatch.setenv("GS_GROUP_PEER_COPY", "1")
    _group_burst_and_error([0, 0, 0, 0], "peer_copy")


def test_group_distinct_devices_use_rccl():
    """With two or more GPUs the group gathers with RCCL (not reachable on a one-GPU box): a
    synchronous frame, then the burst / frame-error sequence over every device of the box (up to 8)."""
    if gs.device_count() < 2:
        pytest.skip("one GPU")
    W, H, n = 640, 480, 100_000
    aos = gs.synth_aos(n, 93, W, H)
    u = gs.bench_uniforms(W, H)
    with gs.Context(0) as ctx, gs.Context([0, 1]) as gc:
        assert gc.info() == (2, "rccl")
        a = gs.Scene(ctx, aos, n, 16).render(u, W, H)
        b = gs.Scene(gc, aos, n, 16).render(u, W, H)
        assert np.array_equal(a, b)
    _group_burst_and_error(list(range(min(8, gs.device_count()))), "rccl")


def test_chunk1_grid_is_resident(gpu_ctx):
    """The context sized k_chunk1's grid from the occupancy query of this device."""
    grid, occ = gs.chunk1_grid(gpu_ctx)
    assert occ >= 1 and 1 <= grid <= 64
    assert grid == gs.chunk1_grid(None, occ, 256)[0] or grid <= occ * 256


def test_explicit_tile_rows_match_full(scene_data, single_images):
    """gs_opts.tile_row_begin/end (explicit, uneven strips): the strips laid end to end are the
    full frame bit for bit, f32 and f16 output."""
    W, H, n, aos, u = scene_data
    TR = (H + 15) // 16
    cuts = [0, 3, 4, 21, TR]
    with gs.Context(0) as ctx:
        sc = gs.Scene(ctx, aos, n, 16)
        parts = [sc.render(u, W, H, gs.make_opts(tile_rows=(a, b))) for a, b in zip(cuts[:-1], cuts[1:])]
        assert [p.shape[0] for p in parts] == [min(16 * b, H) - 16 * a for a, b in zip(cuts[:-1], cuts[1:])]
        assert np.array_equal(np.concatenate(parts, axis=0), single_images[0])
        o16 = dict(out_format=gs.GS_OUT_RGBA_F16, accum=gs.GS_ACCUM_FP16_TARGET)
        parts = [sc.render(u, W, H, gs.make_opts(tile_rows=(a, b), **o16)) for a, b in zip(cuts[:-1], cuts[1:])]
        assert np.array_equal(np.concatenate(parts, axis=0).view(np.uint16), single_images[1].view(np.uint16))
        for bad in ((0, TR + 1), (5, 5), (-1, 3)):
            with pytest.raises(gs.GsError) as e:
                sc.render(u, W, H, gs.make_opts(tile_rows=bad))
            assert e.value.code == gs.GS_ERR_INVALID
        with pytest.raises(gs.GsError):
            sc.render(u, W, H, gs.make_opts(tile_rows=(0, 4), strip_index=0, strip_count=2))


def _top_heavy_scene(n, seed, W, H):
    """The synthetic scene with most Gaussians pulled into the top quarter of the view: the
    strips' costs differ several-fold."""
    a = gs.synth_aos(n, seed, W, H).reshape(n, 80)
    rng = np.random.default_rng(seed)
    pick = rng.random(n) < 0.75
    d = -a[pick, 2]
    a[pick, 1] = d * np.tan(np.radians(30.0)) * rng.uniform(0.5, 1.0, pick.sum()).astype(np.float32)
    return a.reshape(-1)


@pytest.mark.parametrize("G", [2, 4])
def test_group_k_balanced_strips(G):
    """A device group on a top-heavy scene: after a few rebalances (every 8 frames) the strip
    boundaries have moved off the even split toward the dense rows, and every frame -- before,
    during and after the moves -- equals the single-device frame bit for bit."""
    W, H, n = 640, 480, 150_000
    aos = _top_heavy_scene(n, 7, W, H)
    u = gs.bench_uniforms(W, H)
    with gs.Context(0) as ctx:
        ref = gs.Scene(ctx, aos, n, 16).render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16))
    with gs.Context([0] * G) as gc:
        sc = gs.Scene(gc, aos, n, 16)
        o = gs.make_opts(out_format=gs.GS_OUT_RGBA_F16)
        bufs = [gs.DeviceBuffer(H * W * 8) for _ in range(6)]
        bounds = []
        for rnd in range(6):  # 6 x 6 frames in flight, waiting between rounds (statistics arrive)
            for b in bufs:
                sc.render_device(u, W, H, b.ptr.value, b.nbytes, None, o)
            gc.sync()
            bounds.append(gc.strips())
            for b in bufs:
                got = np.empty((H, W, 4), np.float16)
                b.to_host(got)
                assert np.array_equal(got.view(np.uint16), ref.view(np.uint16)), (rnd, bounds[-1])
        for b in bufs:
            b.free()
        TR = (H + 15) // 16
        even = [g * TR // G for g in range(G + 1)]
        assert list(bounds[0]) == even or bounds[0][1] < even[1]
        assert bounds[-1][1] < even[1], bounds  # the first strip shrank toward the dense top rows
        img = sc.render(u, W, H, o)  # the synchronous path on moved strips
        assert np.array_equal(img.view(np.uint16), ref.view(np.uint16))
