"""Present + readback: PostProcessRenderer (src/post_process_render.ts:54-77)
on the device, and the PNG encoder used for visual diffs.

CPU: gs_encode_png decodes (PIL, and an independent zlib parse) to the exact input pixels.
Both against the oracle's restatement (oracle/gs_oracle.cpp or_present, pow(a, 4) as powf): the
flip and RGB bit-exact, alpha within 4 ulp (WGSL's pow is exp2(4 log2 a), a few ulp; here it is
evaluated as (a^2)^2).
GPU: gs_present_device equals the host gs_present bit for bit (f32 out), or that result rounded
to f16 (the reference's rgba16float canvas) / unorm8, from f32 and f16 framebuffers."""
import os
import struct
import sys
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-web_amd"))
import gsplat_amd as gs  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as orc  # noqa: E402

ALPHA_ULP = 4  # stated tolerance on the remapped alpha vs the oracle's powf


def assert_present_matches_oracle(got, fb, W, H):
    ref = orc.present(fb, W, H)
    assert np.array_equal(got[..., :3].view(np.uint32), ref[..., :3].view(np.uint32))
    ulp = np.abs(got[..., 3].view(np.int32).astype(np.int64) - ref[..., 3].view(np.int32).astype(np.int64))
    assert int(ulp.max()) <= ALPHA_ULP, int(ulp.max())
    # the >= 0.99 branch and saturation are exact
    hi = ref[..., 3] >= 0.99
    assert np.array_equal(got[..., 3][hi], ref[..., 3][hi])


def test_present_host_vs_oracle():
    W, H = 257, 131
    rng = np.random.default_rng(5)
    fb = rng.random((H, W, 4), dtype=np.float32)
    a = fb[..., 3].reshape(-1)
    a[:4096] = np.linspace(0.0, 0.7, 4096, dtype=np.float32)  # a ramp through both branches
    a[4096:4106] = [0.0, -0.0, 1e-30, 0.66, 0.6599, 0.66001, 1.0, 2.0, -1.0, 0.65999997]
    got = gs.present(fb, W, H)
    assert_present_matches_oracle(got, fb, W, H)
    assert np.array_equal(got[0, :, :3], fb[H - 1, :, :3])  # row 0 of the canvas = the framebuffer's last


def _decode_png_stored(data):
    """Minimal PNG reader for 8-bit RGBA, filter 0 (independent of PIL)."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, W, H = 8, b"", None, None
    while pos < len(data):
        ln, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + ln]
        crc, = struct.unpack(">I", data[pos + 8 + ln:pos + 12 + ln])
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc, typ
        if typ == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert (depth, ctype) == (8, 6)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + ln
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(H, 1 + 4 * W)
    assert np.all(rows[:, 0] == 0)
    return rows[:, 1:].reshape(H, W, 4)


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (64, 48), (300, 400)])
def test_png_roundtrip(shape):
    H, W = shape
    rng = np.random.default_rng(H * 1000 + W)
    img = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    png = gs.encode_png(img)
    assert np.array_equal(_decode_png_stored(png), img)
    from io import BytesIO
    try:
        from PIL import Image
    except ImportError:
        return
    im = Image.open(BytesIO(png))
    assert im.mode == "RGBA" and im.size == (W, H)
    assert np.array_equal(np.asarray(im), img)


def test_png_multi_block():
    """Raw stream above one stored block (65535 B) splits into several."""
    img = np.arange(200 * 120 * 4, dtype=np.uint32).astype(np.uint8).reshape(120, 200, 4)
    assert np.array_equal(_decode_png_stored(gs.encode_png(img)), img)


def test_png_bad_args():
    n = __import__("ctypes").c_uint64()
    assert gs.lib().gs_encode_png(None, 0, 4, None, 0, __import__("ctypes").byref(n)) == gs.GS_ERR_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("fb_format", [gs.GS_OUT_RGBA_F32, gs.GS_OUT_RGBA_F16])
def test_present_device_matches_host(gpu_ctx, fb_format):
    W, H = 320, 200
    aos = gs.synth_aos(50_000, 4, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, 50_000, 16)
    bpp = 16 if fb_format == gs.GS_OUT_RGBA_F32 else 8
    fb = gs.DeviceBuffer(W * H * bpp)
    sc.render_device(u, W, H, fb.ptr.value, fb.nbytes, opts=gs.make_opts(out_format=fb_format))
    gpu_ctx.sync()
    fb_host = np.empty((H, W, 4), np.float32 if bpp == 16 else np.float16)
    fb.to_host(fb_host)
    ref = gs.present(fb_host.astype(np.float32), W, H)  # host PostProcessRenderer
    assert ref[..., 3].max() > 0.5  # a non-trivial image
    assert_present_matches_oracle(ref, fb_host.astype(np.float32), W, H)
    for fmt, dt in ((gs.GS_PRESENT_RGBA_F32, np.float32), (gs.GS_PRESENT_RGBA_F16, np.float16),
                    (gs.GS_PRESENT_RGBA8, np.uint8)):
        out = gs.DeviceBuffer(W * H * 4 * np.dtype(dt).itemsize)
        gpu_ctx.present_device(fb.ptr, fb_format, W, H, fmt, out.ptr, out.nbytes)
        gpu_ctx.sync()
        got = np.empty((H, W, 4), dt)
        out.to_host(got)
        if dt == np.float32:
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
            assert_present_matches_oracle(got, fb_host.astype(np.float32), W, H)
        elif dt == np.float16:
            assert np.array_equal(got.view(np.uint16), ref.astype(np.float16).view(np.uint16))
        else:
            assert np.array_equal(got, np.rint(np.clip(ref, 0.0, 1.0) * 255.0).astype(np.uint8))
        out.free()
    bad = gs.lib().gs_present_device(gpu_ctx.handle, fb.ptr, fb_format, W, H, 7, fb.ptr, fb.nbytes, None)
    assert bad == gs.GS_ERR_INVALID
    fb.free()
    sc.close()


@pytest.mark.gpu
def test_framebuffer_abi_roundtrip(gpu_ctx):
    """gs_framebuffer_alloc / gs_render_device / gs_framebuffer_read / gs_framebuffer_free: a
    device-resident frame read back equals the host-output render of the same frame."""
    import ctypes
    W, H, n = 256, 160, 30_000
    aos = gs.synth_aos(n, 12, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    L = gs.lib()
    dev = ctypes.c_void_p()
    assert L.gs_framebuffer_alloc(gpu_ctx.handle, W * H * 16, ctypes.byref(dev)) == gs.GS_OK
    assert L.gs_framebuffer_alloc(gpu_ctx.handle, 0, ctypes.byref(ctypes.c_void_p())) == gs.GS_ERR_INVALID
    for _ in range(3):  # frames in flight into the same buffer
        sc.render_device(u, W, H, dev.value, W * H * 16)
    got = np.empty((H, W, 4), np.float32)
    assert L.gs_framebuffer_read(gpu_ctx.handle, dev, got.ctypes.data_as(ctypes.c_void_p), got.nbytes) == gs.GS_OK
    assert np.array_equal(got, sc.render(u, W, H))
    # a read past the allocation, or of memory the context did not allocate, is refused
    big = np.empty(W * H * 16 + 64, np.uint8)
    assert L.gs_framebuffer_read(gpu_ctx.handle, dev, big.ctypes.data_as(ctypes.c_void_p), big.nbytes) == \
        gs.GS_ERR_INVALID
    tail = ctypes.c_void_p(dev.value + W * H * 8)
    assert L.gs_framebuffer_read(gpu_ctx.handle, tail, big.ctypes.data_as(ctypes.c_void_p), W * H * 8) == gs.GS_OK
    assert L.gs_framebuffer_read(gpu_ctx.handle, tail, big.ctypes.data_as(ctypes.c_void_p), W * H * 8 + 1) == \
        gs.GS_ERR_INVALID
    other = gs.DeviceBuffer(1024)
    assert L.gs_framebuffer_read(gpu_ctx.handle, other.ptr, big.ctypes.data_as(ctypes.c_void_p), 16) == \
        gs.GS_ERR_INVALID
    other.free()
    assert L.gs_framebuffer_free(gpu_ctx.handle, dev) == gs.GS_OK


@pytest.mark.gpu
def test_async_readback(gpu_ctx):
    """gs_host_register / gs_readback_start / gs_readback_wait: frames rendered alternately into two
    framebuffers and copied out asynchronously (the Node Renderer's host-readback loop) equal the
    synchronous host-output renders of the same views; bounds and tickets are checked."""
    import ctypes
    W, H, n = 256, 160, 30_000
    aos = gs.synth_aos(n, 13, W, H)
    views = [gs.orbit_uniforms(W, H, k) for k in range(6)]
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    L = gs.lib()
    c = gpu_ctx.handle
    nb = W * H * 16
    devs = [ctypes.c_void_p(), ctypes.c_void_p()]
    for d in devs:
        assert L.gs_framebuffer_alloc(c, nb, ctypes.byref(d)) == gs.GS_OK
    hosts = [np.zeros((H, W, 4), np.float32) for _ in range(3)]
    for h in hosts:
        assert L.gs_host_register(c, h.ctypes.data_as(ctypes.c_void_p), h.nbytes) == gs.GS_OK
    tickets = []
    for k, u in enumerate(views):
        if k >= 2:  # framebuffer k % 2 is rendered again only after its last copy landed
            assert L.gs_readback_wait(c, tickets[k - 2]) == gs.GS_OK
        sc.render_device(u, W, H, devs[k % 2].value, nb)
        t = ctypes.c_uint32()
        assert L.gs_readback_start(c, devs[k % 2], hosts[k % 3].ctypes.data_as(ctypes.c_void_p), nb,
                                   ctypes.byref(t)) == gs.GS_OK
        tickets.append(t.value)
    for k in (len(views) - 2, len(views) - 1):
        assert L.gs_readback_wait(c, tickets[k]) == gs.GS_OK
    ref = gs.Scene(gpu_ctx, aos, n, 16)
    for k in range(len(views) - 3, len(views)):
        assert np.array_equal(hosts[k % 3], ref.render(views[k], W, H)), k
    # a copy past the framebuffer, an unknown ticket, an unregistered buffer are refused
    assert L.gs_readback_start(c, devs[0], hosts[0].ctypes.data_as(ctypes.c_void_p), nb + 1,
                               ctypes.byref(ctypes.c_uint32())) == gs.GS_ERR_INVALID
    assert L.gs_readback_wait(c, 1_000_000) == gs.GS_ERR_INVALID
    spare = np.zeros(16, np.float32)
    assert L.gs_host_unregister(c, spare.ctypes.data_as(ctypes.c_void_p)) == gs.GS_ERR_INVALID
    for h in hosts:
        assert L.gs_host_unregister(c, h.ctypes.data_as(ctypes.c_void_p)) == gs.GS_OK
    for d in devs:
        assert L.gs_framebuffer_free(c, d) == gs.GS_OK
