"""ctypes binding of libgsplat.so (include/gsplat.h) for tests and bench.py.

The user-facing host of this renderer is the reference's own TypeScript surface
(`GpuContext` / `Renderer`, ts/ + addon/); this module is the same C ABI seen from Python.
There is no CPU fallback: importing works without a GPU (the library loads), but every render
call needs a HIP device and fails loudly otherwise.
"""
import atexit
import ctypes
import os
import sys
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSPLAT_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libgsplat.so")

GS_OK = 0
GS_ACCUM_FP32, GS_ACCUM_FP16_TARGET = 0, 1
GS_OUT_RGBA_F32, GS_OUT_RGBA_F16 = 0, 1
GS_PRESENT_RGBA_F32, GS_PRESENT_RGBA_F16, GS_PRESENT_RGBA8 = 0, 1, 2
GS_OK, GS_ERR_INVALID, GS_ERR_NO_DEVICE, GS_ERR_HIP, GS_ERR_OOM, GS_ERR_UNSUPPORTED, GS_ERR_DEVICE_FAULT, \
    GS_ERR_INTERNAL = 0, -1, -2, -3, -4, -5, -6, -7

# every symbol include/gsplat.h declares
EXPORTED_SYMBOLS = (
    "gs_abi_version", "gs_last_error", "gs_device_count", "gs_ctx_create", "gs_ctx_destroy", "gs_ctx_info",
    "gs_scene_upload", "gs_scene_free", "gs_scene_count", "gs_opts_default", "gs_strip_rows", "gs_balance_strips", "gs_ctx_strips",
    "gs_render", "gs_render_device", "gs_framebuffer_alloc", "gs_framebuffer_free", "gs_framebuffer_read",
    "gs_host_register", "gs_host_unregister", "gs_readback_start", "gs_readback_wait",
    "gs_timings", "gs_timings_reset", "gs_sync", "gs_present",
    "gs_present_device", "gs_encode_png", "gs_look_at",
    "gs_perspective", "gs_camera_position", "gs_camera_from_json", "gs_pack_uniforms", "gs_synth_aos", "gs_ply_parse",
    "gs_debug_chunk1_grid", "gs_debug_sort_pairs", "gs_debug_last_order", "gs_debug_last_records", "gs_debug_last_slots",
    "gs_debug_tile_lists", "gs_debug_tile_list_check", "gs_debug_cut_margin",
)


class GsPlyInfo(ctypes.Structure):
    _fields_ = [("num_gaussians", ctypes.c_uint64), ("sh_degree", ctypes.c_int32),
                ("n_sh_coeffs", ctypes.c_int32), ("record_bytes", ctypes.c_uint64),
                ("data_offset", ctypes.c_uint64), ("vertex_stride", ctypes.c_uint64),
                ("min_pos", ctypes.c_float * 3), ("max_pos", ctypes.c_float * 3),
                ("min_pos_d", ctypes.c_double * 3), ("max_pos_d", ctypes.c_double * 3)]


class GsOpts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("accum", ctypes.c_int32),
                ("out_format", ctypes.c_int32), ("t_min", ctypes.c_float),
                ("ref_quirks", ctypes.c_int32), ("strip_index", ctypes.c_int32),
                ("strip_count", ctypes.c_int32), ("timing", ctypes.c_int32),
                ("chunk_fraction", ctypes.c_float), ("tile_row_begin", ctypes.c_int32),
                ("tile_row_end", ctypes.c_int32), ("list_split", ctypes.c_int32)]


class GsStats(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("n_vis", ctypes.c_uint64), ("k_entries", ctypes.c_uint64),
                ("k_total", ctypes.c_uint64), ("tiles_unsaturated", ctypes.c_uint32),
                ("chunk_fraction", ctypes.c_float),
                ("tile_row_begin", ctypes.c_int32), ("tile_row_end", ctypes.c_int32),
                ("tiles_x", ctypes.c_int32), ("frames", ctypes.c_int32),
                ("ms_total", ctypes.c_float), ("ms_project", ctypes.c_float),
                ("ms_sort", ctypes.c_float), ("ms_bin", ctypes.c_float),
                ("ms_tile_sort", ctypes.c_float), ("ms_ranges", ctypes.c_float),
                ("ms_composite", ctypes.c_float), ("ms_other", ctypes.c_float),
                ("k_chunk0", ctypes.c_uint32), ("k_chunk1", ctypes.c_uint32),
                ("wide_chunk0", ctypes.c_uint32), ("wide_chunk1", ctypes.c_uint32),
                ("frames_rendered", ctypes.c_uint32), ("frames_chunked", ctypes.c_uint32),
                ("frames_unsat", ctypes.c_uint32), ("frames_seeded", ctypes.c_uint32),
                ("chunk_depth", ctypes.c_float), ("list_max", ctypes.c_uint32), ("tiles_long", ctypes.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# gs_debug_last_slots row (16 words)
SLOT_DTYPE = np.dtype([("key", "<u4"), ("index", "<u4"), ("chunk", "<u4"), ("rect", "<u4"),
                       ("r0", "<f4", 4), ("r1", "<f4", 4), ("col", "<f4", 3), ("keybits", "<u4")])


class GsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("gsplat error %d: %s" % (code, msg))
        self.code = code


_lib = None
_LIVE = weakref.WeakSet()  # open contexts, closed (with their scenes) at interpreter exit


@atexit.register
def _close_all():
    for c in list(_LIVE):
        c.close()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libgsplat.so not built (run `make -C gaussian-splatting-web_amd`): %s" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        P, U64, I, F, D = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_float, ctypes.c_double
        L.gs_last_error.restype = ctypes.c_char_p
        L.gs_ctx_create.argtypes = [P, I, ctypes.POINTER(P)]
        L.gs_ctx_destroy.argtypes = [P]
        L.gs_ctx_destroy.restype = None
        L.gs_ctx_info.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(I)]
        L.gs_scene_upload.argtypes = [P, P, U64, I, ctypes.POINTER(P)]
        L.gs_scene_free.argtypes = [P]
        L.gs_scene_free.restype = None
        L.gs_scene_count.argtypes = [P]
        L.gs_scene_count.restype = U64
        L.gs_opts_default.argtypes = [ctypes.POINTER(GsOpts)]
        L.gs_opts_default.restype = None
        L.gs_strip_rows.argtypes = [I, I, I, ctypes.POINTER(I), ctypes.POINTER(I)]
        L.gs_balance_strips.argtypes = [I, I, P, P, P]
        L.gs_ctx_strips.argtypes = [P, P, I, ctypes.POINTER(I)]
        L.gs_render.argtypes = [P, P, P, I, I, ctypes.POINTER(GsOpts), P]
        L.gs_render_device.argtypes = [P, P, P, I, I, ctypes.POINTER(GsOpts), P, U64, P]
        L.gs_framebuffer_alloc.argtypes = [P, U64, ctypes.POINTER(ctypes.c_void_p)]
        L.gs_framebuffer_free.argtypes = [P, P]
        L.gs_framebuffer_read.argtypes = [P, P, P, U64]
        L.gs_host_register.argtypes = [P, P, U64]
        L.gs_host_unregister.argtypes = [P, P]
        L.gs_readback_start.argtypes = [P, P, P, U64, ctypes.POINTER(ctypes.c_uint32)]
        L.gs_readback_wait.argtypes = [P, ctypes.c_uint32]
        L.gs_timings.argtypes = [P, ctypes.POINTER(GsStats)]
        L.gs_timings_reset.argtypes = [P]
        L.gs_sync.argtypes = [P]
        L.gs_present.argtypes = [P, I, I, P]
        L.gs_present_device.argtypes = [P, P, I, I, I, I, P, U64, P]
        L.gs_encode_png.argtypes = [P, I, I, P, U64, ctypes.POINTER(U64)]
        L.gs_look_at.argtypes = [P, P, P, P]
        L.gs_perspective.argtypes = [D, D, D, D, P]
        L.gs_camera_position.argtypes = [P, P]
        L.gs_camera_from_json.argtypes = [P, P, D, D, I, I, P, P, P]
        L.gs_pack_uniforms.argtypes = [P, P, P, F, F, F, F, F, P]
        L.gs_synth_aos.argtypes = [U64, U64, I, I, P]
        L.gs_ply_parse.argtypes = [P, U64, ctypes.POINTER(GsPlyInfo), P, U64]
        L.gs_debug_chunk1_grid.argtypes = [P, I, I, ctypes.POINTER(I), ctypes.POINTER(I)]
        L.gs_debug_sort_pairs.argtypes = [P, P, P, U64, I, I]
        L.gs_debug_last_order.argtypes = [P, P, P, P, U64, ctypes.POINTER(U64)]
        L.gs_debug_last_records.argtypes = [P, P, P, U64]
        L.gs_debug_last_slots.argtypes = [P, P, P, U64, ctypes.POINTER(U64)]
        L.gs_debug_tile_lists.argtypes = [P, P, P, U64, P, U64, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        if hasattr(L, "gs_debug_tile_list_check"):  # (absent from older builds loaded for A/B runs via GSPLAT_LIB)
            L.gs_debug_tile_list_check.argtypes = [P, P, P]
            L.gs_debug_cut_margin.argtypes = [P, ctypes.c_float]
        _lib = L
    return _lib


def _check(rc):
    if rc != GS_OK:
        raise GsError(rc, lib().gs_last_error().decode(errors="replace"))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------ camera / uniforms (host)
def look_at(eye, target, up=(0.0, 1.0, 0.0)):
    out = np.zeros(16, np.float32)
    e, t, u = (np.ascontiguousarray(v, np.float64) for v in (eye, target, up))
    _check(lib().gs_look_at(_ptr(e), _ptr(t), _ptr(u), _ptr(out)))
    return out


def perspective(fovy, aspect, z_near, z_far):
    out = np.zeros(16, np.float32)
    _check(lib().gs_perspective(float(fovy), float(aspect), float(z_near), float(z_far), _ptr(out)))
    return out


def camera_position(view):
    v = np.ascontiguousarray(view, np.float32)
    out = np.zeros(3, np.float32)
    _check(lib().gs_camera_position(_ptr(v), _ptr(out)))
    return out


def camera_from_json(cam, W, H):
    """cameraFromJSON (src/camera.ts:476-503) of one cameras.json entry for a W x H canvas:
    returns (view, proj, focal) with focal = the Camera's (focalX, focalY) = (H, W)."""
    pos = np.ascontiguousarray(cam["position"], np.float64)
    rot = np.ascontiguousarray(np.asarray(cam["rotation"], np.float64).reshape(9))
    view, proj, focal = np.zeros(16, np.float32), np.zeros(16, np.float32), np.zeros(2, np.float32)
    _check(lib().gs_camera_from_json(_ptr(pos), _ptr(rot), float(cam["fx"]), float(cam["fy"]), int(W), int(H),
                                     _ptr(view), _ptr(proj), _ptr(focal)))
    return view, proj, focal


def pack_uniforms(view, proj, cam_pos=None, tan_half_fov=(0.0, 0.0), focal=(0.0, 0.0), scale_modifier=1.0):
    v = np.ascontiguousarray(view, np.float32)
    p = np.ascontiguousarray(proj, np.float32)
    c = camera_position(v) if cam_pos is None else np.ascontiguousarray(cam_pos, np.float32)
    out = np.zeros(40, np.float32)
    _check(lib().gs_pack_uniforms(_ptr(v), _ptr(p), _ptr(c), float(tan_half_fov[0]), float(tan_half_fov[1]),
                                  float(focal[0]), float(focal[1]), float(scale_modifier), _ptr(out)))
    return out


def bench_uniforms(W, H):
    """SURVEY §8d synthetic-scene camera: lookAt([0,0,0],[0,0,-1],[0,1,0]), perspective(60deg,W/H,.03,1000)."""
    view = look_at((0.0, 0.0, 0.0), (0.0, 0.0, -1.0))
    proj = perspective(1.04719755, W / H, 0.03, 1000.0)
    return pack_uniforms(view, proj, focal=(W, H))


def orbit_uniforms(W, H, k, period=60):
    """bench.py's moving camera, frame k: at the origin, yaw swinging +-25 deg and pitch +-8 deg
    around the bench view (-z), a new view every frame; part of the screen leaves the scene's
    frustum, so tiles go unsaturated and the chunk split moves."""
    a = 2 * np.pi * k / period
    yaw, pitch = np.radians(25.0) * np.sin(a), np.radians(8.0) * np.sin(2 * a)
    target = (np.sin(yaw) * np.cos(pitch), np.sin(pitch), -np.cos(yaw) * np.cos(pitch))
    view = look_at((0.0, 0.0, 0.0), target)
    return pack_uniforms(view, perspective(1.04719755, W / H, 0.03, 1000.0), focal=(W, H))


# bench.py's camera cuts: four views of the synthetic scene (Gaussians fill the
# bench view's frustum at depths 2..20 along -z), each far from the others in direction or
# position, so every frame of the cycle starts without usable saturation history
COLD_VIEWS = (
    ((0.0, 0.0, 0.0), (0.0, 0.0, -1.0)),       # the bench view
    ((0.0, 0.0, -6.0), (0.0, 0.0, -7.0)),      # from inside the scene, same direction
    ((0.0, 0.0, 0.0), (0.34, -0.1, -0.94)),    # turned 20 deg right, 6 deg down
    ((1.5, 0.8, -2.0), (-1.0, -0.5, -12.0)),   # moved and turned left
)


def cold_uniforms(W, H, k):
    """View k % 4 of bench.py's camera-cut cycle (COLD_VIEWS)."""
    eye, target = COLD_VIEWS[k % len(COLD_VIEWS)]
    view = look_at(eye, target)
    return pack_uniforms(view, perspective(1.04719755, W / H, 0.03, 1000.0), focal=(W, H))


def synth_aos(n, seed, W=1920, H=1080):
    """Seeded synthetic scene as reference AoS records (320 B each, SH degree 3)."""
    out = np.empty(n * 80, np.float32)
    _check(lib().gs_synth_aos(int(n), int(seed), int(W), int(H), _ptr(out)))
    return out


SPARSE_LOGIT_SHIFT = 4.0


def synth_aos_sparse(n, seed, W=1920, H=1080):
    """SURVEY §8d's generator with every opacity logit shifted by -SPARSE_LOGIT_SHIFT (logit ~ N(-4, 2)):
    a scene whose tiles do not saturate (at bench_uniforms, 6.1 M Gaussians at 1920x1080, no 16x16
    tile reaches T < 1e-4), so every frame renders every visible splat as one chunk -- the regime
    of a real capture's sky or background."""
    a = synth_aos(n, seed, W, H)
    a.reshape(n, 80)[:, 12] -= np.float32(SPARSE_LOGIT_SHIFT)
    return a


def parse_ply(data):
    """PackedGaussians(arrayBuffer) (src/ply.ts): .ply bytes -> (AoS records as uint8, info dict)."""
    buf = np.frombuffer(bytes(data), np.uint8)
    info = GsPlyInfo()
    _check(lib().gs_ply_parse(_ptr(buf), buf.size, ctypes.byref(info), None, 0))
    out = np.zeros(int(info.num_gaussians * info.record_bytes), np.uint8)
    _check(lib().gs_ply_parse(_ptr(buf), buf.size, ctypes.byref(info), _ptr(out), out.size))
    return out, {"numGaussians": int(info.num_gaussians), "shDegree": int(info.sh_degree),
                 "nShCoeffs": int(info.n_sh_coeffs), "record_bytes": int(info.record_bytes),
                 "min_pos": list(info.min_pos_d), "max_pos": list(info.max_pos_d)}


def present(rgba, W, H):
    src = np.ascontiguousarray(rgba, np.float32).reshape(-1)
    out = np.empty_like(src)
    _check(lib().gs_present(_ptr(src), int(W), int(H), _ptr(out)))
    return out.reshape(H, W, 4)


def encode_png(rgba8):
    """PNG bytes of an (H, W, 4) uint8 image (row 0 = top), via gs_encode_png."""
    img = np.ascontiguousarray(rgba8, np.uint8)
    H, W = img.shape[0], img.shape[1]
    n = ctypes.c_uint64()
    _check(lib().gs_encode_png(None, W, H, None, 0, ctypes.byref(n)))
    out = np.empty(n.value, np.uint8)
    _check(lib().gs_encode_png(_ptr(img), W, H, _ptr(out), n.value, ctypes.byref(n)))
    return out.tobytes()


def write_png(path, rgba8):
    with open(path, "wb") as f:
        f.write(encode_png(rgba8))


def strip_rows(H, strip_index, strip_count):
    r0, rp = ctypes.c_int(), ctypes.c_int()
    _check(lib().gs_strip_rows(int(H), int(strip_index), int(strip_count), ctypes.byref(r0), ctypes.byref(rp)))
    return r0.value, rp.value


def chunk1_grid(ctx=None, occupancy=0, cus=0):
    """(k_chunk1 grid, occupancy per CU): of a context, or for the given occupancy and CU count."""
    g, o = ctypes.c_int(), ctypes.c_int()
    _check(lib().gs_debug_chunk1_grid(ctx.handle if ctx is not None else None, int(occupancy), int(cus),
                                      ctypes.byref(g), ctypes.byref(o)))
    return g.value, o.value


def device_count():
    n = ctypes.c_int()
    _check(lib().gs_device_count(ctypes.byref(n)))
    return n.value


def make_opts(accum=GS_ACCUM_FP32, out_format=GS_OUT_RGBA_F32, t_min=1e-4, strip_index=0, strip_count=1,
              timing=0, ref_quirks=0, chunk_fraction=0.0, tile_rows=None, list_split=0):
    """gs_opts; tile_rows = (begin, end): an explicit strip of tile rows [begin, end); list_split = 1:
    long tile lists of frames with few tiles split over wave pairs (gs_opts.list_split)."""
    o = GsOpts()
    lib().gs_opts_default(ctypes.byref(o))
    o.accum, o.out_format, o.t_min = accum, out_format, t_min
    o.strip_index, o.strip_count, o.timing, o.ref_quirks = strip_index, strip_count, timing, ref_quirks
    o.chunk_fraction = chunk_fraction
    o.list_split = list_split
    if tile_rows is not None:
        o.tile_row_begin, o.tile_row_end = int(tile_rows[0]), int(tile_rows[1])
    return o


def balance_strips(bounds, cost):
    """gs_balance_strips: K-balanced tile-row boundaries from the current ones and the strips' costs."""
    b = np.ascontiguousarray(bounds, np.int32)
    c = np.ascontiguousarray(cost, np.float64)
    G = b.size - 1
    assert c.size == G
    out = np.zeros(G + 1, np.int32)
    _check(lib().gs_balance_strips(G, int(b[-1]), _ptr(b), _ptr(c), _ptr(out)))
    return out


# ------------------------------------------------------------------ context / scene / render
GATHER_KINDS = {0: "none", 1: "rccl", 2: "peer_copy"}


class Context:
    """GpuContext equivalent: one HIP device, or a device group (a list of devices: row strips on
    each, one RCCL all-gather; see gs_ctx_create)."""

    def __init__(self, device=0):
        self.handle = ctypes.c_void_p()
        self.scenes = weakref.WeakSet()
        devs = list(device) if isinstance(device, (list, tuple)) else [int(device)]
        dev = (ctypes.c_int * len(devs))(*devs)
        _check(lib().gs_ctx_create(dev, len(devs), ctypes.byref(self.handle)))
        _LIVE.add(self)

    def info(self):
        """(devices driven, gather kind: 'none' | 'rccl' | 'peer_copy')."""
        nd, g = ctypes.c_int(), ctypes.c_int()
        _check(lib().gs_ctx_info(self.handle, ctypes.byref(nd), ctypes.byref(g)))
        return nd.value, GATHER_KINDS[g.value]

    def strips(self):
        """A device group's strip boundaries (tile rows, G + 1 values; empty on one device)."""
        n = ctypes.c_int()
        _check(lib().gs_ctx_strips(self.handle, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.int32)
        _check(lib().gs_ctx_strips(self.handle, _ptr(out), n.value, ctypes.byref(n)))
        return out

    def close(self):
        # scenes first: the C side frees attached scenes with the context anyway, but the
        # Python objects must forget their handles before that happens
        for sc in list(self.scenes):
            sc.close()
        if self.handle:
            lib().gs_ctx_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        if not sys.is_finalizing():
            self.close()

    def sync(self):
        _check(lib().gs_sync(self.handle))

    def timings(self):
        st = GsStats()
        _check(lib().gs_timings(self.handle, ctypes.byref(st)))
        return st.as_dict()

    def set_cut_margin(self, margin):
        """gs_debug_cut_margin: 0 default, < 0 per-tile cut off, > 0 its depth margin."""
        _check(lib().gs_debug_cut_margin(self.handle, float(margin)))

    def timings_reset(self):
        _check(lib().gs_timings_reset(self.handle))

    def present_device(self, fb_ptr, fb_format, W, H, out_format, out_ptr, out_bytes, stream_ptr=None):
        """PostProcessRenderer on the device (gs_present_device): framebuffer -> presented image."""
        _check(lib().gs_present_device(self.handle, fb_ptr, int(fb_format), int(W), int(H), int(out_format),
                                       out_ptr, int(out_bytes), stream_ptr))

    def sort_pairs(self, keys, vals, begin_bit=0, end_bit=32):
        k = np.array(keys, np.uint32, copy=True)
        v = np.array(vals, np.uint32, copy=True)
        assert k.shape == v.shape
        _check(lib().gs_debug_sort_pairs(self.handle, _ptr(k), _ptr(v), k.size, begin_bit, end_bit))
        return k, v


class Scene:
    def __init__(self, ctx, aos, n, n_sh=16):
        self.ctx = ctx
        self.n = int(n)
        buf = np.ascontiguousarray(np.frombuffer(aos, np.uint8) if not isinstance(aos, np.ndarray) else aos)
        assert buf.nbytes == self.n * (64 + 16 * n_sh), (buf.nbytes, n, n_sh)
        self.handle = ctypes.c_void_p()
        _check(lib().gs_scene_upload(ctx.handle, _ptr(buf), self.n, int(n_sh), ctypes.byref(self.handle)))
        ctx.scenes.add(self)

    def close(self):
        if self.handle and self.ctx.handle:
            lib().gs_scene_free(self.handle)
        self.handle = ctypes.c_void_p()

    def __del__(self):
        if not sys.is_finalizing():
            self.close()

    def render(self, uniforms, W, H, opts=None):
        o = opts if opts is not None else make_opts()
        if o.tile_row_end > 0:
            rows = min(16 * o.tile_row_end, H) - 16 * o.tile_row_begin
        else:
            rows = H if o.strip_count <= 1 else strip_rows(H, o.strip_index, o.strip_count)[1]
        if o.out_format == GS_OUT_RGBA_F16:
            out = np.empty((rows, W, 4), np.float16)
        else:
            out = np.empty((rows, W, 4), np.float32)
        u = np.ascontiguousarray(uniforms, np.float32)
        _check(lib().gs_render(self.ctx.handle, self.handle, _ptr(u), int(W), int(H), ctypes.byref(o), _ptr(out)))
        return out

    def render_device(self, uniforms, W, H, out_ptr, out_bytes, stream_ptr=None, opts=None):
        o = opts if opts is not None else make_opts()
        u = np.ascontiguousarray(uniforms, np.float32)
        _check(lib().gs_render_device(self.ctx.handle, self.handle, _ptr(u), int(W), int(H), ctypes.byref(o),
                                      ctypes.c_void_p(out_ptr), int(out_bytes),
                                      ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def last_order(self):
        n = ctypes.c_uint64()
        _check(lib().gs_debug_last_order(self.ctx.handle, self.handle, None, None, 0, ctypes.byref(n)))
        keys = np.empty(n.value, np.uint32)
        idx = np.empty(n.value, np.uint32)
        _check(lib().gs_debug_last_order(self.ctx.handle, self.handle, _ptr(keys), _ptr(idx), n.value,
                                         ctypes.byref(n)))
        return keys, idx

    def last_slots(self):
        """Composite slots of the last frame (gs_debug_last_slots): structured array."""
        n = ctypes.c_uint64()
        _check(lib().gs_debug_last_slots(self.ctx.handle, self.handle, None, 0, ctypes.byref(n)))
        out = np.zeros((n.value, 16), np.uint32)
        _check(lib().gs_debug_last_slots(self.ctx.handle, self.handle, _ptr(out), n.value, ctypes.byref(n)))
        return out.view(SLOT_DTYPE).reshape(-1)

    def tile_lists(self):
        """(ranges [n_tiles, 2], entries [n, 2] = (key, reference index)) the composite consumed."""
        nt, ne = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().gs_debug_tile_lists(self.ctx.handle, self.handle, None, 0, None, 0, ctypes.byref(nt),
                                         ctypes.byref(ne)))
        rg = np.zeros((nt.value, 2), np.uint32)
        en = np.zeros((ne.value, 2), np.uint32)
        _check(lib().gs_debug_tile_lists(self.ctx.handle, self.handle, _ptr(rg), nt.value, _ptr(en), ne.value,
                                         ctypes.byref(nt), ctypes.byref(ne)))
        return rg, en

    def tile_list_check(self):
        """Structural check of the last one-chunk frame's tile lists (gs_debug_tile_list_check): dict
        of entries, dup (a (tile, Gaussian) pair listed twice), order (adjacent entries not strictly
        ascending by (key, index)), gaps (a list not starting where the previous one ends), bad
        (an entry that is not a visible splat's slot).  A correct frame has all but entries 0."""
        out = (ctypes.c_uint64 * 5)()
        _check(lib().gs_debug_tile_list_check(self.ctx.handle, self.handle, out))
        return dict(zip(("entries", "dup", "order", "gaps", "bad"), (int(v) for v in out)))

    def last_records(self):
        out = np.empty((self.n, 16), np.float32)
        _check(lib().gs_debug_last_records(self.ctx.handle, self.handle, _ptr(out), self.n))
        return out


# ------------------------------------------------------------------ raw device memory (no torch)
class DeviceBuffer:
    """hipMalloc'd device memory for frames kept on the GPU (bench.py at N=1 needs no torch)."""
    _hip = None

    def __init__(self, nbytes):
        if DeviceBuffer._hip is None:
            h = ctypes.CDLL("libamdhip64.so")
            h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
            h.hipFree.argtypes = [ctypes.c_void_p]
            h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            DeviceBuffer._hip = h
        self.nbytes = int(nbytes)
        self.ptr = ctypes.c_void_p()
        rc = DeviceBuffer._hip.hipMalloc(ctypes.byref(self.ptr), self.nbytes)
        if rc != 0:
            raise GsError(-4, "hipMalloc(%d) failed: %d" % (self.nbytes, rc))

    def to_host(self, out):
        rc = DeviceBuffer._hip.hipMemcpy(_ptr(out), self.ptr, min(out.nbytes, self.nbytes), 2)
        if rc != 0:
            raise GsError(-3, "hipMemcpy D2H failed: %d" % rc)
        return out

    def free(self):
        if self.ptr:
            DeviceBuffer._hip.hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        if not sys.is_finalizing():
            self.free()
