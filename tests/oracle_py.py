"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the parity checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

SPLAT_DTYPE = np.dtype([
    ("key", "<u4"), ("visible", "<i4"), ("clip", "<f4", 4), ("c", "<f4", 2), ("e1", "<f4", 2),
    ("e2", "<f4", 2), ("col", "<f4", 3), ("op", "<f4"), ("rect", "<i4", 4), ("ntiles", "<i4"),
    ("view_z", "<f4"),
])
assert SPLAT_DTYPE.itemsize == 88


class OrStats(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("n_vis", ctypes.c_uint64), ("k_tiles", ctypes.c_uint64),
                ("blends", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            raise ImportError("oracle not built: make -C oracle")
        L = ctypes.CDLL(ORACLE_PATH)
        P, U64, I, F = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_float
        L.or_sortable_key.argtypes = [F]
        L.or_sortable_key.restype = ctypes.c_uint32
        L.or_project.argtypes = [P, U64, I, P, I, I, P]
        L.or_stable_sort_pairs.argtypes = [P, P, U64]
        L.or_stable_sort_pairs.restype = None
        L.or_keyed_slots.argtypes = [U64]
        L.or_keyed_slots.restype = U64
        L.or_draw_order.argtypes = [P, U64, I, P, P, P]
        L.or_composite.argtypes = [P, P, U64, I, I, I, F, P, P]
        L.or_render.argtypes = [P, U64, I, P, I, I, I, F, I, P, P, P, ctypes.POINTER(OrStats)]
        L.or_num_threads.restype = I
        L.or_present.argtypes = [P, I, I, P]
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def sortable_key(f):
    return lib().or_sortable_key(float(np.float32(f)))


def project(aos, n, n_sh, uniforms, W, H):
    a = np.ascontiguousarray(aos)
    u = np.ascontiguousarray(uniforms, np.float32)
    out = np.zeros(n, SPLAT_DTYPE)
    rc = lib().or_project(_p(a), n, n_sh, _p(u), W, H, _p(out))
    assert rc == 0, rc
    return out


def stable_sort_pairs(keys, vals):
    k = np.array(keys, np.uint32, copy=True)
    v = np.array(vals, np.uint32, copy=True)
    lib().or_stable_sort_pairs(_p(k), _p(v), k.size)
    return k, v


def keyed_slots(n):
    return lib().or_keyed_slots(n)


def render(aos, n, n_sh, uniforms, W, H, accum=0, t_min=1e-4, quirk=0, state=None):
    """Full-frame oracle render.  Returns (H x W x 4 float32 image, stats dict)."""
    a = np.ascontiguousarray(aos)
    u = np.ascontiguousarray(uniforms, np.float32)
    out = np.zeros((H, W, 4), np.float32)
    st = OrStats()
    if quirk:
        if state is None:
            state = (np.zeros(n, np.uint32), np.zeros(n, np.uint32))
        sk, sv = state
        rc = lib().or_render(_p(a), n, n_sh, _p(u), W, H, accum, t_min, 1, _p(sk), _p(sv), _p(out),
                             ctypes.byref(st))
    else:
        rc = lib().or_render(_p(a), n, n_sh, _p(u), W, H, accum, t_min, 0, None, None, _p(out),
                             ctypes.byref(st))
    assert rc == 0, rc
    return out, {"n": st.n, "n_vis": st.n_vis, "k_tiles": st.k_tiles, "blends": st.blends}


def num_threads():
    return lib().or_num_threads()


def present(fb, W, H):
    """PostProcessRenderer's pass (src/post_process_render.ts:62-77) on a W x H RGBA f32 framebuffer."""
    a = np.ascontiguousarray(fb, np.float32)
    out = np.empty((H, W, 4), np.float32)
    assert lib().or_present(_p(a), W, H, _p(out)) == 0
    return out
