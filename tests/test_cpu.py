"""CPU-only tests (no GPU): oracle vs the reference's own fixtures, host logic, the C ABI surface."""
import hashlib
import json
import os
import re
import sys

import numpy as np
import pytest

import oracle_py as orc
from conftest import GOLDEN, ROOT, camera, load_scene

gs = pytest.importorskip("gsplat_amd")


# --------------------------------------------------------------------------- depth key (a4)
KNOWN_KEYS = [(-2.0, 0x40000001), (-1.0, 0x3F800001), (-0.5, 0x3F000001), (-0.0, 0x00000001),
              (0.0, 0x80000000), (0.5, 0xBF000000), (1.0, 0xBF800000), (2.0, 0xC0000000)]


@pytest.mark.parametrize("f,k", KNOWN_KEYS)
def test_depth_key_known_answers(f, k):
    """float_to_sortable_uint, src/shaders.ts:36-40."""
    assert orc.sortable_key(f) == k


def test_depth_key_order_closest_first():
    z = -np.array([0.5, 1.0, 2.0, 3.5, 10.0], np.float32)  # -z forward: closer = smaller |z|
    keys = [orc.sortable_key(v) for v in z]
    assert keys == sorted(keys)
    zp = np.array([0.5, 1.0, 2.0], np.float32)  # +z forward (cam.json): closer = smaller z
    kp = [orc.sortable_key(v) for v in zp]
    assert kp == sorted(kp) and min(kp) > max(keys)


# --------------------------------------------------------------------------- layout (a1, a2)
def test_record_layout_matches_reference_packer():
    """Offsets produced by the reference's own packing.ts (gen_ref_fixtures.py)."""
    lay = json.load(open(os.path.join(GOLDEN, "layout.json")))
    for nsh, size in (("1", 80), ("4", 128), ("9", 208), ("16", 320)):
        r = lay["record"][nsh]
        assert r["size"] == size == 64 + 16 * int(nsh)
        assert (r["position"], r["logScale"], r["rotQuat"], r["opacityLogit"], r["sh0"]) == (0, 16, 32, 48, 64)
        assert r["shLastBlue"] == 64 + 16 * (int(nsh) - 1) + 8
    uni = lay["uniforms"]
    assert uni["size"] == 160
    assert (uni["viewMatrix"], uni["view_m01"], uni["view_m10"], uni["projMatrix"]) == (0, 4, 16, 64)
    assert (uni["cameraPosition"], uni["tanHalfFovX"], uni["tanHalfFovY"], uni["focalX"], uni["focalY"],
            uni["scaleModifier"]) == (128, 140, 144, 148, 152, 156)


def test_pack_uniforms_layout():
    v = np.arange(16, dtype=np.float32)
    p = np.arange(16, 32, dtype=np.float32)
    u = gs.pack_uniforms(v, p, cam_pos=(1, 2, 3), tan_half_fov=(4, 5), focal=(6, 7), scale_modifier=8)
    b = u.view(np.uint8)
    assert b.size == 160
    f = b.view(np.float32)
    assert np.array_equal(f[:16], v) and np.array_equal(f[16:32], p)
    assert list(f[32:40]) == [1, 2, 3, 4, 5, 6, 7, 8]


# --------------------------------------------------------------------------- PLY ingest fixtures
@pytest.mark.parametrize("name", ["simple", "pc_short", "m3splat"])
def test_ply_fixture_hashes(name):
    meta = json.load(open(os.path.join(GOLDEN, "ply_meta.json")))[name]
    blob = open(os.path.join(GOLDEN, name + ".aos.bin"), "rb").read()
    assert hashlib.sha256(blob).hexdigest() == meta["sha256"]
    assert len(blob) == meta["numGaussians"] * (64 + 16 * meta["nShCoeffs"])


@pytest.mark.parametrize("name", ["simple", "pc_short", "m3splat"])
def test_ply_fixture_semantics(name):
    """The reference-ingested records obey ply.ts's preprocessing: unit quaternion stored as
    (-x,-y,-z,w), scale = |exp(s)| > 0, padding words zero."""
    aos, n, nsh = load_scene(name)
    rec = aos.view(np.float32).reshape(n, 16 + 4 * nsh)
    q = rec[:, 8:12].astype(np.float64)
    assert np.allclose((q ** 2).sum(1), 1.0, atol=1e-6)
    assert np.all(rec[:, 4:7] > 0)
    assert np.all(rec[:, 3] == 0) and np.all(rec[:, 7] == 0) and np.all(rec[:, 13:16] == 0)
    assert np.all(rec[:, 16 + 4 * np.arange(nsh) + 3] == 0)


# --------------------------------------------------------------------------- camera (a2, WM)
def test_camera_matches_wgpu_matrix_fixtures():
    """gs_look_at / gs_perspective / gs_camera_position bit-exact vs wgpu-matrix 2.9.1 run by node."""
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    n = 0
    for c in cams:
        if c["kind"] != "lookat":
            continue
        v = gs.look_at(c["eye"], c["target"])
        p = gs.perspective(1.04719755, c["W"] / c["H"], 0.03, 1000.0)
        pos = gs.camera_position(v)
        assert np.array_equal(v.view(np.uint32), np.array(c["view"], np.uint32)), c["name"]
        assert np.array_equal(p.view(np.uint32), np.array(c["proj"], np.uint32)), c["name"]
        assert np.array_equal(pos.view(np.uint32), np.array(c["campos"], np.uint32)), c["name"]
        n += 1
    assert n >= 60


def test_camera_position_json_cameras():
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    for c in cams:
        if c["kind"] == "json":
            v = np.array(c["view"], np.uint32).view(np.float32)
            pos = gs.camera_position(v)
            assert np.array_equal(pos.view(np.uint32), np.array(c["campos"], np.uint32)), c["name"]


def test_camera_from_json_matches_fixtures():
    """gs_camera_from_json bit-exact vs camera.ts cameraFromJSON run with wgpu-matrix 2.9.1 by node."""
    cams = [c for c in json.load(open(os.path.join(GOLDEN, "cameras.json"))) if c["kind"] == "json"]
    assert len(cams) >= 8
    for c in cams:
        v, p, f = gs.camera_from_json(c["json"], c["W"], c["H"])
        assert np.array_equal(v.view(np.uint32), np.array(c["view"], np.uint32)), c["name"]
        assert np.array_equal(p.view(np.uint32), np.array(c["proj"], np.uint32)), c["name"]
        assert np.array_equal(gs.camera_position(v).view(np.uint32), np.array(c["campos"], np.uint32))
        assert f.tolist() == [c["H"], c["W"]]
    with pytest.raises(gs.GsError):
        gs.camera_from_json(cams[0]["json"], 0, 10)


# --------------------------------------------------------------------------- synthetic scenes
def test_synth_deterministic_and_hash():
    a = gs.synth_aos(1000, 1, 1920, 1080)
    b = gs.synth_aos(1000, 1, 1920, 1080)
    assert np.array_equal(a, b)
    h = hashlib.sha256(a.tobytes()).hexdigest()
    ref = json.load(open(os.path.join(GOLDEN, "synth_hashes.json")))
    assert h == ref["n1000_seed1_1920x1080"]


def test_synth_distribution():
    n = 20000
    rec = gs.synth_aos(n, 6, 1920, 1080).reshape(n, 80)
    d = -rec[:, 2]
    assert 2 <= d.min() and d.max() < 20
    t30 = np.tan(np.pi / 6)
    assert np.all(np.abs(rec[:, 1]) <= 1.1 * d * t30 + 1e-4)
    assert np.all(np.abs(rec[:, 0]) <= 1.1 * d * t30 * 1920 / 1080 + 1e-4)
    ls = np.log(rec[:, 4:7])
    assert -5.5 - 1e-5 <= ls.min() and ls.max() <= -3.5 + 1e-5
    assert np.allclose((rec[:, 8:12].astype(np.float64) ** 2).sum(1), 1, atol=1e-6)
    assert abs(rec[:, 12].std() - 2.0) < 0.1 and abs(rec[:, 16].std() - 1.0) < 0.05
    assert abs(rec[:, 20].std() - 0.15) < 0.01


# --------------------------------------------------------------------------- oracle properties
def test_oracle_stable_sort():
    rng = np.random.default_rng(0)
    k = rng.integers(0, 50, 10000).astype(np.uint32)
    v = np.arange(10000, dtype=np.uint32)
    ks, vs = orc.stable_sort_pairs(k, v)
    o = np.argsort(k, kind="stable")
    assert np.array_equal(ks, k[o]) and np.array_equal(vs, v[o])


def test_oracle_keyed_slots_reference_grid():
    """src/renderer.ts:306 dispatchWorkgroups(max(N/8,8)) x workgroup 8, WebIDL truncation."""
    assert orc.keyed_slots(62) == 62
    assert orc.keyed_slots(100) == 96
    assert orc.keyed_slots(3) == 3
    assert orc.keyed_slots(1_000_001) == 1_000_000


def test_oracle_isotropic_splat_is_dropped():
    """Reference quirk (src/simple_render.ts:205-216, :309): off = 0 and lambda1 = d1 make
    safe_normalize_v2((0,0)) NaN, so a screen-isotropic splat produces no fragment."""
    W, H = 64, 64
    aos = np.zeros(80, np.float32)
    aos[0:3] = (0.0, 0.0, -5.0)
    aos[4:7] = 0.05
    aos[8:12] = (0.0, 0.0, 0.0, 1.0)
    aos[12] = 3.0
    img, st = orc.render(aos.view(np.uint8), 1, 16, gs.bench_uniforms(W, H), W, H)
    assert st["n_vis"] == 0 and not img.any()


def test_oracle_composite_single_splat_closed_form():
    """One anisotropic splat: pixel value = col * op * exp(-(u^2+v^2)) where covered."""
    W, H = 64, 64
    aos = np.zeros(80, np.float32)
    aos[0:3] = (0.0, 0.0, -5.0)
    aos[4:7] = (0.06, 0.03, 0.04)
    q = np.array([0.3, -0.2, 0.1, 0.9])
    aos[8:12] = q / np.linalg.norm(q)
    aos[12] = 3.0
    aos[16:19] = 1.0
    u = gs.bench_uniforms(W, H)
    img, st = orc.render(aos.view(np.uint8), 1, 16, u, W, H, t_min=0.0)
    sp = orc.project(aos.view(np.uint8), 1, 16, u, W, H)[0]
    assert st["n_vis"] == 1 and sp["visible"]
    op = 1 / (1 + np.exp(-3.0))
    yy, xx = np.mgrid[0:H, 0:W] + 0.5
    dx, dy = xx - sp["c"][0], yy - sp["c"][1]
    uu = (dx * sp["e1"][0] + dy * sp["e1"][1]) / (sp["e1"] ** 2).sum()
    vv = (dx * sp["e2"][0] + dy * sp["e2"][1]) / (sp["e2"] ** 2).sum()
    a = op * np.exp(-(uu ** 2 + vv ** 2))
    a[(np.abs(uu) > 2) | (np.abs(vv) > 2) | (a < 1 / 255)] = 0
    assert np.allclose(img[..., 3], a, atol=2e-6)
    col = sp["col"][0]
    assert np.allclose(img[..., 0], col * a, atol=2e-6)


def test_oracle_fp16_mode_saturates():
    """rgba16float target: dst.a rounds to 1.0 once alpha > 1 - 2^-12 (implicit early stop)."""
    aos, n, nsh = load_scene("pc_short")
    u, _ = camera("pc_short_behind", 256, 256)
    img16, _ = orc.render(aos, n, nsh, u, 256, 256, accum=1, t_min=0.0)
    img32, _ = orc.render(aos, n, nsh, u, 256, 256, accum=0, t_min=0.0)
    assert np.array_equal(img16.astype(np.float16).astype(np.float32), img16)
    d = np.abs(img16 - img32)
    assert ((d ** 2).mean()) < 1e-5 and (d.max(-1) <= 2e-2).mean() >= 0.999


def test_oracle_early_stop_bound():
    """t_min = 1e-4 changes a pixel by at most t_min * max colour."""
    aos, n, nsh = load_scene("pc_short")
    u, _ = camera("pc_short_behind", 256, 256)
    a, _ = orc.render(aos, n, nsh, u, 256, 256, t_min=1e-4)
    b, _ = orc.render(aos, n, nsh, u, 256, 256, t_min=0.0)
    sp = orc.project(aos, n, nsh, u, 256, 256)
    assert np.abs(a - b).max() <= 1e-4 * max(1.0, sp["col"].max()) + 1e-6


def test_present_pass():
    W, H = 5, 4
    img = np.random.default_rng(1).random((H, W, 4)).astype(np.float32)
    out = gs.present(img, W, H)
    assert np.array_equal(out[..., :3], img[::-1, :, :3])
    a = np.clip(img[::-1, :, 3] * 1.5, 0, 1)
    a = np.where(a < 0.99, a ** 4, a)
    assert np.allclose(out[..., 3], a, rtol=1e-6)


def test_strip_geometry_covers_image():
    from gsplat_amd.strips import strip_geometry
    for H in (1, 15, 16, 17, 720, 1080, 2160):
        for G in (1, 2, 3, 4, 8):
            rows = []
            for g in range(G):
                r0, rp, t0, t1 = strip_geometry(H, g, G)
                assert gs.strip_rows(H, g, G) == (r0, rp)
                rows += list(range(t0 * 16, min(t1 * 16, H)))
                assert r0 == g * rp or t0 == t1
            assert rows == list(range(H))


# --------------------------------------------------------------------------- C ABI surface
def test_abi_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "gsplat.h")).read()
    declared = set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(gs_\w+)\s*\(", hdr, re.M))
    assert declared == set(gs.EXPORTED_SYMBOLS), declared ^ set(gs.EXPORTED_SYMBOLS)
    L = gs.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.gs_abi_version() == 5


def test_abi_rejects_without_device():
    """No HIP device here: GpuContext.create must reject, never fall back to a CPU path."""
    if gs.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(gs.GsError) as e:
        gs.Context(0)
    assert e.value.code == -2


def test_kernel_resources_no_scratch():
    """Per-frame kernels in the built library use no scratch memory (a spill or a copied kernel
    argument costs a scratch setup per launch, measured +7-10 us on k_chunk1), and the composite
    keeps the register budget of 5 waves per SIMD it was tuned for."""
    import shutil
    lib = os.path.join(ROOT, "gaussian-splatting-web_amd", "lib", "libgsplat.so")
    if not os.path.exists(lib) or not shutil.which("objcopy") or \
            not os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler"):
        pytest.skip("library or ROCm binutils not present")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import kernel_resources
    res = kernel_resources(lib)
    # every instantiation of each per-frame kernel (names carry their template arguments)
    frame = ["k_cull<", "k_project<", "k_bin_count<", "k_bin_colscan", "k_bin_emit<", "k_tile_sort",
             "k_tile_sort_big", "k_tile_sort_huge", "k_composite<", "k_composite_q<", "k_chunk1<",
             "k_c1_parts", "k_c1_records", "k_c1_tiles<", "k_part_list", "k_frame_end"]
    for k in frame:
        found = [n for n in res if n == k or (k.endswith("<") and n.startswith(k))]
        assert found, (k, sorted(res))
        for n in found:
            assert res[n]["scratch"] == 0, (n, res[n])
    assert res["k_composite<false,1,2>"]["vgpr"] <= 96, res["k_composite<false,1,2>"]
    # the still camera's fused sort + composite: one 8-B value of the sort held in scratch across
    # a barrier (present at any VGPR budget), nothing more
    for n in [n for n in res if n.startswith("k_composite_ts<")]:
        assert res[n]["scratch"] <= 16 and res[n]["vgpr"] <= 96, (n, res[n])


def test_chunk1_grid_residency_rule():
    """k_chunk1's grid barrier needs its whole grid resident: grid = min(64, CUs, occupancy x CUs),
    refused (GS_ERR_UNSUPPORTED) when no workgroup fits (gs_debug_chunk1_grid, host logic)."""
    assert gs.chunk1_grid(None, 1, 256) == (64, 1)
    assert gs.chunk1_grid(None, 4, 256) == (64, 4)
    assert gs.chunk1_grid(None, 1, 40) == (40, 1)   # fewer CUs than 64: one per CU
    assert gs.chunk1_grid(None, 2, 16) == (16, 2)
    for occ, cus in ((0, 256), (1, 0), (-1, 8)):
        with pytest.raises(gs.GsError) as e:
            gs.chunk1_grid(None, occ, cus)
        assert e.value.code == gs.GS_ERR_UNSUPPORTED


def test_balance_strips_equalises_cost():
    """gs_balance_strips (K-balanced row strips): the cost of each current strip is
    spread evenly over its rows and new boundaries equalise it."""
    # two strips of 10 rows, the first three times as costly: the model's cut is 400/2 / 30 per
    # row = 6.7, and the boundary moves half way there (damped)
    assert list(gs.balance_strips([0, 10, 20], [300.0, 100.0])) == [0, 8, 20]
    # uniform cost: even strips stay
    assert list(gs.balance_strips([0, 17, 34, 51, 68], [5.0, 5.0, 5.0, 5.0])) == [0, 17, 34, 51, 68]
    # zero cost, or more strips than rows: unchanged
    assert list(gs.balance_strips([0, 3, 6], [0.0, 0.0])) == [0, 3, 6]
    assert list(gs.balance_strips([0, 1, 1, 2], [1.0, 0.0, 5.0])) == [0, 1, 1, 2]
    # every strip keeps a row even when one strip holds all the cost
    b = gs.balance_strips([0, 2, 4, 6, 8], [0.0, 0.0, 0.0, 100.0])
    assert (np.diff(b) >= 1).all() and b[0] == 0 and b[-1] == 8
    for bad in (([0, 5, 4], [1.0, 1.0]), ([1, 5, 10], [1.0, 1.0]), ([0, 5, 10], [1.0, float("nan")])):
        with pytest.raises(gs.GsError):
            gs.balance_strips(*bad)


def test_balance_strips_converges():
    """Fed back the strips' true costs frame after frame (a dense band of rows, as a real scene's
    horizon), the boundaries converge to within 15 % of equal cost for G = 2, 4, 8."""
    TR = 68
    rows = np.ones(TR)
    rows[20:32] = 25.0  # a dense band
    for G in (2, 4, 8):
        b = np.array([g * TR // G for g in range(G + 1)], np.int32)
        for _ in range(12):
            cost = [rows[b[g]:b[g + 1]].sum() for g in range(G)]
            b = gs.balance_strips(b, cost)
        cost = np.array([rows[b[g]:b[g + 1]].sum() for g in range(G)])
        # a single row can exceed the ideal share: the bound is the row granularity
        assert cost.max() <= max(1.15 * cost.sum() / G, cost.sum() / G + rows.max()), (G, b, cost)
