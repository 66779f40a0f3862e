"""BASELINE.json's configurations on the GPU against the CPU oracle:

  configs[1]  public/pc_short.ply at 1280x720 (fp32 and the rgba16float target; the reference's
              init-sort truncation is tests/test_gpu_order.py::test_ref_quirks_pc_short_1280x720)
  configs[2]  synthetic 1 M at 1920x1080 (test_gpu_parity.py::test_synthetic_1m_1080p)
  configs[3]  the bench scene: synthetic 6.1 M (bicycle stand-in, seed 6) at 1920x1080, full frame
  configs[4]  synthetic 50 M (seed 50) at 3840x2160 on one GPU, and its 8 row strips
configs[0] (simple.ply at 256x256) is test_gpu_parity.py's small-scene suite.

Bars (stated in test_gpu_parity.py): fp32 oracle MSE < 1e-8, max-abs <= 1e-3 outside <= 0.01 %
of pixels; fp16-target oracle MSE < 1e-5 with >= 99.9 % of pixels within 2e-2; strips
bit-identical to the full frame.
"""
import numpy as np
import pytest

import oracle_py as orc
from conftest import camera, load_scene
from test_gpu_parity import image_close_fp16, image_close_fp32, webgpu_bar

pytestmark = pytest.mark.gpu

gs = pytest.importorskip("gsplat_amd")


@pytest.mark.parametrize("cam", ["app", "close", "behind"])
def test_config1_pc_short_1280x720(gpu_ctx, cam):
    aos, n, nsh = load_scene("pc_short")
    W, H = 1280, 720
    u, _ = camera("pc_short_" + cam, W, H)
    sc = gs.Scene(gpu_ctx, aos, n, nsh)
    img = sc.render(u, W, H, gs.make_opts(t_min=1e-4))
    ref, st = orc.render(aos, n, nsh, u, W, H, accum=0, t_min=1e-4)
    r = image_close_fp32(img, ref, name="pc_short_720_" + cam)
    assert r[2], r
    assert gpu_ctx.timings()["n_vis"] == st["n_vis"]
    img16 = sc.render(u, W, H, gs.make_opts(accum=gs.GS_ACCUM_FP16_TARGET, t_min=0.0,
                                             out_format=gs.GS_OUT_RGBA_F16))
    ref16, _ = orc.render(aos, n, nsh, u, W, H, accum=1, t_min=0.0)
    r = image_close_fp16(img16.astype(np.float32), ref16)
    assert r[2], r
    # the bench's timed mode (fp32 accumulation, t_min 1e-4, f16 out) against the WebGPU stand-in
    imgb = sc.render(u, W, H, gs.make_opts(t_min=1e-4, out_format=gs.GS_OUT_RGBA_F16))
    webgpu_bar(imgb, aos, n, nsh, u, W, H, name="pc_short_720_bench_" + cam)


@pytest.mark.timeout(300)
def test_config3_6m_1080p_full_frame(gpu_ctx):
    """The bench configuration itself, every pixel against the oracle: fp32, and the fp16-target
    mode with f16 output that bench.py times."""
    W, H, n = 1920, 1080, 6_100_000
    aos = gs.synth_aos(n, 6, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H)
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, timing=1))
    st_gpu = gpu_ctx.timings()
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    assert st_gpu["n_vis"] == st["n_vis"]
    r = image_close_fp32(img, ref, name="cfg3_6m")
    assert r[2], r
    o16 = gs.make_opts(accum=gs.GS_ACCUM_FP16_TARGET, out_format=gs.GS_OUT_RGBA_F16)
    img16 = sc.render(u, W, H, o16)
    ref16, _ = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=1, t_min=1e-4)
    r = image_close_fp16(img16.astype(np.float32), ref16)
    assert r[2], r
    # the mode bench.py times (fp32 accumulation, t_min 1e-4, f16 out) against the WebGPU
    # stand-in (fp16-target oracle, no cutoff)
    imgb = sc.render(u, W, H, gs.make_opts(out_format=gs.GS_OUT_RGBA_F16))
    webgpu_bar(imgb, aos, n, 16, u, W, H, name="cfg3_6m_bench")


@pytest.mark.timeout(600)
def test_config4_50m_4k(gpu_ctx):
    """configs[4] on one GPU: 50 M Gaussians at 3840x2160 against the fp32 oracle, and the 8 row
    strips of the multi-GPU partition bit-identical to the full frame."""
    W, H, n = 3840, 2160, 50_000_000
    aos = gs.synth_aos(n, 50, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H)
    parts = [sc.render(u, W, H, gs.make_opts(strip_index=g, strip_count=8)) for g in range(8)]
    assert np.array_equal(np.concatenate(parts, axis=0)[:H], img)
    del parts
    sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, timing=1))
    st_gpu = gpu_ctx.timings()
    sc.close()
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    del aos
    assert st_gpu["n_vis"] == st["n_vis"]
    r = image_close_fp32(img, ref, name=None)
    assert r[2], r


@pytest.mark.timeout(300)
def test_two_binning_bands_5120x2880(gpu_ctx):
    """A frame past one binning band (320 x 180 = 57 600 tiles > kBandTilesMax = 36 000: the
    launches split it into two equal bands, each walking every splat for its rows): every pixel
    against the oracle, a chunk split bit-identical to one chunk, and its 4 row strips
    bit-identical to the full frame."""
    W, H, n = 5120, 2880, 200_000
    aos = gs.synth_aos(n, 3, W, H)
    u = gs.bench_uniforms(W, H)
    sc = gs.Scene(gpu_ctx, aos, n, 16)
    img = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0))
    ref, st = orc.render(aos.view(np.uint8), n, 16, u, W, H, accum=0, t_min=1e-4)
    assert gpu_ctx.timings()["n_vis"] == st["n_vis"]
    r = image_close_fp32(img, ref, name="bands_5k")
    assert r[2], r
    split = sc.render(u, W, H, gs.make_opts(chunk_fraction=0.25))
    assert np.array_equal(split, img)
    G = 4
    rows = []
    for g in range(G):
        s = sc.render(u, W, H, gs.make_opts(chunk_fraction=1.0, strip_index=g, strip_count=G))
        rows.append(s)
    full = np.concatenate(rows, axis=0)[:H]
    assert np.array_equal(full, img)
