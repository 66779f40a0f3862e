"""The Node host (N-API addon + JS mirror of the reference's GpuContext/Renderer surface).

CPU: addon exports, string rejection without a device, camera/uniform producer bit-exact against
the wgpu-matrix fixtures.  GPU: the reference's frame loop (create -> Renderer -> animate/draw ->
destroy) driven from node renders the same image as the C ABI and matches the oracle."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, camera, load_scene

NODE = shutil.which("node")
ADDON = os.path.join(ROOT, "gaussian-splatting-web_amd", "lib", "gsplat_napi.node")
pytestmark = pytest.mark.skipif(not NODE or not os.path.exists(ADDON), reason="node or the addon is absent")

EXPORTS = sorted(["abiVersion", "lastError", "deviceCount", "ctxCreate", "ctxDestroy", "sceneUpload", "sceneFree",
                  "render", "renderAsync", "timings", "timingsReset", "sync", "present", "lookAt", "perspective",
                  "cameraPosition", "cameraFromJSON", "fbAlloc", "fbFree", "fbRead", "renderDevice", "presentDevice",
                  "synthAos", "packUniforms", "stripRows", "plyParse", "encodePng", "hostRegister",
                  "hostUnregister", "readbackAsync"])


def run_node(*args, timeout=120):
    r = subprocess.run([NODE] + list(args), capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_node_host_cpu():
    out = run_node(os.path.join(ROOT, "tests", "node", "host_checks.js"), os.path.join(GOLDEN, "cameras.json"))
    assert out["exports"] == EXPORTS
    assert out["abi"] == 5
    if out["deviceCount"] == 0:
        assert out["createRejected"] == "string" and out["requestRejected"] == "string"
    assert out["ctorThrows"] is True
    assert out["badHandle"] == -1
    cams = {(c["name"], c["W"], c["H"]): c for c in json.load(open(os.path.join(GOLDEN, "cameras.json")))}
    assert len(out["cams"]) > 10
    for c in out["cams"]:
        ref = cams[(c["name"], c["W"], c["H"])]
        assert c["view"] == ref["view"] and c["proj"] == ref["proj"] and c["campos"] == ref["campos"], c["name"]
    assert len(out["jsonCams"]) >= 8
    for c in out["jsonCams"]:
        ref = cams[(c["name"], c["W"], c["H"])]
        assert c["view"] == ref["view"] and c["proj"] == ref["proj"] and c["campos"] == ref["campos"], c["name"]
        assert c["focal"] == [c["H"], c["W"]] and c["size"] == [c["W"], c["H"]]
    u = np.array(out["uniforms"], np.uint32).view(np.float32)
    ref = cams[(out["cams"][0]["name"], out["cams"][0]["W"], out["cams"][0]["H"])]
    assert np.array_equal(u[0:16].view(np.uint32), np.array(ref["view"], np.uint32))
    assert np.array_equal(u[35:40], np.array([0.5, 0.25, 100, 200, 1], np.float32))
    assert out["strip"] == {"row0": 3 * 9 * 16, "rowsPadded": 9 * 16}
    meta = json.load(open(os.path.join(GOLDEN, "ply_meta.json")))["simple"]
    assert bytes.fromhex(out["ply"]["hex"]) == open(os.path.join(GOLDEN, "simple.aos.bin"), "rb").read()
    assert out["ply"]["n"] == meta["numGaussians"] and out["ply"]["nsh"] == meta["nShCoeffs"]
    assert out["ply"]["deg"] == meta["shDegree"]
    assert out["ply"]["min"] == meta["min_pos"] and out["ply"]["max"] == meta["max_pos"]
    assert out["plyBad"] == -1
    import gsplat_amd as gs
    png = bytes.fromhex(out["png"])
    assert png == gs.encode_png(np.arange(3 * 2 * 4, dtype=np.uint8).reshape(2, 3, 4))


@pytest.mark.gpu
def test_node_device_group_gpu(tmp_path):
    """GpuContext.create([0, 0, 0]): the Node drop-in driving a device group (three row strips, peer-
    copy gather on one GPU) renders the single-device image bit for bit."""
    import gsplat_amd as gs
    W, H = 320, 200
    n = 30_000
    aos = gs.synth_aos(n, 81, W, H)
    u = gs.bench_uniforms(W, H)
    (tmp_path / "scene.bin").write_bytes(aos.tobytes())
    (tmp_path / "uni.bin").write_bytes(u.tobytes())
    out = run_node(os.path.join(ROOT, "tests", "node", "render_frames.js"), str(tmp_path / "scene.bin"), str(n),
                   "16", str(tmp_path / "uni.bin"), str(W), str(H), str(tmp_path / "img.f32"), "2", "0,0,0")
    assert out["frames"] == 2 and out["destroyed"] is True
    img = np.fromfile(tmp_path / "img.f32", np.float32).reshape(H, W, 4)
    with gs.Context(0) as ctx:
        direct = gs.Scene(ctx, aos, n, 16).render(u, W, H)
    assert np.array_equal(img, direct)


@pytest.mark.gpu
def test_node_frame_loop_gpu(tmp_path):
    import gsplat_amd as gs
    import oracle_py as orc
    W, H = 256, 256
    aos, n, nsh = load_scene("pc_short")
    u, _ = camera("pc_short_app", W, H)
    (tmp_path / "scene.bin").write_bytes(aos.tobytes())
    (tmp_path / "uni.bin").write_bytes(u.tobytes())
    out = run_node(os.path.join(ROOT, "tests", "node", "render_frames.js"), str(tmp_path / "scene.bin"), str(n),
                   str(nsh), str(tmp_path / "uni.bin"), str(W), str(H), str(tmp_path / "img.f32"), "3")
    assert out["frames"] == 3 and out["destroyed"] is True
    img = np.fromfile(tmp_path / "img.f32", np.float32).reshape(H, W, 4)
    # same image as the C ABI path, close to the oracle
    ctx = gs.Context(0)
    sc = gs.Scene(ctx, aos, n, nsh)
    direct = sc.render(u, W, H)
    dd = np.abs(img - direct)
    assert np.array_equal(img, direct), (float(dd.max()), int((dd > 0).sum()), float(np.abs(img).sum()),
                                         float(np.abs(direct).sum()), np.argwhere(dd > 0)[:5].tolist())
    ref, _ = orc.render(aos, n, nsh, u, W, H, accum=0, t_min=1e-4)
    d = np.abs(img.astype(np.float64) - ref)
    assert float((d ** 2).mean()) < 1e-8
    pres = np.fromfile(str(tmp_path / "img.f32") + ".present", np.float32).reshape(H, W, 4)
    assert np.array_equal(pres, gs.present(direct, W, H))
    sc.close()
    ctx.close()


@pytest.mark.gpu
def test_node_device_resident_frame_loop():
    """Renderer({deviceResident: true}): frames stay in HBM (renderDevice, frames in flight) and
    readback() returns the same image as the host-readback loop; both frame rates are measured in JS
    (tools/node_fps.js, also reported by bench.py as node_fps)."""
    out = run_node(os.path.join(ROOT, "tools", "node_fps.js"), "40000", "3", "320", "200", "20", timeout=300)
    assert out["same_image"] is True
    assert out["device_resident_fps"] > 0 and out["host_readback_fps"] > 0
