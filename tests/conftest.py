import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "gaussian-splatting-web_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def load_scene(name):
    """Reference-ingested AoS fixture (tests/golden/<name>.aos.bin, made by gen_ref_fixtures.py)."""
    meta = json.load(open(os.path.join(GOLDEN, "ply_meta.json")))[name]
    aos = np.fromfile(os.path.join(GOLDEN, name + ".aos.bin"), np.uint8)
    return aos, meta["numGaussians"], meta["nShCoeffs"]


def camera(name, W, H):
    """(160-B uniform block as 40 float32, entry) for a fixture camera from cameras.json."""
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    for c in cams:
        if c["name"] == name and c["W"] == W and c["H"] == H:
            u = np.zeros(40, np.float32)
            u[0:16] = np.array(c["view"], np.uint32).view(np.float32)
            u[16:32] = np.array(c["proj"], np.uint32).view(np.float32)
            u[32:35] = np.array(c["campos"], np.uint32).view(np.float32)
            u[37], u[38], u[39] = W, H, 1.0
            return u, c
    raise KeyError((name, W, H))


@pytest.fixture(scope="session")
def gpu_ctx():
    import gsplat_amd as gs
    return gs.Context(0)
