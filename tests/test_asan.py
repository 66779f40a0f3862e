"""Sanitizer build: the host-side C ABI (PLY ingest with truncated and mutated
headers, camera / uniform producer, present, PNG, synthetic scenes) and the CPU oracle under
AddressSanitizer + UndefinedBehaviorSanitizer (tools/asan/host_asan.cpp), and the N-API addon
instrumented the same way under node's host checks.  CPU only: no GPU code is instrumented."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


def _have_asan():
    r = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True)
    return r.returncode == 0 and os.path.isabs(r.stdout.strip())


pytestmark = pytest.mark.skipif(not shutil.which("g++") or not _have_asan(), reason="no g++ sanitizer runtime")


def test_host_and_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", ASAN, "run"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "asan driver clean" in r.stdout


@pytest.mark.skipif(not shutil.which("node") or not os.path.exists("/usr/include/node/node_api.h") or
                    not os.path.exists(os.path.join(ROOT, "gaussian-splatting-web_amd", "lib", "libgsplat.so")),
                    reason="node, its headers or libgsplat.so absent")
def test_addon_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", ASAN, "run-addon"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    out = json.loads(open(os.path.join(ASAN, "addon_asan.json")).read().strip().splitlines()[-1])
    assert out["plyBad"] == -1 and len(out["cams"]) > 10
