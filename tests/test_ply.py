"""PLY ingest (gs_ply_parse) against PackedGaussians (src/ply.ts) run on the same files.

tests/golden/ply/*.ply are the reference's public/*.ply; tests/golden/ply_synth/*.ply are edge
cases written by gen_ref_fixtures.py.  Expected outputs (*.aos.bin, min/max pos, thrown errors)
come from running the reference's own ply.ts under node 12 (gen_ref_fixtures.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT  # noqa: F401

gs = pytest.importorskip("gsplat_amd")
SYNTH = os.path.join(GOLDEN, "ply_synth")


@pytest.mark.parametrize("name", ["simple", "pc_short", "m3splat"])
def test_reference_plys(name):
    meta = json.load(open(os.path.join(GOLDEN, "ply_meta.json")))[name]
    aos, info = gs.parse_ply(open(os.path.join(GOLDEN, "ply", name + ".ply"), "rb").read())
    assert hashlib.sha256(aos.tobytes()).hexdigest() == meta["sha256"]
    assert info["numGaussians"] == meta["numGaussians"] and info["nShCoeffs"] == meta["nShCoeffs"]
    assert info["min_pos"] == meta["min_pos"] and info["max_pos"] == meta["max_pos"]


SYNTH_META = json.load(open(os.path.join(SYNTH, "meta.json")))


@pytest.mark.parametrize("name", sorted(SYNTH_META))
def test_edge_case_plys(name):
    m = SYNTH_META[name]
    data = open(os.path.join(SYNTH, name + ".ply"), "rb").read()
    if "error" in m:  # the reference throws: we return an error status
        with pytest.raises(gs.GsError) as e:
            gs.parse_ply(data)
        want = gs.GS_ERR_UNSUPPORTED if "SH degree" in m["error"] else gs.GS_ERR_INVALID
        assert e.value.code == want, (e.value, m["error"])
        return
    aos, info = gs.parse_ply(data)
    ref = open(os.path.join(SYNTH, name + ".aos.bin"), "rb").read()
    assert aos.tobytes() == ref  # bit-exact, NaN payloads included
    assert info["numGaussians"] == m["numGaussians"] and info["shDegree"] == m["shDegree"]
    assert info["min_pos"] == m["min_pos"] or np.allclose(info["min_pos"], m["min_pos"], equal_nan=True)
    assert info["max_pos"] == m["max_pos"] or np.allclose(info["max_pos"], m["max_pos"], equal_nan=True)


def test_parsed_scene_matches_synth_layout():
    """A parsed scene is the same AoS record gs_scene_upload takes (64 + 16 n_sh bytes)."""
    layout = json.load(open(os.path.join(GOLDEN, "layout.json")))
    for name in ("deg0", "deg1", "deg2"):
        aos, info = gs.parse_ply(open(os.path.join(SYNTH, name + ".ply"), "rb").read())
        assert info["record_bytes"] == layout["record"][str(info["nShCoeffs"])]["size"]
        assert aos.size == info["numGaussians"] * info["record_bytes"]
