"""The dragon_json-style flow on the GPU: a Serializer JSON (tests/golden/json, written by the
reference's own Serializer) read natively (include/jsrt_json.h) and rendered by the HIP kernels equals
the reference's golden renders of the scene it was serialized from -- RGBA8 bit-exact, |dRGB| <= 1e-5.
"""
import gzip
import os

import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JDIR = os.path.join(ROOT, "tests", "golden", "json")
SIDE = {"bunny": os.path.join(ROOT, "tests", "golden", "meshes", "bunny2.obj.gz"),
        "heart": os.path.join(JDIR, "heart.obj.gz"), "cat": os.path.join(JDIR, "cat.obj.gz")}
TOL = 1e-5


def _gz(p):
    with gzip.open(p, "rb") as f:
        return f.read()


@pytest.mark.parametrize("scene", ["cornell_box_path", "SDF_Menger", "SDF_RecursiveUnionTest", "bunny", "heart",
                                   "BoxBall_DOF", "refraction_path"])
def test_gpu_json_scene_matches_reference_goldens(scene):
    import jsraytracer_amd as jr
    side = [_gz(SIDE[scene])] if scene in SIDE else []
    blob, _ = jr.blob_from_json(_gz(os.path.join(JDIR, scene + ".json.gz")), side)
    sc = jr.Scene(blob, device=0)
    tags = [(t, r) for t, r in pyoracle.golden_index().items() if r["scene"] == scene and "_part" not in t]
    assert tags
    for tag, r in tags:
        rgba, colors, _ = sc.render(r["width"], r["height"], r["spp"], r["depth"], r["kind"], r["seed"])
        gcol, grgba = pyoracle.golden_image(tag, r["width"], r["height"])
        assert np.array_equal(rgba, grgba), tag
        fin = np.isfinite(gcol[..., :3])
        assert np.array_equal(np.isfinite(colors[..., :3]), fin), tag
        if fin.any():
            assert float(np.abs(colors[..., :3][fin] - gcol[..., :3][fin]).max()) <= TOL, tag
