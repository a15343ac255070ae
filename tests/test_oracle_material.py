"""The oracle's shading inputs against known answers computed by the reference itself
(oracle/refharness/make_material_kats.js -> tests/golden/material/):
  * material_data -- for every hit of the cast KATs' primary and random rays, what Primitive.color
    (world.js:125-137) hands to Material.color: the world normal after inv_transform.transposed() and
    normalized() (geometry.js materialData per kind; sdf.js:41-47 forward differences), the world hit
    position, UV (planes, spheres, cylinders, triangles' psdata, SDF spheres), triangle barycentric
    coordinates (geometry.js:389-396) and SDF basecolors -- bit for bit, NaN patterns included;
  * SDF.distance -- the root distance of every SDFGeometry primitive (sdf.js:53-477) at random points of
    its bounding box and at the rays' hit points, bit for bit.
A render that differs can then be narrowed to one hit's shading input instead of bisecting images."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle

SCENES = pyoracle.golden_material_scenes()
FIELDS = ("normal", "position", "uv", "bary", "basecolor")


def bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def test_every_golden_scene_has_material_kats():
    assert len(SCENES) >= 28
    kinds = set()
    for name in SCENES:
        m = pyoracle.golden_material(name)["material"]
        hit = m["obj"] >= 0
        kinds |= {f for f in FIELDS if np.isfinite(m[f][hit]).any()}
    assert kinds == set(FIELDS)  # every field is exercised somewhere


def test_sdf_scenes_have_distance_kats():
    sdf = [n for n in SCENES if pyoracle.golden_material(n)["sdf"]]
    assert set(sdf) >= {"SDF_Menger", "SDF_Combinations", "SDF_Sierpinski", "SDF_Simple"}


@pytest.mark.parametrize("name", SCENES)
def test_oracle_material_data_matches_reference(name):
    kat = pyoracle.golden_material(name)
    blob = pyoracle.golden_scene(name)
    assert hashlib.sha256(blob).hexdigest() == kat["blob_sha256"]
    m = kat["material"]
    got = pyoracle.material_data(blob, m["rays"])
    assert np.array_equal(got["obj"], m["obj"]) and bits_equal(got["t"].view(np.uint64), m["t"].view(np.uint64))
    for f in FIELDS:
        bad = np.flatnonzero((got[f].view(np.uint32) != m[f].view(np.uint32)).any(1) &
                             ~(np.isnan(got[f]) & np.isnan(m[f])).all(1))
        assert bad.size == 0, f"{name}.{f}: {bad.size} rays differ, first {bad[0]}: {got[f][bad[0]]} vs {m[f][bad[0]]}"


@pytest.mark.parametrize("name", [n for n in SCENES if n.startswith("SDF")])
def test_oracle_sdf_distance_matches_reference(name):
    kat = pyoracle.golden_material(name)
    blob = pyoracle.golden_scene(name)
    for e in kat["sdf"]:
        d = pyoracle.sdf_distance(blob, e["obj"], e["points"])
        bad = np.flatnonzero(d.view(np.uint64) != e["distance"].view(np.uint64))
        assert bad.size == 0, f"{name} obj {e['obj']}: {bad.size} of {len(d)} distances differ, first {bad[0]}"
