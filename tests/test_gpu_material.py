"""The HIP path's shading inputs against the reference's own known answers (tests/golden/material/,
oracle/refharness/make_material_kats.js), through the C ABI (jsrt_material_data, jsrt_sdf_distance):
  * for every hit of the cast KATs' primary and random rays of all 28 golden scenes, the material_data
    Primitive.color (world.js:125-137) hands to Material.color -- world normal, world position, UV,
    triangle barycentric coordinates, SDF basecolor -- bit for bit (the device computes UV's first two
    components, the ones the materials read; a reference UV's third component, from a 3-component OBJ
    texture coordinate, is not compared);
  * SDF.distance (sdf.js:53-477) of every SDFGeometry primitive at random points and hit points, bit for
    bit: the same program VM the render's sphere tracing runs.
A render that differs can then be narrowed to one hit's shading input."""
import numpy as np
import pytest

from oracle import pyoracle

SCENES = pyoracle.golden_material_scenes()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jr():
    import jsraytracer_amd as jr
    return jr


def _diff_rows(a, b):
    """rows where the f32 bit patterns differ (NaN == NaN: absent on both sides)."""
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return np.flatnonzero(~same.all(1))


@pytest.mark.parametrize("name", SCENES)
def test_gpu_material_data_matches_reference(jr, name):
    kat = pyoracle.golden_material(name)
    m = kat["material"]
    sc = jr.Scene(pyoracle.golden_scene(name), device=0)
    got = sc.material_data(m["rays"])
    assert np.array_equal(got["obj"], m["obj"])
    assert np.array_equal(got["t"].view(np.uint64), m["t"].view(np.uint64))
    hit = m["obj"] >= 0
    for f, cols in (("normal", 4), ("position", 4), ("uv", 2), ("bary", 3), ("basecolor", 3)):
        bad = _diff_rows(got[f][hit, :cols], m[f][hit, :cols])
        assert bad.size == 0, (f"{name}.{f}: {bad.size} of {int(hit.sum())} hits differ, first: "
                               f"{got[f][hit][bad[0]]} vs {m[f][hit][bad[0]]}")
    assert np.isnan(got["normal"][~hit]).all()


@pytest.mark.parametrize("name", [n for n in SCENES if pyoracle.golden_material(n)["sdf"]])
def test_gpu_sdf_distance_matches_reference(jr, name):
    kat = pyoracle.golden_material(name)
    sc = jr.Scene(pyoracle.golden_scene(name), device=0)
    for e in kat["sdf"]:
        d = sc.sdf_distance(e["obj"], e["points"])
        bad = np.flatnonzero(d.view(np.uint64) != e["distance"].view(np.uint64))
        assert bad.size == 0, f"{name} obj {e['obj']}: {bad.size} of {len(d)} differ, first {d[bad[0]]!r} vs {e['distance'][bad[0]]!r}"


def test_gpu_sdf_distance_rejects_non_sdf_object(jr):
    sc = jr.Scene(pyoracle.golden_scene("SDF_Menger"), device=0)
    with pytest.raises(jr.JsrtError, match="not an SDFGeometry"):
        sc.sdf_distance(0, np.zeros((1, 4), np.float32))  # object 0 is the floor plane


def test_gpu_menger_material_data_dense_against_oracle(jr):
    """SDF_Menger's materialData on 16,384 rays from inside and around the sponge (hits on the hole walls at every
    level), against the oracle: the four normal distances sharing each axis's transform/repetition chain and
    getMaterialData's choice from them (sdf_forms.h sdf_form_normal4) must give every f32 bit of the normal,
    position and basecolour.  The sponge: Mat4.translation([-3.5, 0.5, -3.5]) x rotationY(-0.15) of a unit box."""
    blob = pyoracle.golden_scene("SDF_Menger")
    rng = np.random.default_rng(29)
    c = np.array([-3.5, 0.5, -3.5])
    o = (c + rng.uniform(-1.4, 1.4, (16384, 3))).astype(np.float32)
    d = rng.normal(size=(16384, 3))
    d[:4096] = np.round(d[:4096] * 2) / 2 + 1e-3
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    rays = np.concatenate([o, d], 1)
    want = pyoracle.material_data(blob, rays)
    sc = jr.Scene(blob, device=0)
    try:
        got = sc.material_data(rays)
    finally:
        sc.close()
    assert np.array_equal(got["obj"], want["obj"])
    hit = want["obj"] == 1
    assert hit.sum() > 5000
    for f, cols in (("normal", 4), ("position", 4), ("basecolor", 3)):
        bad = _diff_rows(got[f][hit, :cols], want[f][hit, :cols])
        assert bad.size == 0, f"{f}: {bad.size} of {int(hit.sum())} differ, first {got[f][hit][bad[0]]} vs {want[f][hit][bad[0]]}"
