"""World.cast on the GPU (jsrt_cast -> the same world_cast / bvh_cast / SDF march the render kernels
run) against known answers computed by the reference itself (oracle/refharness/make_cast_kats.js):
every golden scene, primary camera rays (per-pixel primary-hit index), random rays and shadow
segments.  Distance bit-exact, hit Primitive exact.  Reference: world.js:7-15, 28-30."""
import numpy as np
import pytest

from oracle import pyoracle

SCENES = pyoracle.golden_cast_scenes()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jr():
    import jsraytracer_amd as jr
    return jr


@pytest.mark.parametrize("name", SCENES)
def test_gpu_cast_matches_reference(jr, name):
    kat = pyoracle.golden_casts(name)
    scene = jr.Scene(pyoracle.golden_scene(name), device=0)
    try:
        for s in kat["sets"]:
            t, obj = scene.cast(s["rays"], s["minD"], s["maxD"], s["transp"])
            bad = np.flatnonzero((t.view(np.uint64) != s["t"].view(np.uint64)) | (obj != s["obj"]))
            assert bad.size == 0, (f"{name}/{s['name']}: {bad.size} of {len(t)} casts differ, first ray {bad[0]}: "
                                   f"t {t[bad[0]]!r} vs {s['t'][bad[0]]!r}, obj {obj[bad[0]]} vs {s['obj'][bad[0]]}")
    finally:
        scene.close()


def test_gpu_cast_dragon_against_oracle(jr):
    """The natively built dragon (199,935 BVH nodes) against the oracle
    on the same blob: 4096 random rays through its bounding box, closest hit and shadow segments."""
    blob, _ = pyoracle.mesh_scene("dragon", jr)
    rng = np.random.default_rng(7)
    c = np.array([0.0, 1.5, -4.0])  # the dragon (tests/dragon/test.mjs:28-30)
    o = (c + rng.uniform(-3, 3, (4096, 3))).astype(np.float32)
    d = c + rng.uniform(-1, 1, (4096, 3)) - o
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    rays = np.concatenate([o, d], 1)
    scene = jr.Scene(blob, device=0)
    try:
        for minD, maxD, tr, rr in ((0.0, float("inf"), True, rays),
                                   (0.0001, 1.0, False, np.concatenate([o, (np.roll(o, 1, 0) - o)], 1))):
            t, obj = scene.cast(rr, minD, maxD, tr)
            te, oe = pyoracle.cast(blob, rr, minD, maxD, tr)
            assert np.isfinite(te).sum() > 1000 and np.unique(oe).size > 100
            np.testing.assert_array_equal(t.view(np.uint64), te.view(np.uint64))
            np.testing.assert_array_equal(obj, oe)
    finally:
        scene.close()


def test_gpu_cast_menger_inside_against_oracle(jr):
    """SDF_Menger's march from points inside and around the sponge (its holes at every level), against the
    oracle: the sponge form's early exit (sdf_forms.h sdf_form_runion; JSRT_SDF_EXIT=0 turns it off) must give
    every distance bit for bit.  The sponge is Mat4.translation([-3.5, 0.5, -3.5]) x rotationY(-0.15) of a
    unit box (tests/SDF_Menger/test.mjs)."""
    blob = pyoracle.golden_scene("SDF_Menger")
    rng = np.random.default_rng(11)
    c = np.array([-3.5, 0.5, -3.5])
    o = (c + rng.uniform(-1.3, 1.3, (8192, 3))).astype(np.float32)
    d = rng.normal(size=(8192, 3))
    d[: 2048] = np.round(d[: 2048] * 2) / 2 + 1e-3  # near axis-aligned: long marches along the hole walls
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    rays = np.concatenate([o, d], 1)
    scene = jr.Scene(blob, device=0)
    try:
        for minD, maxD, tr, rr in ((0.0001, float("inf"), True, rays),
                                   (0.0001, 1.0, False, np.concatenate([o, (np.roll(o, 1, 0) - o)], 1))):
            t, obj = scene.cast(rr, minD, maxD, tr)
            te, oe = pyoracle.cast(blob, rr, minD, maxD, tr)
            assert np.isfinite(te).sum() > 1000
            np.testing.assert_array_equal(t.view(np.uint64), te.view(np.uint64))
            np.testing.assert_array_equal(obj, oe)
    finally:
        scene.close()
