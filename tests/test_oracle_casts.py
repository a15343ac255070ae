"""The oracle's World.cast against known answers computed by the reference itself
(oracle/refharness/make_cast_kats.js -> tests/golden/casts/): per scene, primary camera rays (the
per-pixel primary-hit index), random rays and shadow segments; closest-hit distance bit-exact and
the hit Primitive (its OBJS index in the golden scene blob) exact.  Reference: world.js:7-15, 28-30."""
import hashlib

import numpy as np
import pytest

from oracle import pyoracle

SCENES = pyoracle.golden_cast_scenes()


def test_every_golden_scene_has_cast_kats():
    assert len(SCENES) >= 28


@pytest.mark.parametrize("name", SCENES)
def test_oracle_cast_matches_reference(name):
    kat = pyoracle.golden_casts(name)
    blob = pyoracle.golden_scene(name)
    assert hashlib.sha256(blob).hexdigest() == kat["blob_sha256"], "KATs were made from another export of the scene"
    for s in kat["sets"]:
        t, obj = pyoracle.cast(blob, s["rays"], s["minD"], s["maxD"], s["transp"])
        bad = np.flatnonzero((t.view(np.uint64) != s["t"].view(np.uint64)) | (obj != s["obj"]))
        assert bad.size == 0, (f"{name}/{s['name']}: {bad.size} of {len(t)} casts differ, first ray {bad[0]}: "
                               f"t {t[bad[0]]!r} vs {s['t'][bad[0]]!r}, obj {obj[bad[0]]} vs {s['obj'][bad[0]]}")
