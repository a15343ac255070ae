"""Native Serializer-JSON reader (include/jsrt_json.h, jsraytracer_amd/csrc/json_scene.cpp).

Pinned against the REFERENCE: tests/golden/json/ holds `JSON.stringify(new Serializer(test).plain())`
of every golden scene, written by the reference's own Serializer (oracle/refharness/
regen_json_fixtures.sh, as tests/test_to_json.js:32-35 writes tests/<scene>/test.json).  Reading it
must give the very blob the live-scene exporter wrote (tests/golden/scenes/), byte for byte -- with
the non-finite values JSON writes as null (PhongPathTracingMaterial ratio, infinite BoxSDF sizes and
SDF bounds, a NaN matrix) and the Triangle normals / UVs / signed zeros Triangle.serialize and
JSON.stringify drop (geometry.js:355-357) restored from the OBJ side-channel.  The dragon_json flow
(tests/dragon_json/test.mjs) runs end to end where the reference is present.  Host-only.
"""
import gzip
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import mesh_topology as mt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JDIR = os.path.join(ROOT, "tests", "golden", "json")
MESHES = os.path.join(ROOT, "tests", "golden", "meshes")
SCENES = sorted(f[:-8] for f in os.listdir(JDIR) if f.endswith(".json.gz"))
# the OBJ files each mesh scene loads (tests/<scene>/test.mjs)
SIDE = {"bunny": [os.path.join(MESHES, "bunny2.obj.gz")], "cat": ["cat.obj.gz"], "heart": ["heart.obj.gz"],
        "diamond": ["diamond.obj.gz"], "AHollowTetrahedron": ["hollow_tetrahedron.obj.gz"],
        "AMultipleBVH": ["hollow_tetrahedron.obj.gz", "star.obj.gz"]}


def _gz(p):
    with gzip.open(p if os.path.isabs(p) else os.path.join(JDIR, p), "rb") as f:
        return f.read()


@pytest.fixture(scope="module")
def jr():
    from jsraytracer_amd import build as jb
    jb.build()
    import jsraytracer_amd
    return jsraytracer_amd


@pytest.mark.parametrize("scene", SCENES)
def test_json_reads_to_the_live_export(jr, oracle, scene):
    text = _gz(scene + ".json.gz")
    blob, info = jr.blob_from_json(text, [_gz(p) for p in SIDE.get(scene, [])])
    assert blob == oracle.golden_scene(scene)
    if scene in SIDE:
        assert info["psdata_matched"] == info["triangles"] > 0


@pytest.mark.parametrize("scene,null_fields", [("cornell_box_path", 7), ("SDF_Menger", 3), ("SDF_RecursiveUnionTest", 37),
                                               ("SDF_SphereRepetition", 3)])
def test_json_nulls_are_the_non_finite_values(jr, oracle, scene, null_fields):
    """These scenes' JSON holds nulls where the live scene held Infinity / NaN; the blob equality
    above shows they are read back as +Infinity (ratios, box sizes, half sizes) and NaN (matrices)."""
    text = _gz(scene + ".json.gz").decode()
    assert text.count("null") == null_fields
    blob, _ = jr.blob_from_json(text)
    assert blob == oracle.golden_scene(scene)


def test_json_without_side_channel_has_face_normals(jr, oracle):
    """No OBJ side-channel: the triangles carry no vertex data -- what the reference renders after its
    own deserializeJSON (psdata = ps), and the same tree and everything else."""
    blob, info = jr.blob_from_json(_gz("bunny.json.gz"))
    assert info["psdata_matched"] == 0 and info["triangles"] == 4968
    c, raw = mt.sections(blob)["TRIS"]
    assert not np.frombuffer(raw, np.uint32).reshape(c, 64)[:, 36:38].any()  # has_normal, has_uv
    g = mt.sections(oracle.golden_scene("bunny"))
    s = mt.sections(blob)
    assert all(s[k] == g[k] for k in g if k != "TRIS")


def test_json_errors(jr):
    ok = _gz("ASimpleScene.json.gz").decode()
    cases = [(ok[:-5], "JSON parse error"), (ok + "x", "trailing characters"),
             ('{"_t":["Object",0],"_v":{"renderer":{"_r":7}}}', "references out of order"),
             ('{"_t":["Object",0],"_v":{"width":1}}', "renderer is missing"),
             (ok.replace('"smoothness":100', '"smoothness":null', 1), "smoothness is null"),
             (ok.replace('"Sphere"', '"Torus"', 1), "unsupported Geometry Torus")]
    for text, msg in cases:
        assert text != ok, msg
        with pytest.raises(jr.JsrtError, match=msg):
            jr.blob_from_json(text)


def test_json_side_channel_conflict(jr):
    """Two faces with the same vertex positions but different normals cannot be told apart."""
    obj = _gz("heart.obj.gz").decode()
    f0 = next(ln for ln in obj.split("\n") if ln.startswith("f ")).split()
    vn_new = sum(ln.startswith("vn ") for ln in obj.split("\n")) + 1
    dup = "f " + " ".join(t.split("/")[0] + "//" + str(vn_new) for t in f0[1:])
    with pytest.raises(jr.JsrtError, match="side-channel"):
        jr.blob_from_json(_gz("heart.json.gz"), [obj + "\nvn 0 0 1\n" + dup + "\n"])


NODE = shutil.which("node")


@pytest.mark.skipif(NODE is None or not os.path.exists("/root/reference/src/serializer.js"),
                    reason="needs node and the reference sources (dev container only)")
def test_dragon_json_flow_matches_the_blob_path(jr, oracle, tmp_path):
    """tests/dragon_json: the dragon's Serializer JSON (100k triangles, 200k BVH nodes, made by the
    reference here) read natively gives the reference's tree (topology digest) and renders like the
    reference's own dragon renders (oracle, tests/golden/meshes goldens)."""
    subprocess.run([NODE, "--max-old-space-size=16000", os.path.join(ROOT, "oracle", "refharness", "make_json_fixtures.js"),
                    str(tmp_path), "dragon"], check=True, capture_output=True, timeout=600)
    text = (tmp_path / "dragon.json").read_bytes()
    blob, info = jr.blob_from_json(text, [_gz(os.path.join(MESHES, "dragon.obj.gz"))])
    topo = json.load(open(os.path.join(MESHES, "topology.json")))["dragon"]
    assert mt.digest(blob) == (topo["sha256"], topo["nodes"], topo["max_depth"], topo["triangles"])
    assert info["psdata_matched"] == topo["triangles"]
    renders = json.load(open(os.path.join(MESHES, "index.json")))["renders"]
    for tag, r in renders.items():
        if r["scene"] != "dragon":
            continue
        _, rgba, _ = oracle.render(blob, r["width"], r["height"], r["spp"], r["depth"], r["kind"], r["seed"])
        g = np.fromfile(os.path.join(MESHES, "images", tag + ".rgba"), np.uint8).reshape(r["height"], r["width"], 4)
        assert np.array_equal(rgba, g), tag
