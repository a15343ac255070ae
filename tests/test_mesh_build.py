"""Native OBJ ingest + BVH build (include/jsrt_mesh.h, jsraytracer_amd/csrc/mesh_build.cpp).

Pinned against the REFERENCE (fixtures from oracle/refharness/regen_mesh_fixtures.sh):
  * bunny: the natively built tree equals the one in the reference-exported golden scene
    (tests/golden/scenes/bunny.jsrt.gz) node for node, triangle for triangle (mesh_topology.digest);
  * dragon: equals the reference's tree digest (199,935 nodes, depth 24, 99,968 triangles after the
    minArea filter) in tests/golden/meshes/topology.json;
  * the oracle renders the natively built dragon bit-exactly like the reference's own renders.
Host-only: these run without a GPU.
"""
import gzip
import json
import os

import numpy as np
import pytest

import mesh_topology as mt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MESHES = os.path.join(ROOT, "tests", "golden", "meshes")
TOPO = json.load(open(os.path.join(MESHES, "topology.json")))


@pytest.fixture(scope="module")
def jr():
    from jsraytracer_amd import build as jb
    jb.build()
    import jsraytracer_amd
    return jsraytracer_amd


def skeleton(name):
    with gzip.open(os.path.join(MESHES, TOPO[name]["skeleton"]), "rb") as f:
        return f.read()


def native_scene(jr, name):
    return jr.load_obj_scene(skeleton(name), os.path.join(MESHES, TOPO[name]["obj_fixture"]))


def test_bunny_tree_equals_reference_export(jr, oracle):
    blob, info = native_scene(jr, "bunny")
    ref = mt.digest(oracle.golden_scene("bunny"))
    got = mt.digest(blob)
    assert got == ref
    assert got[0] == TOPO["bunny"]["sha256"]
    assert (info["triangles"], info["nodes"], info["max_depth"]) == (4968, 9935, 15)


def test_dragon_tree_equals_reference(jr):
    blob, info = native_scene(jr, "dragon")
    t = TOPO["dragon"]
    assert (info["triangles"], info["nodes"], info["max_depth"]) == (t["triangles"], t["nodes"], t["max_depth"])
    assert mt.digest(blob) == (t["sha256"], t["nodes"], t["max_depth"], t["triangles"])


def test_bunny_native_scene_renders_like_reference(jr, oracle):
    blob, _ = native_scene(jr, "bunny")
    for tag, r in oracle.golden_index().items():
        if r["scene"] != "bunny":
            continue
        _, rgba, _ = oracle.render(blob, r["width"], r["height"], r["spp"], r["depth"], r["kind"], r["seed"])
        _, grgba = oracle.golden_image(tag, r["width"], r["height"])
        assert np.array_equal(rgba, grgba), tag


MESH_RENDERS = json.load(open(os.path.join(MESHES, "index.json")))["renders"]


def mesh_golden(tag, r):
    rgba = np.fromfile(os.path.join(MESHES, "images", tag + ".rgba"), np.uint8).reshape(r["height"], r["width"], 4)
    col = np.fromfile(os.path.join(MESHES, "images", tag + ".f32"), np.float32).reshape(r["height"], r["width"], 4)
    return col, rgba


@pytest.mark.parametrize("tag", sorted(MESH_RENDERS))
def test_oracle_renders_native_dragon_like_reference(jr, oracle, tag):
    r = MESH_RENDERS[tag]
    blob, _ = native_scene(jr, r["scene"])
    col, rgba, st = oracle.render(blob, r["width"], r["height"], r["spp"], r["depth"], r["kind"], r["seed"])
    gcol, grgba = mesh_golden(tag, r)
    assert np.array_equal(rgba, grgba)
    same = (col.view(np.uint32) == gcol.view(np.uint32)) | (np.isnan(col) & np.isnan(gcol))
    assert same.all()
    assert st["draws"] == r["draws"] and st["color_calls"] == r["color_calls"]


def test_small_obj_forms_and_errors(jr):
    """objloader.js:144-221 forms: v with w, vt/vn, v/vt/vn, v//vn, polygon fans, comments, CRLF."""
    skel = skeleton("bunny")
    obj = ("# quad + triangle\r\nv 0 0 0\r\nv 1 0 0\nv 1 1 0 1\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 1 1\nvn 0 0 1\n"
           "o thing\ng grp\ns off\nf 1/1/1 2/2/1 3/3/1 4/1/1\nf 1//1 3//1 4//1\n")
    blob, info = jr.attach_obj(skel, obj)
    assert info["triangles"] == 3 and info["nodes"] == 5
    sec = mt.sections(blob)
    tris = np.frombuffer(sec["TRIS"][1], np.uint8).reshape(-1, 256)
    new = tris[-3:]
    flags = new[:, 144:156].view(np.uint32)  # has_normal, has_uv, uv_len
    assert flags.tolist() == [[1, 1, 3], [1, 1, 3], [1, 0, 0]]
    # area filter: a degenerate triangle is dropped (objloader.js:211, minArea 0.00001)
    _, info = jr.attach_obj(skel, "v 0 0 0\nv 1 0 0\nv 2 0 0\nv 0 1 0\nf 1 2 3\nf 1 2 4\n")
    assert info["triangles"] == 1 and info["nodes"] == 1
    with pytest.raises(jr.JsrtError, match="Error while attempting to parse obj file"):
        jr.attach_obj(skel, "v 0 0 0\nbogus 1\n")
    with pytest.raises(jr.JsrtError, match="usemtl"):
        jr.attach_obj(skel, "usemtl gold\n")
    with pytest.raises(jr.JsrtError, match="missing vertex"):
        jr.attach_obj(skel, "v 0 0 0\nf 1 2 3\n")
    with pytest.raises(jr.JsrtError, match="no triangle"):
        jr.attach_obj(skel, "v 0 0 0\n")
    from oracle import pyoracle
    with pytest.raises(jr.JsrtError, match="BVHAggregate"):
        jr.attach_obj(pyoracle.golden_scene("cornell_box_path"), obj)
    with pytest.raises(jr.JsrtError, match="template"):  # the full bunny tree is not a one-leaf template
        jr.attach_obj(pyoracle.golden_scene("bunny"), obj)
