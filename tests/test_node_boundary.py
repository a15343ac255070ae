"""The Node side of the drop-in boundary: the N-API addon over libjsrt
(jsraytracer_amd/js/jsrt_node.cpp) and the HipRenderer class keeping the reference's
render(img, timelimit, callback, x_offset, x_delt) contract (src/renderers.js:10,70).

CPU: the addon builds, loads in node, exports its functions, and fails loudly (a thrown Error with
jsrt_last_error's message) without a device or with a bad blob.  GPU: node renders reference scenes
through HipRenderer (sync, async, and the worker-protocol harness of src/worker.js) and the RGBA8
bytes equal the reference-generated goldens."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import pyoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "jsraytracer_amd", "js")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


@pytest.fixture(scope="module")
def addon():
    from jsraytracer_amd import build as jb
    jb.build()
    subprocess.run(["sh", os.path.join(JS, "build_addon.sh")], check=True)
    p = os.path.join(ROOT, "jsraytracer_amd", "_build", "jsrt_node.node")
    assert os.path.exists(p)
    return p


def _node(code, timeout=120):
    return subprocess.run([NODE, "-e", code], capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def test_addon_exports(addon):
    r = _node(f"const a=require({json.dumps(addon)}); console.log(JSON.stringify(Object.keys(a).sort()));"
              "console.log(a.abiVersion(), a.ownedColumns(40,1,2,8), a.ownedColumns(10,1,3,1));")
    assert r.returncode == 0, r.stderr
    keys, nums = r.stdout.strip().split("\n")
    assert json.loads(keys) == sorted(["sceneCreate", "sceneDestroy", "renderSync", "render", "deviceCount",
                                       "abiVersion", "ownedColumns", "attachObj", "blobFromJson"])
    assert nums.split() == ["4", "16", "3"]


def test_addon_attach_obj_matches_python_and_reference(addon, tmp_path):
    """attachObj (loadObjFile + BVHAggregate.build, natively) from node: the same blob bytes as the
    Python binding, and the bunny tree equals the reference's (tests/test_mesh_build.py digest)."""
    import gzip

    import jsraytracer_amd as jr
    import mesh_topology as mt
    meshes = os.path.join(ROOT, "tests", "golden", "meshes")
    out = tmp_path / "bunny.jsrt"
    code = (f"const a=require({json.dumps(addon)}); const z=require('zlib'), fs=require('fs');"
            f"const skel=z.gunzipSync(fs.readFileSync({json.dumps(os.path.join(meshes, 'bunny.skel.jsrt.gz'))}));"
            f"const obj=z.gunzipSync(fs.readFileSync({json.dumps(os.path.join(meshes, 'bunny2.obj.gz'))})).toString();"
            "const r=a.attachObj(skel, obj, {minArea: 0.00001});"
            f"fs.writeFileSync({json.dumps(str(out))}, r.blob); console.log(r.triangles, r.nodes, r.maxDepth);"
            "try { a.attachObj(skel, 'v 0 0 0\\nbogus\\n'); console.log('no throw'); } catch (e) { console.log(e.message); }")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert lines[0].split() == ["4968", "9935", "15"]
    assert lines[1].startswith("jsrt_blob_attach_obj: Error while attempting to parse obj file")
    with gzip.open(os.path.join(meshes, "bunny.skel.jsrt.gz"), "rb") as f:
        py, _ = jr.attach_obj(f.read(), jr.mesh.read_obj(os.path.join(meshes, "bunny2.obj.gz")))
    assert out.read_bytes() == py
    assert mt.digest(py) == mt.digest(pyoracle.golden_scene("bunny"))


def test_addon_attach_obj_with_mtl_matches_python(addon, tmp_path):
    """attachObj(skel, obj, {mtl: [text...], bvhObject}) -- the x-wing with its mtllib (usemtl on every
    face) -- gives the Python binding's bytes."""
    from oracle import pyoracle
    meshes = os.path.join(ROOT, "tests", "golden", "meshes")
    t = pyoracle.mesh_topology()["x-wing"]
    out = tmp_path / "xwing.jsrt"
    rd = "(f)=>z.gunzipSync(fs.readFileSync(" + json.dumps(meshes) + "+'/'+f))"
    code = (f"const a=require({json.dumps(addon)}); const z=require('zlib'), fs=require('fs'); const rd={rd};"
            f"const r=a.attachObj(rd({json.dumps(t['skeleton'])}), rd({json.dumps(t['obj_fixture'])}),"
            f"{{bvhObject:{t['bvh_object']}, mtl:[rd({json.dumps(t['mtl_fixtures'][0])}).toString()]}});"
            f"fs.writeFileSync({json.dumps(str(out))}, r.blob); console.log(r.triangles, r.nodes);")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == [str(t["triangles"]), str(t["nodes"])]
    assert out.read_bytes() == pyoracle.mesh_scene("x-wing")[0]


def test_addon_blob_from_json_matches_reference_export(addon, tmp_path):
    """blobFromJson (a dragon_json-style test.json, natively) from node: the bunny's Serializer JSON with
    its OBJ as psdata side-channel gives the golden blob the live exporter wrote."""
    jdir = os.path.join(ROOT, "tests", "golden", "json")
    obj = os.path.join(ROOT, "tests", "golden", "meshes", "bunny2.obj.gz")
    out = tmp_path / "bunny.jsrt"
    code = (f"const a=require({json.dumps(addon)}); const z=require('zlib'), fs=require('fs');"
            f"const j=z.gunzipSync(fs.readFileSync({json.dumps(os.path.join(jdir, 'bunny.json.gz'))})).toString();"
            f"const r=a.blobFromJson(j, {{psdataObj: [z.gunzipSync(fs.readFileSync({json.dumps(obj)}))]}});"
            f"fs.writeFileSync({json.dumps(str(out))}, r.blob); console.log(r.triangles, r.psdataMatched);"
            "try { a.blobFromJson('{\"_r\":3}'); console.log('no throw'); } catch (e) { console.log(e.message); }")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert lines[0].split() == ["4968", "4968"]
    assert lines[1].startswith("jsrt_blob_from_json: ")
    assert out.read_bytes() == pyoracle.golden_scene("bunny")


def test_addon_errors_are_thrown(addon):
    r = _node(f"const a=require({json.dumps(addon)});"
              "try {{ a.sceneCreate(new Uint8Array(10)); console.log('no throw'); }} catch (e) {{ console.log(e.message); }}"
              .replace("{{", "{").replace("}}", "}"))
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("jsrt_scene_create: ") and "no throw" not in r.stdout


def test_hiprenderer_without_device_throws(addon):
    from jsraytracer_amd import _native
    if _native.lib().jsrt_device_count() > 0:
        pytest.skip("a GPU is visible")
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "ASimpleScene.jsrt.gz")
    r = _node("const fs=require('fs'),z=require('zlib');const {HipRenderer}=require('./jsraytracer_amd/js/hip_renderer');"
              f"const b=z.gunzipSync(fs.readFileSync({json.dumps(scene)}));"
              "try { new HipRenderer(new Uint8Array(b)); console.log('no throw'); } catch (e) { console.log(e.message); }")
    assert r.returncode == 0, r.stderr
    assert "no throw" not in r.stdout and "jsrt_scene_create" in r.stdout


def _render_cli(tmp_path, tag, mode="sync", xo=0, xd=1):
    r = pyoracle.golden_index()[tag]
    scene = os.path.join(ROOT, "tests", "golden", "scenes", r["scene"] + ".jsrt.gz")
    out = tmp_path / f"{tag}_{mode}_{xo}.rgba"
    cmd = [NODE, os.path.join(JS, "render_cli.js"), scene, str(out)] + [
        str(r[k]) for k in ("width", "height", "spp", "depth", "kind", "seed")] + [str(xo), str(xd), mode]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    return np.fromfile(out, np.uint8).reshape(r["height"], r["width"], 4), json.loads(p.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_node_hiprenderer_matches_reference(addon, tmp_path, mode):
    tag = "ASimpleScene_incremental_64x64_s1_d4_seed1"
    rgba, info = _render_cli(tmp_path, tag, mode)
    r = pyoracle.golden_index()[tag]
    _, grgba = pyoracle.golden_image(tag, r["width"], r["height"])
    assert np.array_equal(rgba, grgba)
    assert info["stats"]["samples"] == r["width"] * r["height"] * r["spp"]


@pytest.mark.gpu
def test_node_partition_matches_reference_workers(addon, tmp_path):
    """x_offset/x_delt through the Node boundary equals the reference's own x_delt=3 worker images."""
    full = "cornell_box_path_incremental_32x32_s2_d8_seed5"
    for k in range(3):
        rgba, _ = _render_cli(tmp_path, full, "sync", k, 3)
        _, grgba = pyoracle.golden_image(full + f"_part{k}of3", 32, 32)
        assert np.array_equal(rgba, grgba)


def test_device_for_worker_round_robin():
    """Worker i of N (src/raytrace_launcher.js:65-101) renders on GPU i % deviceCount: 16 workers over an
    8-GPU node take devices 0..7 twice; without a device (count 0) every worker names device 0."""
    code = ("const {deviceForWorker}=require('./jsraytracer_amd/js/hip_renderer');"
            "const m=(n,c)=>Array.from({length:n},(_,i)=>deviceForWorker(i,c));"
            "console.log(JSON.stringify([m(16,8),m(3,1),m(4,0),m(5,2)]));")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    a, b, c, d = json.loads(r.stdout)
    assert a == [i % 8 for i in range(16)]
    assert b == [0, 0, 0] and c == [0, 0, 0, 0] and d == [0, 1, 0, 1, 0]


def test_node_wrapper_checks_abi_version(addon, tmp_path):
    """hip_renderer.js refuses an addon whose libjsrt reports another ABI (a stale .so would misread the
    stats struct): a stub addon reporting ABI 1 makes the wrapper throw before any scene is created."""
    stub = tmp_path / "stub_addon.js"
    stub.write_text("module.exports={abiVersion:()=>1, deviceCount:()=>0};")
    code = ("const {addon}=require('./jsraytracer_amd/js/hip_renderer');"
            "try { addon(); console.log('no throw'); } catch (e) { console.log(String(e)); }")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, timeout=60, cwd=ROOT,
                       env=dict(os.environ, JSRT_NODE_ADDON=str(stub)))
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("HipRenderer: libjsrt ABI 1, expected 4")


@pytest.mark.gpu
def test_node_worker_protocol_composite(addon, tmp_path):
    """worker_harness.js: N worker_threads speaking src/worker.js's protocol, composited like
    raytrace_launcher.js:92-97, equal the single-renderer image (partition invariance).  Each worker
    reports the device it took: worker i on GPU i % deviceCount (all on 0 on a one-GPU box)."""
    tag = "cornell_box_path_incremental_32x32_s2_d8_seed5"
    r = pyoracle.golden_index()[tag]
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "cornell_box_path.jsrt.gz")
    out = tmp_path / "composite.rgba"
    p = subprocess.run([NODE, os.path.join(JS, "worker_harness.js"), scene, "3", str(out), "32", "32", "2", "5"],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert p.returncode == 0, p.stderr
    got = np.fromfile(out, np.uint8).reshape(32, 32, 4)
    _, grgba = pyoracle.golden_image(tag, 32, 32)
    assert r["depth"] == 8
    assert np.array_equal(got, grgba)
    from jsraytracer_amd import _native
    ndev = _native.lib().jsrt_device_count()
    import re
    devs = {int(w): int(d) for w, d in re.findall(r"worker (\d+) on device (\d+) finished", p.stderr)}
    assert devs == {i: i % ndev for i in range(3)}, p.stderr


@pytest.mark.skipif(not os.path.exists("/root/reference/src/math.js"), reason="reference sources absent (GPU box)")
def test_live_scene_graph_export_matches_committed_blob(addon):
    """HipRenderer(test.renderer) exports the LIVE reference scene graph (configureTest of
    tests/cornell_box_path/test.mjs) to the same blob the GPU tests render; it then fails only for
    want of a device here."""
    code = ("const {loadScene}=require('./oracle/refharness/load_reference.js');"
            "const {HipRenderer}=require('./jsraytracer_amd/js/hip_renderer.js');"
            "const {exportScene}=require('./jsraytracer_amd/js/scene_blob.js');"
            "const z=require('zlib'),fs=require('fs');"
            "loadScene('cornell_box_path').then(t=>{const b=exportScene(t);"
            f"const g=z.gunzipSync(fs.readFileSync({json.dumps(os.path.join(ROOT, 'tests/golden/scenes/cornell_box_path.jsrt.gz'))}));"
            "console.log(Buffer.compare(Buffer.from(b),g)===0?'same':'differs');"
            "try{new HipRenderer(t.renderer,{width:t.width,height:t.height});console.log('created')}"
            "catch(e){console.log(e.message.split(':')[0])}}).catch(e=>{console.error(e);process.exit(1)});")
    r = subprocess.run([NODE, "--experimental-modules", "-e", code], capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split()
    assert lines[0] == "same"
    from jsraytracer_amd import _native
    assert lines[1] == ("created" if _native.lib().jsrt_device_count() > 0 else "jsrt_scene_create")


@pytest.mark.gpu
def test_node_progress_per_pass_running_mean(addon, tmp_path):
    """renderers.js:103-112 on the reference's own runtime: HipRenderer.render(img, timelimit, cb) on the
    Incremental renderer fires callback({pass, completion}) per pass with completion increasing, and the
    img the callback sees holds the running mean of passes 0..pass -- the spp = pass+1 frame."""
    import jsraytracer_amd as jr
    W, H, spp = 40, 32, 5
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "cornell_box_path.jsrt.gz")
    code = ("const fs=require('fs'),z=require('zlib');"
            "const {HipRenderer,NodePixelBuffer}=require('./jsraytracer_amd/js/hip_renderer');"
            f"const b=new Uint8Array(z.gunzipSync(fs.readFileSync({json.dumps(scene)})));"
            f"const r=new HipRenderer(b,{{samplesPerPixel:{spp},maxRecursionDepth:8,seed:5}});"
            f"const img=new NodePixelBuffer({W},{H}); const seen=[];"
            "r.render(img, 1e-9, (p)=>{seen.push(p); fs.writeFileSync("
            f"{json.dumps(str(tmp_path))}+'/pass'+p.pass+'.rgba', Buffer.from(img.imgdata.data));}});"
            f"fs.writeFileSync({json.dumps(str(tmp_path))}+'/final.rgba', Buffer.from(img.imgdata.data));"
            "console.log(JSON.stringify(seen)); r.destroy();")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    seen = json.loads(r.stdout.strip().split("\n")[-1])
    assert [s["pass"] for s in seen] == list(range(spp - 1))  # the last pass is the final image
    comp = [s["completion"] for s in seen]
    assert comp == sorted(comp) and all(0 < c < 1 for c in comp)
    sc = jr.Scene(pyoracle.golden_scene("cornell_box_path"), device=0)
    for s in seen:
        got = np.fromfile(tmp_path / f"pass{s['pass']}.rgba", np.uint8).reshape(H, W, 4)
        ref, _, _ = sc.render(W, H, s["pass"] + 1, 8, 1, 5, want_colors=False)
        assert np.array_equal(got, ref), f"pass {s['pass']}"
    final = np.fromfile(tmp_path / "final.rgba", np.uint8).reshape(H, W, 4)
    assert np.array_equal(final, sc.render(W, H, spp, 8, 1, 5, want_colors=False)[0])


@pytest.mark.gpu
def test_node_destroy_while_async_render_in_flight(addon):
    """sceneDestroy (HipRenderer.destroy) right after an un-awaited renderAsync: the render keeps its
    scene alive and completes correctly; the scene is destroyed after it, and a new render throws."""
    scene = os.path.join(ROOT, "tests", "golden", "scenes", "ASimpleScene.jsrt.gz")
    tag = "ASimpleScene_incremental_64x64_s1_d4_seed1"
    code = ("const fs=require('fs'),z=require('zlib');"
            "const {HipRenderer,NodePixelBuffer}=require('./jsraytracer_amd/js/hip_renderer');"
            f"const b=new Uint8Array(z.gunzipSync(fs.readFileSync({json.dumps(scene)})));"
            "const r=new HipRenderer(b,{samplesPerPixel:1,maxRecursionDepth:4,seed:1});"
            "const img=new NodePixelBuffer(64,64); const p=r.renderAsync(img); r.destroy();"
            "p.then(()=>{ let t='no throw'; try { r.render(img); } catch(e) { t='throws'; }"
            "process.stdout.write(Buffer.from(img.imgdata.data).toString('base64')+'\\n'+t+'\\n'); })"
            ".catch(e=>{console.error(e); process.exit(1);});")
    r = _node(code)
    assert r.returncode == 0, r.stderr
    data, thrown = r.stdout.strip().split("\n")
    import base64
    got = np.frombuffer(base64.b64decode(data), np.uint8).reshape(64, 64, 4)
    _, grgba = pyoracle.golden_image(tag, 64, 64)
    assert np.array_equal(got, grgba)
    assert thrown == "throws"
