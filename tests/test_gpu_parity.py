"""GPU parity: the HIP renderer (through the C-ABI) against the reference-generated goldens and the
oracle (oracle/jsrt_oracle.c, itself pinned bit-exact to the reference by test_oracle_golden.py).

Bar (BASELINE.json north_star): bit-exact on integer paths (RGBA8 bytes, RNG draw order), and
|dRGB| <= 1e-5 on the float colour handed to PixelBuffer.setColor.  In practice the kernels
reproduce the float colours bit for bit; the tolerance is asserted, bit-exactness is reported.
"""
import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.gpu
RENDERS = pyoracle.golden_index()
TOL = 1e-5


@pytest.fixture(scope="module")
def jr():
    import jsraytracer_amd as jr
    return jr


_scenes = {}


def _scene(jr, name):
    if name not in _scenes:
        _scenes[name] = jr.Scene(pyoracle.golden_scene(name), device=0)
    return _scenes[name]


def _compare(rgba, colors, grgba, gcol, label):
    bad = (rgba != grgba).any(-1)
    assert not bad.any(), f"{label}: {int(bad.sum())} RGBA8 pixels differ, max {int(np.abs(rgba.astype(int) - grgba).max())}"
    fin = np.isfinite(gcol[..., :3])
    assert np.array_equal(np.isfinite(colors[..., :3]), fin), f"{label}: NaN/inf pattern differs"
    err = float(np.abs(colors[..., :3][fin] - gcol[..., :3][fin]).max()) if fin.any() else 0.0
    assert err <= TOL, f"{label}: max |dRGB| {err}"


@pytest.mark.parametrize("tag", sorted(RENDERS))
def test_gpu_matches_reference_golden(jr, tag):
    r = RENDERS[tag]
    sc = _scene(jr, r["scene"])
    W, H = r["width"], r["height"]
    rgba = np.zeros((H, W, 4), np.uint8)
    rgba, colors, _ = sc.render(W, H, r["spp"], r["depth"], r["kind"], r["seed"], r.get("x_offset", 0),
                                r.get("x_delt", 1), rgba=rgba)
    gcol, grgba = pyoracle.golden_image(tag, W, H)
    if r.get("x_delt", 1) > 1:  # untouched columns stay zero (worker.js: fresh ImageData)
        cols = [c for c in range(W) if c >= r["x_offset"] and (c - r["x_offset"]) % r["x_delt"] == 0]
        assert not np.delete(rgba, cols, axis=1).any()
        rgba, colors, grgba, gcol = rgba[:, cols], colors[:, cols], grgba[:, cols], gcol[:, cols]
    _compare(rgba, colors, grgba, gcol, tag)


CONFIG_CASES = [  # (scene, W, H, spp, kind, seed) — larger than the goldens, checked against the oracle
    ("ASimpleScene", 256, 256, 1, 1, 3),
    ("cornell_box_path", 96, 96, 8, 1, 7),
    ("bunny", 128, 96, 1, 0, 1),
    ("bunny", 64, 48, 4, 1, 2),
    ("SDF_Menger", 48, 48, 2, 1, 4),
    ("refraction_path", 48, 48, 4, 1, 9),
    ("BoxBall_DOF", 64, 64, 2, 1, 6),
    ("heart", 64, 64, 2, 1, 5),
]


@pytest.mark.parametrize("case", CONFIG_CASES, ids=lambda c: f"{c[0]}_{c[1]}x{c[2]}_s{c[3]}")
def test_gpu_matches_oracle_larger(jr, case):
    name, W, H, spp, kind, seed = case
    blob = pyoracle.golden_scene(name)
    depth = pyoracle.scene_header(blob)["max_depth"]
    rgba, colors, st = _scene(jr, name).render(W, H, spp, depth, kind, seed)
    ocol, orgba, _ = pyoracle.render(blob, W, H, spp, depth, kind, seed)
    _compare(rgba, colors, orgba, ocol, f"{name} {W}x{H}x{spp}")
    assert st["samples"] == W * H * (spp if kind else 1)


def test_gpu_batching_is_invisible(jr):
    """The wavefront schedule's batch size (paths per batch) must not change a bit."""
    sc = _scene(jr, "cornell_box_path")
    a, ca, s1 = sc.render(40, 40, 6, 8, 1, 11)
    b, cb, s2 = sc.render(40, 40, 6, 8, 1, 11, max_paths=640)
    assert s2["batches"] > s1["batches"] >= 1
    assert np.array_equal(a, b) and np.array_equal(ca.view(np.uint32), cb.view(np.uint32))
    c, cc, _ = _scene(jr, "bunny").render(48, 40, 2, 4, 1, 3, max_paths=64)  # Fresnel: 2 children per hit
    d, cd, _ = _scene(jr, "bunny").render(48, 40, 2, 4, 1, 3)
    assert np.array_equal(c, d) and np.array_equal(cc.view(np.uint32), cd.view(np.uint32))


def test_gpu_frame_redo_paths(jr, monkeypatch):
    """Tree schedule: a batch that outgrows its pool, or a level that outgrows its learned launch
    bound, poisons the frame and the frame is redone; the result must not change a bit."""
    blob_b, blob_c = pyoracle.golden_scene("bunny"), pyoracle.golden_scene("cornell_box_path")
    ref_b = _scene(jr, "bunny").render(48, 40, 2, 4, 1, 3, max_paths=512)
    ref_c = _scene(jr, "cornell_box_path").render(40, 40, 6, 8, 1, 11, max_paths=640)
    monkeypatch.setenv("JSRT_POOL_FACTOR", "1")  # first pool far too small for Fresnel trees
    got_b = jr.Scene(blob_b, device=0).render(48, 40, 2, 4, 1, 3, max_paths=512)
    monkeypatch.delenv("JSRT_POOL_FACTOR")
    monkeypatch.setenv("JSRT_BOUND_MARGIN", "0.5")  # learned bounds below the real level counts
    got_c = jr.Scene(blob_c, device=0).render(40, 40, 6, 8, 1, 11, max_paths=640)
    assert got_b[2]["attempts"] > 1 and got_c[2]["attempts"] == 2  # both redo paths were taken
    for (a, ca, _), (b, cb, _) in ((ref_b, got_b), (ref_c, got_c)):
        assert np.array_equal(a, b) and np.array_equal(ca.view(np.uint32), cb.view(np.uint32))


@pytest.mark.parametrize("name,W,H,spp,seed", [("cornell_box_path", 48, 48, 4, 13), ("refraction_path", 40, 40, 4, 3),
                                               ("bunny", 48, 40, 2, 5)])
def test_gpu_exact_pick_fixup_path(jr, monkeypatch, name, W, H, spp, seed):
    """Every diffuse spherePick through k_fix_dirs (JSRT_FORCE_EXACT_PICK=1: each pick treated as unstable, its
    direction recomputed with fdlibm by the one-block kernel after k_shade), in the hybrid chain (cornell), the
    tree with two children per hit (refraction_path) and a mesh (bunny): the frame must equal the oracle's and
    the default path's bit for bit.  (Unforced, about one pick in 10^5 takes this path.)"""
    blob = pyoracle.golden_scene(name)
    depth = pyoracle.scene_header(blob)["max_depth"]
    ref = jr.Scene(blob, device=0).render(W, H, spp, depth, 1, seed)
    monkeypatch.setenv("JSRT_FORCE_EXACT_PICK", "1")
    got = jr.Scene(blob, device=0).render(W, H, spp, depth, 1, seed)
    monkeypatch.delenv("JSRT_FORCE_EXACT_PICK")
    ocol, orgba, _ = pyoracle.render(blob, W, H, spp, depth, 1, seed)
    _compare(got[0], got[1], orgba, ocol, f"{name} forced exact picks")
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1].view(np.uint32), got[1].view(np.uint32))


def test_gpu_progress_callback(jr):
    """renderers.js:103-112: callback({pass, completion}) while rendering, completion increasing."""
    sc = _scene(jr, "cornell_box_path")
    seen = []
    sc.render(64, 64, 8, 8, 1, 1, max_paths=4096, progress=lambda p, c: seen.append((p, c)), timelimit_ms=1e-6)
    assert seen and all(0 < c < 1 for _, c in seen)
    assert [c for _, c in seen] == sorted(c for _, c in seen)


@pytest.mark.parametrize("kind,spp", [(0, 1), (2, 3)])
def test_gpu_progress_simple_and_random(jr, kind, spp):
    """renderers.js:28-37: SimpleRenderer / RandomMultisamplingRenderer report {pass: 0, completion:
    pixels done / total} from inside their pixel loop; here after a batch when a callback is due.  A frame
    of several batches with a tiny timelimit fires callbacks with pass 0 and completion increasing in
    (0, 1); the image equals the render without a callback, through Scene.render and HipRenderer (whose
    48x40 frame is one batch: a callback never reports completion 1)."""
    sc = _scene(jr, "cornell_box_path")
    seen = []
    got, _, _ = sc.render(48, 40, spp, 8, kind, 3, want_colors=False, max_paths=512,
                          progress=lambda p, c: seen.append((p, c)), timelimit_ms=1e-6)
    assert seen and all(p == 0 and 0 < c < 1 for p, c in seen)
    assert [c for _, c in seen] == sorted(c for _, c in seen)
    ref, _, _ = sc.render(48, 40, spp, 8, kind, 3, want_colors=False)
    assert np.array_equal(got, ref)
    img = jr.PixelBuffer(48, 40)
    seen2 = []
    jr.HipRenderer(sc, samplesPerPixel=spp, maxRecursionDepth=8, kind=kind, seed=3).render(
        img, 1e-9, lambda p: seen2.append((p["pass"], p["completion"])))
    assert all(p == 0 and 0 < c < 1 for p, c in seen2)
    assert np.array_equal(img.imgdata, ref)


@pytest.mark.parametrize("scene,W,H,spp,depth,x_offset,x_delt", [
    ("cornell_box_path", 40, 32, 6, 8, 0, 1),   # chain schedule
    ("cornell_box_path", 40, 32, 4, 8, 1, 3),   # one worker's columns
    ("bunny", 32, 24, 4, 4, 0, 1),              # tree schedule (Fresnel children)
])
def test_gpu_progress_preview_is_running_mean(jr, scene, W, H, spp, depth, x_offset, x_delt):
    """renderers.js:93-112: the Incremental renderer setColor()s the running mean every pass, so the
    img its callback sees after pass p is the frame of the first p+1 samples.  The keyed RNG makes
    sample k of a pixel independent of spp, so that frame is the spp=p+1 render, bit for bit."""
    sc = _scene(jr, scene)
    img = np.zeros((H, W, 4), np.uint8)
    snaps = {}
    sc.render(W, H, spp, depth, 1, 5, x_offset, x_delt, samples_per_launch=1, rgba=img, want_colors=False,
              progress=lambda p, c: snaps.__setitem__(p, img.copy()), timelimit_ms=1e-6)
    assert sorted(snaps) == list(range(spp - 1))  # every pass but the last, which the final write covers
    for p, snap in snaps.items():
        ref = np.zeros((H, W, 4), np.uint8)
        ref, _, _ = sc.render(W, H, p + 1, depth, 1, 5, x_offset, x_delt, rgba=ref, want_colors=False)
        assert np.array_equal(snap, ref), f"{scene} pass {p}: {int((snap != ref).any(-1).sum())} pixels differ"
    final, _, _ = sc.render(W, H, spp, depth, 1, 5, x_offset, x_delt, want_colors=False)
    assert np.array_equal(img, final)


def test_gpu_partition_invariance(jr):
    """renderers.js:88 column interleave: N workers' images composite to the single-worker image."""
    sc = _scene(jr, "cornell_box_path")
    full, fcol, _ = sc.render(36, 28, 3, 8, 1, 21)
    comp = np.zeros_like(full)
    for k in range(4):
        part = np.zeros_like(full)
        part, pcol, _ = sc.render(36, 28, 3, 8, 1, 21, k, 4, rgba=part)
        comp[:, k::4] = part[:, k::4]
        assert not part[:, [c for c in range(36) if c % 4 != k]].any()
    assert np.array_equal(comp, full)


def test_gpu_device_output_block_partition(jr):
    """jsrt_render_device with column blocks (the multi-GPU tile layout) equals the host path."""
    torch = pytest.importorskip("torch")
    sc = _scene(jr, "ASimpleScene")
    W, H = 72, 40
    full, fcol, _ = sc.render(W, H, 2, 4, 1, 5)
    comp = np.zeros_like(full)
    for r in range(3):
        nc = jr.owned_columns(W, r, 3, 8)
        d = torch.zeros(nc * H, dtype=torch.int32, device="cuda:0")
        sc.render_device(d.data_ptr(), col_block=8, width=W, height=H, spp=2, max_depth=4, kind=1, seed=5,
                         x_offset=r, x_delt=3)
        torch.cuda.synchronize()
        got = d.cpu().numpy().view(np.uint8).reshape(nc, H, 4)
        cols = [c for c in range(W) if (c // 8) % 3 == r]
        assert len(cols) == nc
        comp[:, cols] = got.transpose(1, 0, 2)
    assert np.array_equal(comp, full)


def test_gpu_bad_scene_raises(jr):
    with pytest.raises(jr.JsrtError):
        jr.Scene(b"not a scene blob at all", device=0)
