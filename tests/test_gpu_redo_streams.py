"""A frame rendered on two batch streams must be complete when jsrt_render_device returns, on every schedule,
including a frame that is redone because a batch outgrew its pool or a learned launch bound.

Round 4 saw this fail once mid-round (gpurun_out/gpu_tests_r04_s2.log, the bench's two-rank gloo rehearsal:
2,493 of 4,096 oracle-checked pixels wrong, max |d| 109): in the draft of the hybrid chain schedule the frame
loop left through the plain chain's exit -- `if (e != hipSuccess || chain) break;` with `chain` true for the
hybrid layout -- before it read the frame flags, so a hybrid frame whose side chains outgrew their slots
(LVL_FLAG) was returned, never redone, with its poisoned batches' pixels missing (k_resolve_paths / k_accum
skip a poisoned batch).  The committed schedule reads the flags of both pools after every frame on every
schedule (render.hip render_frame).  Each case here renders through jsrt_render_device on a
caller stream, copies the tile on that same stream at once, and compares it with the oracle: the chain
schedule (no node with two children), the hybrid chain (flat scene with a Fresnel sphere) and the tree
(mesh), each over several batches on the two batch streams with an odd spp, plain and with the redo paths
forced.  The reference's workers post only complete images (src/worker.js:30-32)."""
import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.gpu

CASES = [  # scene, schedule it runs on, W, H, spp, max_paths (several batches -> two streams)
    ("BoxBall_path", "chain", 48, 40, 5, 4096),
    ("cornell_box_path", "hybrid", 48, 40, 5, 4096),
    ("refraction_path", "hybrid", 40, 40, 3, 1600),
    ("bunny_path", "tree", 40, 32, 3, 1280),
]
# JSRT_FIX_CAP=0 with every diffuse pick through k_fix_dirs (JSRT_FORCE_EXACT_PICK=1): the chain schedule's fix
# records run out on both pools, and the frame is redone with a record per ray slot on both (advisor, round 5:
# the redo used to enlarge only the first pool's records, so an overflow in a twin-pool batch failed again)
FIXCAP = {"JSRT_FIX_CAP": "0", "JSRT_FORCE_EXACT_PICK": "1"}
# both orders of a batch's paths (WArgs::pixel_major): a pixel's samples side by side, or sample by sample
# and the pixel-major batches' tile order (pixel_of) with partial tiles at the image edges
KNOBS = [{}, {"JSRT_POOL_FACTOR": "1"}, {"JSRT_BOUND_MARGIN": "0.5"}, FIXCAP, {"JSRT_PIXEL_MAJOR": "1"},
         {"JSRT_PIXEL_MAJOR": "0"}, {"JSRT_PIXEL_MAJOR": "1", "JSRT_TILE_PATCHES": "2"},
         {"JSRT_PIXEL_MAJOR": "1", "JSRT_TILE_PATCHES": "3", "JSRT_BATCH_SPP": "2"}]


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: "+".join(f"{a}={b}" for a, b in k.items()) or "default")
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}_{c[1]}")
def test_device_frame_complete_on_return(monkeypatch, case, knobs):
    torch = pytest.importorskip("torch")
    import jsraytracer_amd as jr
    name, sched, W, H, spp, max_paths = case
    if sched == "chain" and knobs and knobs is not FIXCAP and "JSRT_PIXEL_MAJOR" not in knobs:
        pytest.skip("the chain schedule has no learned pool or bounds")
    if sched != "chain" and knobs is FIXCAP:
        pytest.skip("fix-record redo: the chain schedule's (learned schedules grow their records with the pool)")
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    blob = pyoracle.golden_scene(name)
    depth = pyoracle.scene_header(blob)["max_depth"]
    sc = jr.Scene(blob, device=0)
    stream = torch.cuda.Stream()
    tile = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    kw = dict(width=W, height=H, spp=spp, max_depth=depth, kind=1, seed=3, max_paths=max_paths)
    with torch.cuda.stream(stream):
        tile.fill_(-1)  # (a pixel the frame never wrote reads as 0xFFFFFFFF)
        # stats=False: the call returns without waiting for the device (stats would synchronise the stream)
        sc.render_device(tile.data_ptr(), stream_ptr=stream.cuda_stream, stats=False, **kw)
        got = tile.clone()  # enqueued on the render's stream right behind it
    stream.synchronize()
    img = got.cpu().numpy().view(np.uint8).reshape(W, H, 4).transpose(1, 0, 2)  # [owned column][row] -> [row][col]
    _, ref, _ = pyoracle.render(blob, W, H, spp, depth, 1, 3)
    bad = (img != ref).any(-1)
    assert not bad.any(), f"{name} ({sched}, {knobs}): {int(bad.sum())} of {bad.size} pixels differ"
    # the same frame on a fresh scene, with stats: it ran as several batches, and the knob took the redo path
    st = jr.Scene(blob, device=0).render_device(tile.data_ptr(), stream_ptr=stream.cuda_stream, **kw)
    assert st["batches"] >= 3
    if knobs.get("JSRT_BOUND_MARGIN") or (knobs.get("JSRT_POOL_FACTOR") and sched == "tree") or knobs is FIXCAP:
        assert st["attempts"] >= 2
