"""Re-entrancy of the C-ABI (include/jsrt.h: renders of one scene are re-entrant).

Node runs each render() as napi async work on the libuv pool and the worker harness keeps one addon
instance per worker thread, so several renders of one scene (or of several scenes) may be in flight
on different host threads.  ctypes releases the GIL around the call, so these Python threads really
overlap inside libjsrt: the SDF scene takes the persistent-cast path (persistent_grid's per-kernel
cache), the second render of a scene finds its cached wavefront busy and uses its own buffers."""
import threading

import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.gpu


def _run_concurrently(jobs):
    out, errs = [None] * len(jobs), []

    def go(k):
        try:
            out[k] = jobs[k]()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)
    ts = [threading.Thread(target=go, args=(k,)) for k in range(len(jobs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return out


@pytest.mark.parametrize("scene,W,H,spp", [("SDF_Menger", 96, 80, 2), ("cornell_box_path", 96, 96, 4)])
def test_gpu_concurrent_renders_of_one_scene(scene, W, H, spp):
    import jsraytracer_amd as jr
    blob = pyoracle.golden_scene(scene)
    depth = pyoracle.scene_header(blob)["max_depth"]
    serial = jr.Scene(blob, device=0).render(W, H, spp, depth, 1, 3)
    shared = jr.Scene(blob, device=0)
    res = _run_concurrently([lambda: shared.render(W, H, spp, depth, 1, 3)] * 4)
    for rgba, colors, _ in res:
        assert np.array_equal(rgba, serial[0])
        assert np.array_equal(colors.view(np.uint32), serial[1].view(np.uint32))


def test_gpu_concurrent_renders_of_fresh_scenes():
    """First renders of fresh SDF scenes on several threads at once: each fills persistent_grid's
    cache for its kernels while the others read it."""
    import jsraytracer_amd as jr
    blob = pyoracle.golden_scene("SDF_Menger")
    depth = pyoracle.scene_header(blob)["max_depth"]
    ref = jr.Scene(blob, device=0).render(64, 48, 1, depth, 1, 9)[0]
    res = _run_concurrently([lambda: jr.Scene(blob, device=0).render(64, 48, 1, depth, 1, 9)] * 6)
    for rgba, _, _ in res:
        assert np.array_equal(rgba, ref)
