"""jsrt_params' numeric mode and device mask (include/jsrt.h, ABI 4; SURVEY §8(b): `mode {strict, fast}`,
`device_mask`), through the C ABI on the GPU.

- mode: strict is the reference's numeric model and the only one built; fast (pure f32) is refused with -1 by
  every render entry point, never silently rendered in strict.
- device_mask: jsrt_render interleaves the call's owned columns over the masked devices (device j: x_offset +
  j * x_delt, step x_delt * k -- the reference's worker partition, src/renderers.js:88) and composites the host
  image.  The box has one GPU, so the split itself runs through JSRT_MASK_REPEAT (each masked device n times):
  the composite must equal the oracle's frame bit for bit, for the full frame and for a reference worker's
  partition.  A mask naming an invisible device, a mask with a progress callback, and a foreign mask on the
  device entry points are refused."""
import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene():
    import jsraytracer_amd as jr
    blob = pyoracle.golden_scene("cornell_box_path")
    return jr.Scene(blob, device=0), blob


def test_fast_mode_is_refused(scene):
    import jsraytracer_amd as jr
    sc, _ = scene
    with pytest.raises(jr.JsrtError, match="fast"):
        sc.render(16, 16, 1, 2, 1, 1, mode="fast")
    with pytest.raises(jr.JsrtError, match="unknown numeric mode"):
        sc.render(16, 16, 1, 2, 1, 1, mode=7)
    torch = pytest.importorskip("torch")
    t = torch.zeros(16 * 16, dtype=torch.int32, device="cuda:0")
    with pytest.raises(jr.JsrtError, match="fast"):
        sc.render_device(t.data_ptr(), width=16, height=16, spp=1, max_depth=2, kind=1, mode=1)
    rgba, _, _ = sc.render(16, 16, 1, 2, 1, 1, mode="strict")  # strict: renders
    assert rgba[..., 3].min() == 255


@pytest.mark.parametrize("x_offset,x_delt", [(0, 1), (1, 3)])
@pytest.mark.parametrize("repeat", [1, 3])
def test_device_mask_split_is_bit_exact(monkeypatch, scene, x_offset, x_delt, repeat):
    sc, blob = scene
    W, H, spp, depth = 40, 24, 3, 8
    monkeypatch.setenv("JSRT_MASK_REPEAT", str(repeat))
    rgba = np.zeros((H, W, 4), np.uint8)
    got, col, st = sc.render(W, H, spp, depth, 1, 5, x_offset, x_delt, rgba=rgba, device_mask=1)
    ocol, orgba, _ = pyoracle.render(blob, W, H, spp, depth, 1, 5, x_offset, x_delt)
    own = np.zeros(W, bool)
    own[x_offset::x_delt] = True
    assert np.array_equal(got[:, own], orgba[:, own])
    assert not got[:, ~own].any()  # columns the call does not own stay as the caller left them
    assert np.array_equal(col[:, own, :3].view(np.uint32), ocol[:, own, :3].view(np.uint32))
    assert st["samples"] == int(own.sum()) * H * spp


def test_device_mask_refusals(scene):
    import jsraytracer_amd as jr
    from jsraytracer_amd import _native
    sc, _ = scene
    with pytest.raises(jr.JsrtError, match="not visible"):
        sc.render(16, 16, 1, 2, 1, 1, device_mask=1 << 31)
    with pytest.raises(jr.JsrtError, match="single device"):
        sc.render(16, 16, 1, 2, 1, 1, device_mask=3, progress=lambda p, c: None, timelimit_ms=1e-9)
    torch = pytest.importorskip("torch")
    t = torch.zeros(16 * 16, dtype=torch.int32, device="cuda:0")
    with pytest.raises(jr.JsrtError, match="own device"):
        sc.render_device(t.data_ptr(), width=16, height=16, spp=1, max_depth=2, kind=1, device_mask=2)
    sc.render_device(t.data_ptr(), width=16, height=16, spp=1, max_depth=2, kind=1, device_mask=1)  # its own device
    assert _native.lib().jsrt_device_count() >= 1
