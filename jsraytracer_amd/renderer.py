"""Host-side mirror of the reference's renderer interface, backed by the HIP library.

Reference: src/renderers.js (SimpleRenderer.render :10-41, IncrementalMultisamplingRenderer.render
:70-117), src/pixelbuffer.js (PixelBuffer :1-50), src/worker.js (:17-40).  Same names, argument
meaning and error behaviour: ``render(img, timelimit=0, callback=False, x_offset=0, x_delt=1)``
fills ``img``'s RGBA8 bytes for the columns px = x_offset, x_offset + x_delt, ... and calls
``callback({"pass": p, "completion": c})`` no more often than every ``timelimit`` ms.
"""
import ctypes

import numpy as np

from . import _native
from ._native import JsrtError, Params, Stats, check

RENDERER_KINDS = {"SimpleRenderer": 0, "IncrementalMultisamplingRenderer": 1, "RandomMultisamplingRenderer": 2}
MODE_STRICT, MODE_FAST = 0, 1  # include/jsrt.h JSRT_MODE_*: numeric modes; only strict is built
MODES = {"strict": MODE_STRICT, "fast": MODE_FAST}


def mode_code(mode):
    """None / "strict" / "fast" / an int -> JSRT_MODE_* (the library refuses what it does not build)."""
    if mode is None:
        return MODE_STRICT
    if isinstance(mode, str):
        if mode not in MODES:
            raise JsrtError(f"unknown numeric mode {mode!r}")
        return MODES[mode]
    return int(mode)


class PixelBuffer:
    """pixelbuffer.js:1-50 — RGBA8 image (ImageData-like) with the reference's setColor rules."""

    def __init__(self, width, height=None):
        if isinstance(width, np.ndarray):
            self.imgdata = width
        else:
            self.imgdata = np.zeros((height, width, 4), np.uint8)  # new ImageData: zero-filled

    def width(self):
        return self.imgdata.shape[1]

    def height(self):
        return self.imgdata.shape[0]

    def coord(self, x, y):
        return y * (self.width() * 4) + x * 4

    def getColor(self, x, y):
        return self.imgdata[y, x].astype(np.float64) / 255


class Scene:
    """A JSRT scene blob (include/jsrt_scene.h) uploaded to one HIP device."""

    def __init__(self, blob, device=0):
        L = _native.lib()
        if L.jsrt_device_count() <= 0:
            raise JsrtError("no HIP device visible: the MI355X renderer has no CPU fallback")
        self._blob = bytes(blob)
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(self._blob, len(self._blob))
        check(L.jsrt_scene_create(buf, len(self._blob), device, ctypes.byref(h)), "jsrt_scene_create")
        self._h = h
        self.device = device

    def cast(self, rays, min_dist=0.0, max_dist=float("inf"), intersect_transparent=True):
        """World.cast (world.js:28-30) of rays (n x 6 f32: origin xyz w=1, direction xyz w=0) on the
        device: (distance f64, hit Primitive's OBJS index i32, -1 none) per ray."""
        import numpy as np
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = len(rays)
        t = np.empty(n, np.float64)
        obj = np.empty(n, np.int32)
        check(_native.lib().jsrt_cast(self._h, rays.ctypes.data, n, min_dist, max_dist, int(bool(intersect_transparent)),
                                      t.ctypes.data, obj.ctypes.data), "jsrt_cast")
        return t, obj

    def material_data(self, rays):
        """World.color(ray, 1) up to Material.color (include/jsrt.h jsrt_material_data): dict of t, obj,
        normal (n x 4), position (n x 4), uv (n x 3), bary (n x 3), basecolor (n x 3); NaN = absent."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        n = len(rays)
        out = {"t": np.empty(n, np.float64), "obj": np.empty(n, np.int32)}
        for k, w in (("normal", 4), ("position", 4), ("uv", 3), ("bary", 3), ("basecolor", 3)):
            out[k] = np.empty((n, w), np.float32)
        check(_native.lib().jsrt_material_data(self._h, rays.ctypes.data, n, out["t"].ctypes.data,
                                               out["obj"].ctypes.data, out["normal"].ctypes.data,
                                               out["position"].ctypes.data, out["uv"].ctypes.data,
                                               out["bary"].ctypes.data, out["basecolor"].ctypes.data),
              "jsrt_material_data")
        return out

    def sdf_distance(self, obj, points):
        """SDF.distance of SDFGeometry primitive `obj` (OBJS index) at local points (include/jsrt.h)."""
        points = np.ascontiguousarray(points, np.float32).reshape(-1, 4)
        out = np.empty(len(points), np.float64)
        check(_native.lib().jsrt_sdf_distance(self._h, int(obj), points.ctypes.data, len(points), out.ctypes.data),
              "jsrt_sdf_distance")
        return out

    def close(self):
        if getattr(self, "_h", None):
            _native.lib().jsrt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def params(width=0, height=0, spp=0, max_depth=0, kind=-1, seed=1, x_offset=0, x_delt=1, device=0,
               samples_per_launch=0, timelimit_ms=0.0, max_paths=0, stage_events=0, mode=MODE_STRICT, device_mask=0):
        return Params(width, height, spp, max_depth, kind, seed, x_offset, x_delt, device, samples_per_launch,
                      timelimit_ms, max_paths, stage_events, mode, device_mask)

    def render(self, width=0, height=0, spp=0, max_depth=0, kind=-1, seed=1, x_offset=0, x_delt=1,
               samples_per_launch=0, rgba=None, want_colors=True, progress=None, timelimit_ms=0.0, max_paths=0,
               mode=None, device_mask=0):
        """Render into host arrays.  Returns (rgba u8[H,W,4], colors f32[H,W,4] or None, stats).
        mode: "strict" (the only numeric mode built; "fast" raises) or MODE_*; device_mask: bit d = HIP device d
        renders part of the columns (jsrt.h jsrt_params::device_mask; 0 = the scene's device)."""
        L = _native.lib()
        p = self.params(width, height, spp, max_depth, kind, seed, x_offset, x_delt, self.device,
                        samples_per_launch, timelimit_ms, max_paths, mode=mode_code(mode), device_mask=device_mask)
        W = width if width > 0 else self.header()["width"]
        H = height if height > 0 else self.header()["height"]
        if rgba is None:
            rgba = np.zeros((H, W, 4), np.uint8)
        assert rgba.shape == (H, W, 4) and rgba.dtype == np.uint8 and rgba.flags.c_contiguous
        colors = np.full((H, W, 4), np.nan, np.float32) if want_colors else None
        st = Stats()
        cb = PROGRESS_NONE
        if progress is not None:
            cb = _native.PROGRESS_FN(lambda ps, c, u: progress(int(ps), float(c)))
        rc = L.jsrt_render(self._h, ctypes.byref(p), rgba.ctypes.data,
                           colors.ctypes.data if colors is not None else None, cb, None, ctypes.byref(st))
        check(rc, "jsrt_render")
        return rgba, colors, st.as_dict()

    def render_device(self, d_rgba_ptr, d_colors_ptr=None, stream_ptr=0, col_block=1, stats=True, progress=None,
                      progress_ex=None, **kw):
        """Render owned columns into device buffers (see jsrt.h jsrt_render_device).  stats=False
        records no per-launch HIP events (and returns None).  progress(pass, completion): called at the
        timelimit_ms cadence with the device buffers holding the running mean of the passes done (Incremental;
        jsrt_render_device_progress) -- synchronous, the stream idle in the callback.
        progress_ex(pass, completion, clean) -> truthy to abort (jsrt_render_device_progress_ex): called for every
        reported pass, clean or not (the multi-rank form, tiles.render_progressive); an exception it raises
        aborts the frame and is re-raised here."""
        L = _native.lib()
        p = self.params(device=self.device, **kw)
        st = Stats() if stats else None
        if progress is None and progress_ex is None:
            rc = L.jsrt_render_device(self._h, ctypes.byref(p), col_block, d_rgba_ptr, d_colors_ptr, stream_ptr,
                                      ctypes.byref(st) if stats else None)
            check(rc, "jsrt_render_device")
            return st.as_dict() if stats else None
        err = []
        if progress_ex is not None:
            def tramp_ex(pass_, completion, clean, _user):
                try:
                    return 1 if progress_ex(int(pass_), float(completion), bool(clean)) else 0
                except BaseException as e:  # noqa: BLE001 -- re-raised after the frame
                    err.append(e)
                    return 1
            cb = _native.PROGRESS_EX_FN(tramp_ex)
            rc = L.jsrt_render_device_progress_ex(self._h, ctypes.byref(p), col_block, d_rgba_ptr, d_colors_ptr,
                                                  stream_ptr, cb, None, ctypes.byref(st) if stats else None)
            if err:
                raise err[0]
            if rc == _native.RC_ABORTED:
                return None
            check(rc, "jsrt_render_device_progress_ex")
            return st.as_dict() if stats else None

        def tramp(pass_, completion, _user):
            try:
                progress(int(pass_), float(completion))
            except BaseException as e:  # noqa: BLE001 -- re-raised after the frame
                err.append(e)
        cb = _native.PROGRESS_FN(tramp)
        rc = L.jsrt_render_device_progress(self._h, ctypes.byref(p), col_block, d_rgba_ptr, d_colors_ptr, stream_ptr,
                                           cb, None, ctypes.byref(st) if stats else None)
        if err:
            raise err[0]
        check(rc, "jsrt_render_device_progress")
        return st.as_dict() if stats else None

    def render_device_accum(self, d_accum_ptr, stream_ptr=0, col_block=1, stats=True, **kw):
        """Render owned columns into a device f32 accumulator (jsrt.h jsrt_render_device_accum: ncols * H * 4 f32,
        [owned column][row], w = 0), the multi-GPU accumulator exchange's tile; no RGBA8."""
        L = _native.lib()
        p = self.params(device=self.device, **kw)
        st = Stats() if stats else None
        check(L.jsrt_render_device_accum(self._h, ctypes.byref(p), col_block, d_accum_ptr, stream_ptr,
                                         ctypes.byref(st) if stats else None), "jsrt_render_device_accum")
        return st.as_dict() if stats else None

    def header(self):
        return scene_header(self._blob)


PROGRESS_NONE = ctypes.cast(None, _native.PROGRESS_FN)


def finish_accum(d_accum_ptr, n, kind, passes, d_rgba_ptr, d_colors_ptr=None, stream_ptr=0):
    """setColor of n device accumulators (jsrt.h jsrt_finish_accum): RGBA8 (+ f32 colours) on a device stream."""
    check(_native.lib().jsrt_finish_accum(d_accum_ptr, int(n), int(kind), int(passes), d_rgba_ptr, d_colors_ptr,
                                          stream_ptr), "jsrt_finish_accum")


def owned_columns(width, x_offset, x_delt, col_block=1):
    return int(_native.lib().jsrt_owned_columns(width, x_offset, x_delt, col_block))


def scene_header(blob):
    import struct
    magic, version, nsec, _ = struct.unpack_from("<4I", blob, 0)
    if magic != 0x5452534A or version != 1:
        raise JsrtError("not a JSRT v1 scene blob")
    for i in range(nsec):
        tag, count, off, nbytes = struct.unpack_from("<IIQQ", blob, 16 + 24 * i)
        if tag == 0x52444E52:  # 'RNDR'
            kind, spp, depth, w, h = struct.unpack_from("<5I", blob, off)
            return {"kind": kind, "spp": spp, "max_depth": depth, "width": w, "height": h}
    raise JsrtError("scene blob has no renderer record")


class HipRenderer:
    """Drop-in for SimpleRenderer / IncrementalMultisamplingRenderer / RandomMultisamplingRenderer
    (renderers.js).  ``scene`` is a Scene (or blob); kind/spp/depth default to the blob's renderer."""

    def __init__(self, scene, samplesPerPixel=None, maxRecursionDepth=None, kind=None, seed=1, device=0, mode="strict",
                 device_mask=0):
        self.scene = scene if isinstance(scene, Scene) else Scene(scene, device)
        self.mode, self.device_mask = mode, device_mask  # jsrt_params::mode / device_mask
        hdr = self.scene.header()
        self.kind = hdr["kind"] if kind is None else (RENDERER_KINDS[kind] if isinstance(kind, str) else kind)
        self.samplesPerPixel = hdr["spp"] if samplesPerPixel is None else samplesPerPixel
        self.maxRecursionDepth = hdr["max_depth"] if maxRecursionDepth is None else maxRecursionDepth
        self.seed = seed

    @staticmethod
    def computePixelCount(img, x_offset, x_delt):  # renderers.js:7-9
        return ((img.width() / x_delt) + round(1 - x_offset / x_delt) * (img.width() % x_delt)) * img.height()

    def render(self, img, timelimit=0, callback=False, x_offset=0, x_delt=1):
        if x_delt <= 0:
            raise JsrtError("x_delt must be positive")
        progress = None
        spl = 0
        if timelimit and callback:
            # the Incremental renderer reports per pass (renderers.js:103-112): one sample per pixel per
            # launch, so each callback sees that pass's running mean in img; other kinds report on the
            # library's batches
            spl = 1 if self.kind == RENDERER_KINDS["IncrementalMultisamplingRenderer"] else 0

            def progress(p, c):
                callback({"pass": p, "completion": c})
        self.scene.render(img.width(), img.height(), self.samplesPerPixel, self.maxRecursionDepth, self.kind,
                          self.seed, x_offset, x_delt, samples_per_launch=spl, rgba=img.imgdata, want_colors=False,
                          progress=progress, timelimit_ms=float(timelimit or 0), mode=self.mode,
                          device_mask=self.device_mask)
        return img
