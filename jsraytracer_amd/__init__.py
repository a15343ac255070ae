"""jsraytracer_amd — MI355X-native drop-in for alitteneker/jsraytracer's CPU render path.

The product is libjsrt.so (include/jsrt.h): hand-written HIP kernels for gfx950 behind a C-ABI.
This package is the Python host side mirroring the reference's renderer interface
(src/renderers.js, src/pixelbuffer.js); the Node host side lives in jsraytracer_amd/js/.
"""
from ._native import JsrtError, LIB_PATH  # noqa: F401
from .renderer import HipRenderer, PixelBuffer, Scene, finish_accum, owned_columns, scene_header  # noqa: F401
from .mesh import attach_obj, load_obj_scene  # noqa: F401
from .serial import blob_from_json, load_json_scene  # noqa: F401

__all__ = ["HipRenderer", "PixelBuffer", "Scene", "JsrtError", "finish_accum", "owned_columns", "scene_header", "LIB_PATH",
           "attach_obj", "load_obj_scene", "blob_from_json", "load_json_scene"]
