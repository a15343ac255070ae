"""Native mesh ingest (include/jsrt_mesh.h): OBJ text -> Triangle primitives -> BVHAggregate.

Mirrors the reference's `loadObjFile(filename, defaultMaterial, callback, transform, minArea)`
(src/objloader.js:224-231) followed by `BVHAggregate.build(triangles, transform)`
(src/aggregates.js:33-41): the tree libjsrt builds is bit-identical to the reference's.  The scene
blob supplies a one-leaf BVHAggregate whose single Primitive is the template (material, per-triangle
transform, shadow flag) -- what the JS scene passes to loadObjFile -- and the aggregate's transform.
Host-only: runs without a GPU.
"""
import ctypes
import gzip

from . import _native


def attach_obj(blob, obj_text, bvh_object=-1, min_area=0.00001):
    """Return (new_blob: bytes, info: dict) with the OBJ's triangles and their BVH spliced into the
    BVHAggregate object `bvh_object` (< 0: the first one).  Raises JsrtError as the reference throws."""
    L = _native.lib()
    if isinstance(obj_text, str):
        obj_text = obj_text.encode()
    blob = bytes(blob)
    opt = _native.MeshOptions(int(bvh_object), 0, float(min_area))
    out, n, info = ctypes.c_void_p(), ctypes.c_size_t(), _native.MeshInfo()
    rc = L.jsrt_blob_attach_obj(blob, len(blob), obj_text, len(obj_text), ctypes.byref(opt), ctypes.byref(out),
                                ctypes.byref(n), ctypes.byref(info))
    _native.check(rc, "jsrt_blob_attach_obj")
    try:
        data = ctypes.string_at(out, n.value)
    finally:
        L.jsrt_blob_free(out)
    return data, {"triangles": int(info.triangles), "nodes": int(info.nodes), "max_depth": int(info.max_depth),
                  "bvh_object": int(info.bvh_object)}


def read_obj(path):
    """OBJ text from a file (gzip-compressed when the name ends in .gz)."""
    opener = gzip.open if str(path).endswith(".gz") else open
    with opener(path, "rb") as f:
        return f.read()


def load_obj_scene(skeleton_blob, obj_path, **kw):
    """Skeleton blob + OBJ file -> full scene blob (what the reference's test.mjs builds in JS)."""
    return attach_obj(skeleton_blob, read_obj(obj_path), **kw)
