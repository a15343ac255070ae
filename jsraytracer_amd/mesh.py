"""Native mesh ingest (include/jsrt_mesh.h): OBJ text -> Triangle primitives -> BVHAggregate.

Mirrors the reference's `loadObjFile(filename, defaultMaterial, callback, transform, minArea)`
(src/objloader.js:224-231) followed by `BVHAggregate.build(triangles, transform)`
(src/aggregates.js:33-41): the tree libjsrt builds is bit-identical to the reference's.  The scene
blob supplies a one-leaf BVHAggregate whose single Primitive is the template (material, per-triangle
transform, shadow flag) -- what the JS scene passes to loadObjFile -- and the aggregate's transform.
`usemtl` takes its materials from the OBJ's mtllib files (parseMtlFile / makeMaterial,
objloader.js:9-20,58-123).  Host-only: runs without a GPU.
"""
import ctypes
import gzip
import os

from . import _native


def _bytes(t):
    return t.encode() if isinstance(t, str) else bytes(t)


def attach_obj(blob, obj_text, bvh_object=-1, min_area=0.00001, mtl_texts=()):
    """Return (new_blob: bytes, info: dict) with the OBJ's triangles and their BVH spliced into the
    BVHAggregate object `bvh_object` (< 0: the first one).  `mtl_texts`: the OBJ's mtllib files'
    texts in mtllib order.  Raises JsrtError as the reference throws."""
    L = _native.lib()
    obj_text, blob = _bytes(obj_text), bytes(blob)
    mtl = b"\0".join(_bytes(t) for t in mtl_texts)
    opt = _native.MeshOptions(int(bvh_object), 0, float(min_area))
    out, n, info = ctypes.c_void_p(), ctypes.c_size_t(), _native.MeshInfo()
    rc = L.jsrt_blob_attach_obj_mtl(blob, len(blob), obj_text, len(obj_text), mtl, len(mtl), ctypes.byref(opt),
                                    ctypes.byref(out), ctypes.byref(n), ctypes.byref(info))
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


def mtllibs(obj_text):
    """The `mtllib` names of an OBJ in file order (parseObjFile's first pass, objloader.js:153-162)."""
    out = []
    for line in _bytes(obj_text).split(b"\n"):
        t = line.split()
        if t and not t[0].startswith(b"#") and t[0] == b"mtllib":
            out.append((t[1] if len(t) > 1 else b"undefined").decode())
    return out


def load_obj_scene(skeleton_blob, obj_path, **kw):
    """Skeleton blob + OBJ file -> full scene blob (what the reference's test.mjs builds in JS).
    mtllib files are read next to the OBJ (loadObjFile's prefix, objloader.js:226-229); a `.gz` copy
    is used when the plain file is absent."""
    text = read_obj(obj_path)
    if "mtl_texts" not in kw:
        d, texts = os.path.dirname(str(obj_path)), []
        for name in mtllibs(text):
            p = os.path.join(d, name)
            texts.append(read_obj(p if os.path.exists(p) or not os.path.exists(p + ".gz") else p + ".gz"))
        kw["mtl_texts"] = texts
    return attach_obj(skeleton_blob, text, **kw)
