"""Native reader of the reference's Serializer JSON (include/jsrt_json.h).

`blob_from_json(text)` is `Serializer.deserializeJSON(text)` (src/serializer.js:69-71) followed by the
scene export of jsraytracer_amd/js/scene_blob.js, in C++: the JSON that tests/test_to_json.js writes
(the input of the reference's dragon_json / toledo_json scenes) becomes the JSRT scene blob that
`Scene` / `HipRenderer` render.  Non-finite values the JSON wrote as null, and Triangle vertex
normals / UVs that Triangle.serialize drops (geometry.js:355-357), are restored as include/jsrt_json.h
describes; `psdata_objs` are the OBJ texts the meshes came from.  Host-only: runs without a GPU.
"""
import ctypes
import gzip

from . import _native


def _bytes(t):
    return t.encode() if isinstance(t, str) else bytes(t)


def blob_from_json(json_text, psdata_objs=()):
    """Return (blob: bytes, info: dict).  Raises JsrtError with the reader's message."""
    L = _native.lib()
    js = _bytes(json_text)
    side = b"\0".join(_bytes(t) for t in psdata_objs)
    out, n, info = ctypes.c_void_p(), ctypes.c_size_t(), _native.JsonInfo()
    rc = L.jsrt_blob_from_json(js, len(js), side, len(side), ctypes.byref(out), ctypes.byref(n), ctypes.byref(info))
    _native.check(rc, "jsrt_blob_from_json")
    try:
        data = ctypes.string_at(out, n.value)
    finally:
        L.jsrt_blob_free(out)
    return data, {k: int(getattr(info, k)) for k, _ in _native.JsonInfo._fields_}


def load_json_scene(path, psdata_obj_paths=()):
    """A test.json (gzip-compressed when the name ends in .gz) -> scene blob; see blob_from_json."""
    def rd(p):
        with (gzip.open if str(p).endswith(".gz") else open)(p, "rb") as f:
            return f.read()
    return blob_from_json(rd(path), [rd(p) for p in psdata_obj_paths])
