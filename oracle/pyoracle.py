"""TEST INFRASTRUCTURE ONLY — ctypes binding of the C oracle (oracle/jsrt_oracle.c).

The oracle is the CPU restatement of the reference render path used as the parity checker.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product (jsraytracer_amd) never does.
"""
import ctypes
import gzip
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libjsrt_oracle.so")
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")


class OracleParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("kind", ctypes.c_int32), ("seed", ctypes.c_uint32),
                ("x_offset", ctypes.c_int32), ("x_delt", ctypes.c_int32), ("threads", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


STAT_FIELDS = ["samples", "color_calls", "casts", "object_tests", "node_visits", "tri_tests", "sdf_evals", "draws",
               "shadow_casts", "shadow_object_tests", "shadow_node_visits", "shadow_tri_tests", "shadow_sdf_evals"]


class OracleStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in STAT_FIELDS]


def build():
    """Compile the oracle with its own Makefile (gcc, strict IEEE)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.jsrt_oracle_render.restype = ctypes.c_int
        L.jsrt_oracle_render.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(OracleParams),
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(OracleStats)]
        L.jsrt_oracle_render_accum.restype = ctypes.c_int
        L.jsrt_oracle_render_accum.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(OracleParams),
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.POINTER(OracleStats)]
        L.jsrt_oracle_last_error.restype = ctypes.c_char_p
        L.jsrt_oracle_fmod.restype = ctypes.c_double
        L.jsrt_oracle_fmod.argtypes = [ctypes.c_double, ctypes.c_double]
        L.jsrt_oracle_to_precision8.restype = ctypes.c_double
        L.jsrt_oracle_to_precision8.argtypes = [ctypes.c_double]
        L.jsrt_oracle_rng.restype = ctypes.c_double
        L.jsrt_oracle_rng.argtypes = [ctypes.c_uint32] * 5
        L.jsrt_oracle_mix.restype = ctypes.c_uint32
        L.jsrt_oracle_mix.argtypes = [ctypes.c_uint32] * 2
        L.jsrt_oracle_cast.restype = ctypes.c_int
        L.jsrt_oracle_cast.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_void_p]
        L.jsrt_oracle_material_data.restype = ctypes.c_int
        L.jsrt_oracle_material_data.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t] + \
            [ctypes.c_void_p] * 7
        L.jsrt_oracle_sdf_distance.restype = ctypes.c_int
        L.jsrt_oracle_sdf_distance.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_void_p]
        _lib = L
    return _lib


def render(blob, width=0, height=0, spp=0, max_depth=0, kind=-1, seed=1, x_offset=0, x_delt=1, threads=None,
           accum=False):
    """Render with the oracle. Returns (colors f32[H,W,4], rgba u8[H,W,4], stats dict) and, with accum=True, the
    renderer's f32 accumulators f32[H,W,4] (rgb, w = 0) as a fourth item."""
    L = lib()
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    p = OracleParams(width, height, spp, max_depth, kind, seed, x_offset, x_delt, threads, 0)
    hdr = scene_header(blob)
    W = width if width > 0 else hdr["width"]
    H = height if height > 0 else hdr["height"]
    colors = np.full((H, W, 4), np.nan, np.float32)
    rgba = np.zeros((H, W, 4), np.uint8)
    st = OracleStats()
    buf = ctypes.create_string_buffer(bytes(blob), len(blob))
    acc = np.zeros((H, W, 4), np.float32) if accum else None
    rc = L.jsrt_oracle_render_accum(buf, len(blob), ctypes.byref(p), colors.ctypes.data, rgba.ctypes.data,
                                    acc.ctypes.data if accum else None, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError("oracle: " + L.jsrt_oracle_last_error().decode())
    stats = {n: getattr(st, n) for n in STAT_FIELDS}
    return (colors, rgba, stats, acc) if accum else (colors, rgba, stats)


def scene_header(blob):
    """Minimal blob reader: renderer record fields (kind, spp, depth, width, height)."""
    import struct
    magic, version, nsec, _ = struct.unpack_from("<4I", blob, 0)
    assert magic == 0x5452534A and version == 1
    for i in range(nsec):
        tag, count, off, nbytes = struct.unpack_from("<IIQQ", blob, 16 + 24 * i)
        if tag == 0x52444E52:  # 'RNDR'
            kind, spp, depth, w, h = struct.unpack_from("<5I", blob, off)
            return {"kind": kind, "spp": spp, "max_depth": depth, "width": w, "height": h}
    raise ValueError("no renderer record")


# ---- golden fixtures (generated from the reference by oracle/refharness/regen_goldens.sh) ----
def golden_index():
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)["renders"]


def golden_scene(name):
    with gzip.open(os.path.join(GOLDEN, "scenes", name + ".jsrt.gz"), "rb") as f:
        return f.read()


def golden_image(tag, width, height):
    rgba = np.fromfile(os.path.join(GOLDEN, "images", tag + ".rgba"), np.uint8).reshape(height, width, 4)
    colors = np.fromfile(os.path.join(GOLDEN, "images", tag + ".f32"), np.float32).reshape(height, width, 4)
    return colors, rgba


def golden_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def cast(blob, rays, min_dist=0.0, max_dist=float("inf"), transparent=True):
    """World.cast (world.js:28-30) of rays (n x 6 f32: origin xyz w=1, direction xyz w=0):
    (distance f64, hit Primitive's OBJS index i32, -1 none)."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = len(rays)
    t = np.empty(n, np.float64)
    obj = np.empty(n, np.int32)
    L = lib()
    if L.jsrt_oracle_cast(bytes(blob), len(blob), rays.ctypes.data, n, min_dist, max_dist, int(bool(transparent)),
                          t.ctypes.data, obj.ctypes.data):
        raise RuntimeError(L.jsrt_oracle_last_error().decode())
    return t, obj


def material_data(blob, rays):
    """World.color(ray, 1) up to Material.color (world.js:31-41, 125-137): dict of t (f64), obj (i32),
    normal (n x 4), position (n x 4), uv (n x 3), bary (n x 3), basecolor (n x 3) f32, NaN = absent."""
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = len(rays)
    out = {"t": np.empty(n, np.float64), "obj": np.empty(n, np.int32)}
    for k, w in (("normal", 4), ("position", 4), ("uv", 3), ("bary", 3), ("basecolor", 3)):
        out[k] = np.empty((n, w), np.float32)
    L = lib()
    if L.jsrt_oracle_material_data(bytes(blob), len(blob), rays.ctypes.data, n, out["t"].ctypes.data,
                                   out["obj"].ctypes.data, out["normal"].ctypes.data, out["position"].ctypes.data,
                                   out["uv"].ctypes.data, out["bary"].ctypes.data, out["basecolor"].ctypes.data):
        raise RuntimeError(L.jsrt_oracle_last_error().decode())
    return out


def sdf_distance(blob, obj, points):
    """SDF.distance (sdf.js:53-74) of SDFGeometry primitive `obj`'s root at local points (n x 4 f32)."""
    points = np.ascontiguousarray(points, np.float32).reshape(-1, 4)
    out = np.empty(len(points), np.float64)
    L = lib()
    if L.jsrt_oracle_sdf_distance(bytes(blob), len(blob), int(obj), points.ctypes.data, len(points), out.ctypes.data):
        raise RuntimeError(L.jsrt_oracle_last_error().decode())
    return out


def golden_material(name):
    """Known answers computed by the reference (oracle/refharness/make_material_kats.js): the material_data
    of hits ("material": rays, t, obj, normal, position, uv, bary, basecolor) and SDF.distance samples
    ("sdf": [{obj, points, distance}])."""
    import base64
    with gzip.open(os.path.join(GOLDEN, "material", name + ".json.gz"), "rt") as f:
        d = json.load(f)
    m = d["material"]
    shapes = {"rays": (np.float32, 6), "t": (np.float64, 0), "obj": (np.int32, 0), "normal": (np.float32, 4),
              "position": (np.float32, 4), "uv": (np.float32, 3), "bary": (np.float32, 3), "basecolor": (np.float32, 3)}
    for k, (dt, w) in shapes.items():
        a = np.frombuffer(base64.b64decode(m[k]), dt)
        m[k] = a.reshape(-1, w) if w else a
    for e in d["sdf"]:
        e["points"] = np.frombuffer(base64.b64decode(e["points"]), np.float32).reshape(-1, 4)
        e["distance"] = np.frombuffer(base64.b64decode(e["distance"]), np.float64)
    return d


def golden_material_scenes():
    return sorted(f[:-len(".json.gz")] for f in os.listdir(os.path.join(GOLDEN, "material")) if f.endswith(".json.gz"))


def golden_casts(name):
    """World.cast known answers computed by the reference (oracle/refharness/make_cast_kats.js):
    {"blob_sha256", "sets": [{name, minD, maxD, transp, rays (n x 6 f32), t (f64), obj (i32)}]}."""
    import base64
    with gzip.open(os.path.join(GOLDEN, "casts", name + ".json.gz"), "rt") as f:
        d = json.load(f)
    for s in d["sets"]:
        s["maxD"] = float(s["maxD"])
        s["rays"] = np.frombuffer(base64.b64decode(s["rays"]), np.float32).reshape(-1, 6)
        s["t"] = np.frombuffer(base64.b64decode(s["t"]), np.float64)
        s["obj"] = np.frombuffer(base64.b64decode(s["obj"]), np.int32)
    return d


def golden_cast_scenes():
    return sorted(f[:-len(".json.gz")] for f in os.listdir(os.path.join(GOLDEN, "casts")) if f.endswith(".json.gz"))


# ---- mesh fixtures (oracle/refharness/regen_mesh_fixtures.sh): skeleton + OBJ + MTL per scene ----
MESHES = os.path.join(GOLDEN, "meshes")


def mesh_topology():
    with open(os.path.join(MESHES, "topology.json")) as f:
        return json.load(f)


def mesh_index():
    with open(os.path.join(MESHES, "index.json")) as f:
        return json.load(f)["renders"]


def mesh_scene(name, jr=None):
    """(blob, [info per tree]) of a mesh scene: its reference-exported skeleton with every OBJ (and its
    mtllib files) attached by the native ingest (include/jsrt_mesh.h), one BVHAggregate.build each, in
    the reference's call order.  The trees are pinned to the reference's by tests/test_mesh_build.py."""
    if jr is None:
        import jsraytracer_amd as jr
    topo = mesh_topology()[name]

    def read(f):
        with gzip.open(os.path.join(MESHES, f), "rb") as g:
            return g.read()
    blob, infos = read(topo["skeleton"]), []
    for t in topo["trees"]:
        blob, info = jr.attach_obj(blob, read(t["obj_fixture"]), bvh_object=t["bvh_object"],
                                   mtl_texts=[read(m) for m in t["mtl_fixtures"]])
        infos.append(info)
    return blob, infos
