"""ctypes binding of libjsrt.so (include/jsrt.h).

The library is built in-tree (jsraytracer_amd/_build/libjsrt.so, see build.py) so the GPU box loads
exactly the code object compiled here.  There is no CPU fallback: if the library or a HIP device is
missing, every render entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JSRT_LIB") or os.path.join(HERE, "_build", "libjsrt.so")  # JSRT_LIB: A/B builds
ABI_VERSION = 4  # include/jsrt.h JSRT_ABI_VERSION: the Params / Stats layouts below
EVENTS_ONE_STREAM = 0x40000000  # include/jsrt.h JSRT_EVENTS_ONE_STREAM (a Params.stage_events flag)


class JsrtError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("kind", ctypes.c_int32), ("seed", ctypes.c_uint32),
                ("x_offset", ctypes.c_int32), ("x_delt", ctypes.c_int32), ("device", ctypes.c_int32),
                ("samples_per_launch", ctypes.c_int32), ("timelimit_ms", ctypes.c_double),
                ("max_paths", ctypes.c_int32), ("stage_events", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("device_mask", ctypes.c_uint32), ("reserved", ctypes.c_int32 * 2)]


STAGES = ["k_gen", "k_extend", "k_shade", "k_shadow", "k_reduce", "k_accum", "k_final", "k_resolve", "spare8",
          "spare9", "spare10", "spare11"]
NSTAGES = len(STAGES)  # JSRT_STAGES


class Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("samples", ctypes.c_uint64),
                ("launches", ctypes.c_uint32), ("batches", ctypes.c_uint32), ("stage_ms", ctypes.c_double * NSTAGES),
                ("stage_launches", ctypes.c_uint32 * NSTAGES), ("attempts", ctypes.c_uint32), ("events_lost", ctypes.c_uint32)]

    def as_dict(self):
        return {"kernel_ms": self.kernel_ms, "total_ms": self.total_ms, "samples": int(self.samples),
                "launches": int(self.launches), "batches": int(self.batches),
                "stage_ms": {STAGES[k]: self.stage_ms[k] for k in range(NSTAGES) if not STAGES[k].startswith("spare")},
                "stage_launches": {STAGES[k]: int(self.stage_launches[k]) for k in range(NSTAGES) if not STAGES[k].startswith("spare")},
                "attempts": int(self.attempts), "events_lost": int(self.events_lost)}


PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_int32, ctypes.c_double, ctypes.c_void_p)
# jsrt_progress_ex_fn(pass, completion, clean, user) -> non-zero aborts the frame
PROGRESS_EX_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_int32, ctypes.c_void_p)
RC_ABORTED = -4  # jsrt_render_device_progress_ex: the callback asked to stop the frame

# exported symbols of include/jsrt.h (checked by tests/test_capi_symbols.py)
EXPORTS = ["jsrt_scene_create", "jsrt_scene_destroy", "jsrt_render", "jsrt_render_device", "jsrt_cast",
           "jsrt_material_data", "jsrt_sdf_distance", "jsrt_owned_columns", "jsrt_last_error", "jsrt_abi_version",
           "jsrt_device_count", "jsrt_build_id", "jsrt_render_device_progress", "jsrt_render_device_progress_ex",
           "jsrt_render_device_accum", "jsrt_finish_accum"]
# exported symbols of include/jsrt_mesh.h (native OBJ ingest + BVH build; host-only, no GPU needed)
MESH_EXPORTS = ["jsrt_blob_attach_obj", "jsrt_blob_attach_obj_mtl", "jsrt_blob_free"]
# exported symbols of include/jsrt_json.h (Serializer-JSON reader; host-only)
JSON_EXPORTS = ["jsrt_blob_from_json"]


class MeshOptions(ctypes.Structure):
    _fields_ = [("bvh_object", ctypes.c_int32), ("pad", ctypes.c_int32), ("min_area", ctypes.c_double)]


class JsonInfo(ctypes.Structure):
    _fields_ = [("objects", ctypes.c_int64), ("triangles", ctypes.c_int64), ("bvh_nodes", ctypes.c_int64),
                ("psdata_matched", ctypes.c_int64)]


class MeshInfo(ctypes.Structure):
    _fields_ = [("triangles", ctypes.c_int64), ("nodes", ctypes.c_int64), ("max_depth", ctypes.c_int32),
                ("bvh_object", ctypes.c_int32)]

_lib = None


def lib():
    """Load libjsrt.so (raises JsrtError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 (same SONAME as
    # /opt/rocm's).  Loading torch first makes libjsrt bind to that already-loaded copy, so torch
    # tensors/streams/RCCL and libjsrt share one runtime (loading ours first breaks torch.cuda).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise JsrtError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__; __graft_entry__.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    # a stale library (the .so travels to the GPU box on its own) would write past Stats or misread it:
    # the ABI version first, before any other symbol is bound (a missing one would raise AttributeError)
    L.jsrt_abi_version.restype = ctypes.c_int32
    if L.jsrt_abi_version() != ABI_VERSION:
        raise JsrtError(f"{LIB_PATH}: ABI {L.jsrt_abi_version()}, these bindings expect {ABI_VERSION}: rebuild it")
    L.jsrt_build_id.restype = ctypes.c_char_p
    built = L.jsrt_build_id().decode()
    if not os.environ.get("JSRT_LIB"):  # A/B variants (JSRT_LIB) carry their own defines, hence their own id
        from . import build as _b
        try:
            want = _b.build_id()
        except OSError as e:  # a tree without the sources the id is computed from
            raise JsrtError(f"cannot verify {LIB_PATH}: its sources are missing ({e})") from e
        if built != want:
            raise JsrtError(f"{LIB_PATH} was built from other sources (build id {built}, this tree {want}): rebuild it")
    L.jsrt_scene_create.restype = ctypes.c_int
    L.jsrt_scene_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]
    L.jsrt_scene_destroy.restype = None
    L.jsrt_scene_destroy.argtypes = [ctypes.c_void_p]
    L.jsrt_render.restype = ctypes.c_int
    L.jsrt_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_void_p, ctypes.c_void_p,
                              PROGRESS_FN, ctypes.c_void_p, ctypes.POINTER(Stats)]
    L.jsrt_render_device.restype = ctypes.c_int
    L.jsrt_render_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(Stats)]
    L.jsrt_render_device_progress.restype = ctypes.c_int
    L.jsrt_render_device_progress.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, PROGRESS_FN, ctypes.c_void_p,
                                              ctypes.POINTER(Stats)]
    L.jsrt_render_device_progress_ex.restype = ctypes.c_int
    L.jsrt_render_device_progress_ex.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_int32,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, PROGRESS_EX_FN,
                                                 ctypes.c_void_p, ctypes.POINTER(Stats)]
    L.jsrt_render_device_accum.restype = ctypes.c_int
    L.jsrt_render_device_accum.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.POINTER(Stats)]
    L.jsrt_finish_accum.restype = ctypes.c_int
    L.jsrt_finish_accum.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p]
    L.jsrt_cast.restype = ctypes.c_int
    L.jsrt_cast.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
                            ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    L.jsrt_material_data.restype = ctypes.c_int
    L.jsrt_material_data.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_void_p] * 7
    L.jsrt_sdf_distance.restype = ctypes.c_int
    L.jsrt_sdf_distance.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.jsrt_owned_columns.restype = ctypes.c_int32
    L.jsrt_owned_columns.argtypes = [ctypes.c_int32] * 4
    L.jsrt_last_error.restype = ctypes.c_char_p
    L.jsrt_device_count.restype = ctypes.c_int32
    L.jsrt_blob_attach_obj.restype = ctypes.c_int
    L.jsrt_blob_attach_obj.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.POINTER(MeshOptions), ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(MeshInfo)]
    L.jsrt_blob_attach_obj_mtl.restype = ctypes.c_int
    L.jsrt_blob_attach_obj_mtl.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(MeshOptions),
                                           ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                           ctypes.POINTER(MeshInfo)]
    L.jsrt_blob_from_json.restype = ctypes.c_int
    L.jsrt_blob_from_json.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(JsonInfo)]
    L.jsrt_blob_free.restype = None
    L.jsrt_blob_free.argtypes = [ctypes.c_void_p]
    _lib = L
    return L


def build_id():
    """The build id embedded in the loaded library (hash of its sources, flags and defines)."""
    return lib().jsrt_build_id().decode()


def last_error():
    return lib().jsrt_last_error().decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise JsrtError(f"{what} failed ({rc}): {last_error()}")
