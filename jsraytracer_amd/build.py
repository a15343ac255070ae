"""Builds libjsrt.so in-tree with hipcc for gfx950 (no JIT caches: the .so travels to the GPU box).

The level kernels are compiled once per kernel profile (render_pf.hip with -DJSRT_PF=..., see
csrc/render_levels.h) as separate objects, all objects in parallel.
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libjsrt.so")
PROFILES = {"analytic": 0, "mesh": 9, "sdf": 4, "all": 15}  # device_scene.h PF_ANALYTIC / PF_MESH / PF_SDF / PF_ALL
HEADERS = ["device_common.h", "fdlibm.h", "js_number.h", "device_scene.h", "render_kernel.h", "render_levels.h", "scene_load.h", "sdf_forms.h",
           "sdf_program.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("JSRT_OFFLOAD_ARCH", "gfx950")

# Strict IEEE (the reference's numeric model): no FMA contraction, no fast-math,
# f32 denormals preserved (HIP's default), correctly rounded f32 div/sqrt (HIP's default).
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function"]

INCLUDE = os.path.join(HERE, "..", "include")
PUBLIC = ["jsrt.h", "jsrt_scene.h", "jsrt_mesh.h", "jsrt_json.h"]
# objects: (object stem, source, extra defines, dependencies); an object is rebuilt only when these change
UNITS = [("render", "render.hip", [], HEADERS + ["jsrt.h", "jsrt_scene.h"])]
# each profile in three parts (render_pf.hip JSRT_PART: chain kernels, tree kernels, single-cast entries)
UNITS += [(f"render_pf{pf}_{part}", "render_pf.hip", [f"-DJSRT_PF={pf}", f"-DJSRT_PART={part}"],
           HEADERS + ["jsrt.h", "jsrt_scene.h"]) for pf in PROFILES.values() for part in range(3)]
UNITS += [("capi", "capi.cpp", [], HEADERS + ["jsrt.h", "jsrt_scene.h"]),
          ("scene_load", "scene_load.cpp", [], HEADERS + ["jsrt.h", "jsrt_scene.h"]),
          ("mesh_build", "mesh_build.cpp", [], ["jsrt_mesh.h", "jsrt_scene.h", "obj_parse.h"]),
          ("json_scene", "json_scene.cpp", [], ["jsrt_json.h", "jsrt_scene.h", "obj_parse.h"])]
OBJ_FLAGS = [f for f in FLAGS if f != "-shared"]
# No machine-level loop-invariant code motion: it hoists address and f64-constant materialisations out
# of the light-sample and traversal loops into VGPRs and then spills them (k_shade_lit: 66 spilled
# VGPRs at 128; k_extend 80 -> 74 VGPRs without it).  -DJSRT_MACHINE_LICM (a variant define) keeps it.
NO_MLICM = ["-mllvm", "-disable-machine-licm"]


def _path(f):
    return os.path.join(INCLUDE, f) if f in PUBLIC else os.path.join(CSRC, f)


def build_id(defines=()):
    """Identity of a library build: a hash of every source and header it is compiled from, the compiler
    flags and the variant defines.  Embedded in libjsrt.so (jsrt_build_id) and recomputed from the tree by
    _native.lib(), which refuses a library built from other sources (the .so travels to the GPU box on its
    own, so a stale one would otherwise run silently)."""
    h = hashlib.sha256()
    files = sorted({src for _, src, _, _ in UNITS} | {d for _, _, _, deps in UNITS for d in deps})
    for f in files:
        h.update(f.encode() + b"\0")
        with open(_path(f), "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    # the flags without the target: a library built with JSRT_OFFLOAD_ARCH set is still the same sources' build
    # (its code object names its own target), and a run-time environment cannot make a valid library stale
    flags = [f for f in FLAGS if not f.startswith("--offload-arch=")]
    h.update(" ".join(flags + NO_MLICM + list(defines)).encode())
    return h.hexdigest()[:16]


def _id_file(lib):
    return lib + ".id"


def _write_id_unit(bid, tag):
    """A one-function translation unit exporting the build id (compiled into the library at link time)."""
    src = os.path.join(OUT, f"build_id{tag}.cpp")
    with open(src, "w") as f:
        f.write('extern "C" const char *jsrt_build_id(void) { return "%s"; }\n' % bid)
    return src


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _src_stamp(deps, cmd):
    """Content hash of an object's sources and its compile command (the object's .src sidecar): an object is
    rebuilt when its inputs' contents differ, whatever the mtimes say (a tool that rewrites an object in place,
    or a copy that keeps old mtimes, must not let a stale object into the library)."""
    h = hashlib.sha256(" ".join(cmd).encode())
    for d in deps:
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _obj_stale(o, deps, cmd):
    if not os.path.exists(o) or not os.path.exists(o + ".src"):
        return True
    with open(o + ".src") as f:
        return f.read().strip() != _src_stamp(deps, cmd)


def _obj(stem, tag=""):
    return os.path.join(OUT, f"{stem}{tag}.o")


def _deps(src, deps):
    return [os.path.join(CSRC, src)] + [_path(d) for d in deps]


def _cmd(src, defs, extra, o):
    """The hipcc command line of one object (the .tmp output is renamed over `o` once it succeeds)."""
    dev = [] if "-DJSRT_MACHINE_LICM" in extra or not src.endswith(".hip") else NO_MLICM
    return [HIPCC] + OBJ_FLAGS + dev + defs + list(extra) + ["-c", os.path.join(CSRC, src), "-o", o + ".tmp"]


def _stale():
    objs = [_obj(stem) for stem, _, _, _ in UNITS]
    if not os.path.exists(LIB) or not os.path.exists(_id_file(LIB)):
        return True
    with open(_id_file(LIB)) as f:
        if f.read().strip() != build_id():
            return True  # built from other sources (mtimes do not survive every copy; the id does)
    if not any(os.path.exists(o) for o in objs):
        return False  # a prebuilt library shipped without its objects (the GPU box's snapshot), same id: use it
    return any(_obj_stale(_obj(stem), _deps(src, deps), _cmd(src, defs, [], _obj(stem)))
               for stem, src, defs, deps in UNITS) or _newer(LIB, objs)


def build(force=False, verbose=False, variant=None, defines=(), profiles=None):
    """variant: build _build/libjsrt_<variant>.so with extra -D defines (A/B experiments).  profiles:
    for a variant, the kernel profiles (PF numbers) recompiled with the defines; the other objects are
    the default build's (fast A/B of one scene class).  Concurrent callers (pytest-xdist workers) are
    serialised on a lock file, so a stale library is rebuilt once."""
    os.makedirs(OUT, exist_ok=True)
    import fcntl
    with open(os.path.join(OUT, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return _build_locked(force, verbose, variant, defines, profiles)


def _build_locked(force, verbose, variant, defines, profiles):
    lib = LIB if variant is None else os.path.join(OUT, f"libjsrt_{variant}.so")
    tag = "" if variant is None else f"_{variant}"
    if variant is None and not force and not _stale():
        return LIB
    if variant is not None:
        _build_locked(False, verbose, None, (), None)  # the default objects a partial variant links against
    jobs, objs = [], []
    for stem, src, defs, deps in UNITS:
        mine = variant is not None and (profiles is None or any(stem.startswith(f"render_pf{p}_") for p in profiles))
        o = _obj(stem, tag if mine else "")
        objs.append(o)
        extra = list(defines) if mine else []
        cmd = _cmd(src, defs, extra, o)
        if force or mine or _obj_stale(o, _deps(src, deps), cmd):
            jobs.append((cmd, o, _src_stamp(_deps(src, deps), cmd)))

    def run(job):
        cmd, o, stamp = job
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(o + ".tmp", o)
        if stamp is not None:
            with open(o + ".src", "w") as f:
                f.write(stamp + "\n")

    bid = build_id(defines if variant is not None else ())
    id_src = _write_id_unit(bid, tag)
    id_obj = _obj("build_id", tag)
    jobs.append(([HIPCC] + OBJ_FLAGS + ["-c", id_src, "-o", id_obj + ".tmp"], id_obj, None))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(run, jobs))
    cmd = [HIPCC] + FLAGS + objs + [id_obj, "-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    with open(_id_file(lib), "w") as f:
        f.write(bid + "\n")
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    var = args[args.index("--variant") + 1] if "--variant" in args else None
    prof = [int(x) for x in args[args.index("--profiles") + 1].split(",")] if "--profiles" in args else None
    print(build(force="--force" in args, verbose=True, variant=var, defines=[a for a in args if a.startswith("-D")],
                profiles=prof))
