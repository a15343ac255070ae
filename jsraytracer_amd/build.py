"""Builds libjsrt.so in-tree with hipcc for gfx950 (no JIT caches: the .so travels to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libjsrt.so")
SOURCES = ["render.hip", "capi.cpp", "scene_load.cpp", "mesh_build.cpp"]
HEADERS = ["device_common.h", "js_number.h", "device_scene.h", "render_kernel.h", "scene_load.h", "sdf_program.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("JSRT_OFFLOAD_ARCH", "gfx950")

# Strict IEEE (the reference's numeric model): no FMA contraction, no fast-math,
# f32 denormals preserved (HIP's default), correctly rounded f32 div/sqrt (HIP's default).
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function"]


INCLUDE = os.path.join(HERE, "..", "include")
PUBLIC = ["jsrt.h", "jsrt_scene.h", "jsrt_mesh.h"]
# per-source dependencies (objects are rebuilt only when these change; render.hip dominates build time)
DEPS = {
    "render.hip": HEADERS + ["jsrt.h", "jsrt_scene.h"],
    "capi.cpp": HEADERS + ["jsrt.h", "jsrt_scene.h"],
    "scene_load.cpp": HEADERS + ["jsrt.h", "jsrt_scene.h"],
    "mesh_build.cpp": ["jsrt_mesh.h", "jsrt_scene.h"],
}
OBJ_FLAGS = [f for f in FLAGS if f != "-shared"]


def _path(f):
    return os.path.join(INCLUDE, f) if f in PUBLIC else os.path.join(CSRC, f)


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _obj(src, tag, defines):
    return os.path.join(OUT, f"{os.path.splitext(src)[0]}{tag}.o")


def _stale():
    return any(_newer(_obj(s, "", ()), [os.path.join(CSRC, s)] + [_path(d) for d in DEPS[s]]) for s in SOURCES) or \
        any(_newer(LIB, [_obj(s, "", ())]) for s in SOURCES)


def build(force=False, verbose=False, variant=None, defines=()):
    """variant: build _build/libjsrt_<variant>.so with extra -D defines (A/B experiments)."""
    os.makedirs(OUT, exist_ok=True)
    lib = LIB if variant is None else os.path.join(OUT, f"libjsrt_{variant}.so")
    tag = "" if variant is None else f"_{variant}"
    if variant is None and not force and not _stale():
        return LIB
    objs = []
    for s in SOURCES:  # one object per source: an edit recompiles only what depends on it
        o = _obj(s, tag, defines)
        deps = [os.path.join(CSRC, s)] + [_path(d) for d in DEPS[s]]
        if force or variant is not None or _newer(o, deps):
            cmd = [HIPCC] + OBJ_FLAGS + list(defines) + ["-c", os.path.join(CSRC, s), "-o", o + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            os.replace(o + ".tmp", o)
        objs.append(o)
    cmd = [HIPCC] + FLAGS + objs + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    var = args[args.index("--variant") + 1] if "--variant" in args else None
    print(build(force="--force" in args, verbose=True, variant=var, defines=[a for a in args if a.startswith("-D")]))
