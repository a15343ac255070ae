"""Builds libjsrt.so in-tree with hipcc for gfx950 (no JIT caches: the .so travels to the GPU box)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
LIB = os.path.join(OUT, "libjsrt.so")
SOURCES = ["render.hip", "capi.cpp", "scene_load.cpp"]
HEADERS = ["device_common.h", "js_number.h", "device_scene.h", "render_kernel.h", "scene_load.h", "sdf_program.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("JSRT_OFFLOAD_ARCH", "gfx950")

# Strict IEEE (the reference's numeric model): no FMA contraction, no fast-math,
# f32 denormals preserved (HIP's default), correctly rounded f32 div/sqrt (HIP's default).
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(HERE, "..", "include", f) for f in ("jsrt.h", "jsrt_scene.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, variant=None, defines=()):
    """variant: build _build/libjsrt_<variant>.so with extra -D defines (A/B experiments)."""
    os.makedirs(OUT, exist_ok=True)
    lib = LIB if variant is None else os.path.join(OUT, f"libjsrt_{variant}.so")
    if variant is None and not force and not _stale():
        return LIB
    cmd = [HIPCC] + FLAGS + list(defines) + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    args = sys.argv[1:]
    var = args[args.index("--variant") + 1] if "--variant" in args else None
    print(build(force="--force" in args, verbose=True, variant=var, defines=[a for a in args if a.startswith("-D")]))
