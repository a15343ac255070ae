"""The device's Math.sin / Math.cos / Math.acos (jsraytracer_amd/csrc/fdlibm.h: V8's fdlibm algorithms),
compiled for the host, against node's own results (tests/golden/trig_v8.npz, oracle/refharness/
regen_trig_kats.py): bit for bit on 3.3 M arguments -- the reference's angles 2 pi r and acos(2 r - 1),
wider ranges, the neighbours of multiples of pi/4 and pi/2, tiny and special values."""
import ctypes
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "fdlibm_host.hip")
OUT = os.path.join(ROOT, "tests", "native", "_build", "libfdlibm_host.so")
HDR = os.path.join(ROOT, "jsraytracer_amd", "csrc", "fdlibm.h")  # (rebuilt when it changes)


@pytest.fixture(scope="module")
def lib():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fno-fast-math", "-fPIC", "-shared", SRC, "-o", OUT + f".{os.getpid()}.tmp"], check=True)
        os.replace(OUT + f".{os.getpid()}.tmp", OUT)
    L = ctypes.CDLL(OUT)
    L.trig_n.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    return L


def _trig(L, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty((len(x), 3))
    L.trig_n(x.ctypes.data, y.ctypes.data, len(x))
    return y


def _same(a, b):
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def test_fdlibm_matches_v8_subsample(lib):
    g = np.load(os.path.join(ROOT, "tests", "golden", "trig_v8.npz"))
    y = _trig(lib, g["sub_x"])
    for k, name in enumerate(("sin", "cos", "acos")):
        ok = _same(y[:, k], g["sub_y"][:, k])
        assert ok.all(), f"{name}: {int((~ok).sum())} differ, e.g. x = {g['sub_x'][~ok][:4].tolist()}"


def test_fdlibm_matches_v8_everywhere(lib):
    sys.path.insert(0, os.path.join(ROOT, "oracle", "refharness"))
    from regen_trig_kats import digest, trig_args
    g = np.load(os.path.join(ROOT, "tests", "golden", "trig_v8.npz"))
    x = trig_args(int(g["args_seed"][0]))
    assert len(x) == int(g["n"][0])
    y = _trig(lib, x)
    for k, name in enumerate(("sin", "cos", "acos")):
        assert digest(y[:, k]) == str(g[f"sha_{name}"]), name


def test_reduction_table_computed(lib):
    """fdlibm.h computes rem_pio2's npio2_hw table (high words of n pi/2) instead of indexing it per lane."""
    assert lib.npio2_hw_ok() == 1


def _uv(L, xy):
    import ctypes as C
    L.uv_n.argtypes = [C.c_void_p, C.c_void_p, C.c_long]
    xy = np.ascontiguousarray(xy, dtype=np.float64)
    y = np.empty((len(xy), 2))
    L.uv_n(xy.ctypes.data, y.ctypes.data, len(xy))
    return y


def test_fdlibm_atan2_asin_match_v8(lib):
    """Math.atan2 / Math.asin (fdlibm.h) against node on 4 M pairs (tests/golden/uv_v8.npz): f32 unit-vector
    components as cartesianToSpherical takes them, cylinder points, wide pairs, signed zeros, infinities, NaN."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "refharness"))
    from regen_trig_kats import digest
    from regen_uv_kats import uv_args
    g = np.load(os.path.join(ROOT, "tests", "golden", "uv_v8.npz"))
    sub = _uv(lib, g["sub_xy"])
    for k, name in enumerate(("atan2", "asin")):
        ok = _same(sub[:, k], g["sub_y"][:, k])
        assert ok.all(), f"{name}: {int((~ok).sum())} differ, e.g. {g['sub_xy'][~ok][:4].tolist()}"
    xy = uv_args(int(g["args_seed"][0]))
    assert len(xy) == int(g["n"][0])
    y = _uv(lib, xy)
    for k, name in enumerate(("atan2", "asin")):
        assert digest(y[:, k]) == str(g[f"sha_{name}"]), name
