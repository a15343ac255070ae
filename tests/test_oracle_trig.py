"""The oracle's Math.sin / Math.cos / Math.acos (oracle/js_fdlibm.h, V8's fdlibm restated in C) against
node's own results (tests/golden/trig_v8.npz): bit for bit on 3.3 M arguments, so the checker's scatter
directions are the reference's, not the C library's (which differ in the last bit on ~3 % of them)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trig(x):
    from oracle import pyoracle
    L = pyoracle.lib()
    L.jsrt_oracle_trig.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty((len(x), 3))
    L.jsrt_oracle_trig(x.ctypes.data, y.ctypes.data, len(x))
    return y


def test_oracle_trig_matches_v8():
    sys.path.insert(0, os.path.join(ROOT, "oracle", "refharness"))
    from regen_trig_kats import digest, trig_args
    g = np.load(os.path.join(ROOT, "tests", "golden", "trig_v8.npz"))
    sub = _trig(g["sub_x"])
    for k, name in enumerate(("sin", "cos", "acos")):
        ok = (sub[:, k].view(np.uint64) == g["sub_y"][:, k].view(np.uint64)) | (np.isnan(sub[:, k]) & np.isnan(g["sub_y"][:, k]))
        assert ok.all(), f"{name}: {int((~ok).sum())} differ"
    y = _trig(trig_args(int(g["args_seed"][0])))
    for k, name in enumerate(("sin", "cos", "acos")):
        assert digest(y[:, k]) == str(g[f"sha_{name}"]), name


def test_oracle_atan2_asin_match_v8():
    """The oracle's Math.atan2 / Math.asin (oracle/js_fdlibm.h) against node on 4 M pairs (tests/golden/uv_v8.npz)."""
    from oracle import pyoracle
    sys.path.insert(0, os.path.join(ROOT, "oracle", "refharness"))
    from regen_trig_kats import digest
    from regen_uv_kats import uv_args
    L = pyoracle.lib()
    L.jsrt_oracle_uv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    g = np.load(os.path.join(ROOT, "tests", "golden", "uv_v8.npz"))
    xy = np.ascontiguousarray(uv_args(int(g["args_seed"][0])))
    y = np.empty((len(xy), 2))
    L.jsrt_oracle_uv(xy.ctypes.data, y.ctypes.data, len(xy))
    for k, name in enumerate(("atan2", "asin")):
        assert digest(y[:, k]) == str(g[f"sha_{name}"]), name
