"""The box-union SDF with one square root (device_common.h sdf_minbox), compiled for the host, against the
reference's UnionSDF of BoxSDFs (sdf.js:83-85, 276-279): Math.min of sqrt(|max(q, 0)|^2) + min(max(q), 0)
per box.  The SDF_Menger hole pattern evaluates such a union 7 times per distance (sdf_forms.h)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "sdf_box_host.hip")
OUT = os.path.join(ROOT, "tests", "native", "_build", "libsdf_box_host.so")
HDRS = [os.path.join(ROOT, "jsraytracer_amd", "csrc", h) for h in ("device_common.h", "js_number.h", "sdf_forms.h")]


@pytest.fixture(scope="module")
def lib():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(f) for f in [SRC] + HDRS):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fno-fast-math", "-fPIC", "-shared", SRC, "-o", OUT + f".{os.getpid()}.tmp"], check=True)
        os.replace(OUT + f".{os.getpid()}.tmp", OUT)
    L = ctypes.CDLL(OUT)
    L.box_union.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                            ctypes.c_void_p]
    L.cross_union.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    return L


def _run(L, boxes, pts):
    boxes = np.ascontiguousarray(boxes, np.float64)
    pts = np.ascontiguousarray(pts, np.float32)
    ref, got = np.empty(len(pts)), np.empty(len(pts))
    L.box_union(boxes.ctypes.data, len(boxes), pts.ctypes.data, len(pts), ref.ctypes.data, got.ctypes.data)
    return ref, got


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_minbox_equals_reference_union(lib, n):
    rng = np.random.default_rng(n)
    menger = np.array([[np.inf, 1, 1, 0], [1, np.inf, 1, 0], [1, 1, np.inf, 0], [0.5, 0.25, 2, 0], [1e-3, 3, 0.7, 0]])
    for boxes in (menger[:n], np.c_[np.float32(rng.uniform(0.01, 2, (n, 3))).astype(np.float64), np.zeros(n)]):
        pts = [rng.uniform(-3, 3, (200_000, 3)), rng.uniform(-1.2, 1.2, (200_000, 3)),
               np.round(rng.uniform(-2, 2, (100_000, 3)) * 4) / 4,           # on faces, edges, corners
               np.c_[rng.choice([-1.0, 1.0, 0.5, -0.5, 0.0, -0.0], (50_000, 3))],
               np.array([[np.nan, 0, 0], [0, np.nan, 1], [np.inf, 0, 0], [-np.inf, 1, 1], [0, 0, 0], [-0.0, 0, 0]])]
        ref, got = _run(lib, boxes, np.concatenate(pts))
        same = (ref.view(np.uint64) == got.view(np.uint64)) | (np.isnan(ref) & np.isnan(got))
        assert same.all(), f"{int((~same).sum())} differ"


@pytest.mark.parametrize("h", [1 / 3, 1.0, 0.0, 1e-30])
def test_cross_equals_minbox(lib, h):
    """sdf_cross (the Menger cross: box i infinite along axis i, half size h across) is bit-identical to the
    generic union on points everywhere, on the bars' faces, edges and corners, at +-0, and at non-finite
    coordinates (which it hands to sdf_minbox)."""
    rng = np.random.default_rng(int(h * 1000) + 3)
    boxes = np.full((3, 4), h)
    boxes[:, 3] = 0
    boxes[[0, 1, 2], [0, 1, 2]] = np.inf
    hf = np.float32(h)
    edge = np.array([0.0, -0.0, hf, -hf, np.nextafter(hf, np.float32(1)), np.nextafter(hf, np.float32(0))], np.float32)
    pts = [rng.uniform(-3, 3, (300_000, 3)), rng.uniform(-1.2 * h - 1e-6, 1.2 * h + 1e-6, (300_000, 3)),
           rng.choice(edge, (100_000, 3)),
           np.c_[rng.choice(edge, 100_000), rng.uniform(-2, 2, (100_000, 2))][:, rng.permutation(3)],
           np.array([[np.nan, 0, 0], [0, np.nan, 1], [np.inf, 0, 0], [-np.inf, 1, 1], [0, 0, np.inf], [3e38, 0, 0]])]
    pts = np.ascontiguousarray(np.concatenate(pts), np.float32)
    ref, got = np.empty(len(pts)), np.empty(len(pts))
    lib.cross_union(np.ascontiguousarray(boxes).ctypes.data, pts.ctypes.data, len(pts), ref.ctypes.data, got.ctypes.data)
    same = (ref.view(np.uint64) == got.view(np.uint64)) | (np.isnan(ref) & np.isnan(got))
    assert same.all(), f"{int((~same).sum())} differ, e.g. {pts[~same][:3].tolist()}"
