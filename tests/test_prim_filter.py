"""The f32 pre-tests of the analytic primitives (jsraytracer_amd/csrc/prim_filter.h), compiled for the host.

world_cast asks every top-level Plane / Square / Circle / UnitBox / Sphere first for an f32 decision with
error bounds (accepted / rejected / too close to call) and runs the exact f64 intersection
(geometry.js:173-179, 246-248, 287-291, 310-314, 429-442 restated in device_common.h) only for the last.
Parity rests on a decisive answer never disagreeing with the exact one.  This checks that on millions of
rays built to sit on the decision boundaries: origins on the surface (the self-intersection every shadow
ray makes), grazing rays at edges and silhouettes, axis-parallel directions (the slab's |d| <= 1e-7 rule),
distances next to minD and next to the caller's limit, and transforms like the reference scenes' (scale,
rotation, translation; Mat4 inverse in f64).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "prim_filter_host.hip")
OUT = os.path.join(ROOT, "tests", "native", "_build", "libprim_filter_host.so")
CSRC = os.path.join(ROOT, "jsraytracer_amd", "csrc")
DEPS = [SRC] + [os.path.join(CSRC, f) for f in ("prim_filter.h", "device_common.h", "device_scene.h")]



def _geom_ids():
    import re
    txt = open(os.path.join(ROOT, "include", "jsrt_scene.h")).read()
    ids = {}
    for name in ("PLANE", "SQUARE", "CIRCLE", "AABB", "SPHERE"):
        m = re.search(r"JSRT_GEOM_%s\s*=\s*(\d+)" % name, txt)
        ids[name] = int(m.group(1))
    return ids


@pytest.fixture(scope="module")
def lib():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(d) for d in DEPS):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fno-fast-math", "-fPIC", "-shared", SRC, "-o", OUT + ".tmp"], check=True)
        os.replace(OUT + ".tmp", OUT)
    L = ctypes.CDLL(OUT)
    L.filt_eval.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_long] + [ctypes.c_void_p] * 3
    return L


def _rot(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    x, y, z = axis
    c, s = np.cos(ang), np.sin(ang)
    C = 1 - c
    return np.array([[x * x * C + c, x * y * C - z * s, x * z * C + y * s, 0],
                     [y * x * C + z * s, y * y * C + c, y * z * C - x * s, 0],
                     [z * x * C - y * s, z * y * C + x * s, z * z * C + c, 0], [0, 0, 0, 1]])


def _transforms(rng, n):
    """Forward matrices like the scenes' Mat4.translation(t).times(scale(s)).times(rotation(a, v))."""
    out = [np.diag([10.0, 10.0, 1.0, 1.0]) @ np.eye(4), np.eye(4)]  # cornell wall-like, identity
    out[0][:3, 3] = [0, 5, -5]
    for _ in range(n):
        T = np.eye(4)
        T[:3, 3] = rng.uniform(-6, 6, 3)
        S = np.diag(list(rng.choice([0.5, 1, 2, 4, 10], 3) * rng.uniform(0.8, 1.25, 3)) + [1.0])
        if rng.random() < 0.3:
            S = np.diag([S[0, 0]] * 3 + [1.0])
        R = _rot(rng.normal(size=3), rng.uniform(-np.pi, np.pi)) if rng.random() < 0.7 else \
            _rot(np.eye(3)[rng.integers(3)], rng.choice([np.pi / 2, -np.pi / 2, np.pi / 4, np.pi]))
        out.append(T @ S @ R)
    return out


def _surface_points(rng, kind, ids, n):
    """Local points on (or next to) the primitive's surface and its edges."""
    if kind in (ids["PLANE"], ids["SQUARE"], ids["CIRCLE"]):
        p = np.zeros((n, 3))
        if kind == ids["CIRCLE"]:
            a, r = rng.uniform(0, 2 * np.pi, n), np.sqrt(rng.uniform(0, 1.1, n))
            r[: n // 3] = 1.0 + rng.normal(0, 1e-6, n // 3)  # rim
            p[:, 0], p[:, 1] = r * np.cos(a), r * np.sin(a)
        else:
            p[:, :2] = rng.uniform(-0.6, 0.6, (n, 2))
            e = rng.integers(0, 2, n // 3)
            p[np.arange(n // 3), e] = rng.choice([-0.5, 0.5], n // 3) * (1 + rng.normal(0, 1e-6, n // 3))  # edges
        return p
    if kind == ids["SPHERE"]:
        v = rng.normal(size=(n, 3))
        return v / np.linalg.norm(v, axis=1, keepdims=True)
    # unit box [-1, 1]^3: a face point, some on edges / corners
    p = rng.uniform(-1, 1, (n, 3))
    ax = rng.integers(0, 3, n)
    p[np.arange(n), ax] = rng.choice([-1.0, 1.0], n)
    m = n // 4
    ax2 = (ax[:m] + 1) % 3
    p[np.arange(m), ax2] = rng.choice([-1.0, 1.0], m)
    return p


def _rays(rng, kind, ids, M, n):
    """World-space rays (f32 o, d) and (minD, maxD, lim) from several boundary-seeking families."""
    Minv = np.linalg.inv(M)
    fam = []
    # 1. origin on the surface (shadow rays and bounces leave from hit points), random directions
    s = _surface_points(rng, kind, ids, n)
    o = (M[:3, :3] @ s.T).T + M[:3, 3]
    d = rng.normal(size=(n, 3))
    fam.append((o, d))
    # 2. shadow-like segments: origin anywhere, towards a surface point (edges included), t in (1e-4, 1)
    o2 = rng.uniform(-12, 12, (n, 3))
    tgt = (M[:3, :3] @ _surface_points(rng, kind, ids, n).T).T + M[:3, 3]
    fam.append((o2, (tgt - o2) * rng.choice([0.999, 1.0, 1.0001, 0.5, 2.0], (n, 1))))
    # 3. axis-parallel and near-parallel directions (slab skip rule, planes seen edge-on)
    d3 = rng.normal(size=(n, 3))
    k = rng.integers(0, 3, n)
    d3[np.arange(n), k] = rng.choice([0.0, 1e-7, -1e-7, 1.0000001e-7, 9.99e-8, 1e-9], n)
    local_d = (Minv[:3, :3] @ rng.normal(size=(n, 3)).T).T
    local_d[np.arange(n), k] = 0.0
    d3[: n // 2] = (M[:3, :3] @ local_d[: n // 2].T).T
    fam.append((rng.uniform(-12, 12, (n, 3)), d3))
    # 4. random rays from far away, through the object's neighbourhood
    o4 = rng.normal(size=(n, 3)) * 20
    fam.append((o4, (M[:3, 3] + rng.normal(size=(n, 3)) * 3) - o4))
    rays, lims = [], []
    for o, d in fam:
        o = o.astype(np.float32)
        d = d.astype(np.float32)
        m = len(o)
        mode = rng.integers(0, 3, m)
        lim = np.full((m, 3), [1e-4, np.inf, np.inf])
        lim[mode == 1] = [1e-4, 1.0, 1.0]  # shadow cast
        lim[mode == 2, 0] = 0.0  # camera ray
        sel = mode == 2
        lim[sel, 2] = rng.uniform(0.1, 40, sel.sum())  # a closer hit already found
        rays.append(np.concatenate([o, d], 1))
        lims.append(lim)
    return np.concatenate(rays).astype(np.float32), np.concatenate(lims)


def _eval(lib, kind, inv12, rays, lims):
    n = len(rays)
    exact, filt, t = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.float64)
    c = np.zeros(3, np.float32)
    h = np.ones(3, np.float32)
    inv12 = np.ascontiguousarray(inv12, np.float64)
    rays = np.ascontiguousarray(rays, np.float32)
    lims = np.ascontiguousarray(lims, np.float64)
    lib.filt_eval(kind, inv12.ctypes.data, c.ctypes.data, h.ctypes.data, rays.ctypes.data, lims.ctypes.data, n,
                  exact.ctypes.data, filt.ctypes.data, t.ctypes.data)
    return exact, filt, t


def _tie_lims(t, lims, rng):
    """Second pass: minD or the caller's limit moved next to the exact distance (ties at the bounds)."""
    L = lims.copy()
    ok = np.isfinite(t) & (t > 0)
    eps = rng.choice([-1e-6, -1e-9, -1e-15, 0.0, 1e-15, 1e-9, 1e-6], len(t))
    which = rng.integers(0, 2, len(t))
    sel = ok & (which == 0)
    L[sel, 2] = t[sel] * (1 + eps[sel])  # lim next to t
    L[sel, 1] = np.maximum(L[sel, 1], L[sel, 2])
    sel = ok & (which == 1)
    L[sel, 0] = t[sel] * (1 + eps[sel])  # minD next to t
    L[sel, 1] = np.inf
    L[sel, 2] = np.inf
    return L


@pytest.mark.parametrize("name", ["PLANE", "SQUARE", "CIRCLE", "AABB", "SPHERE"])
def test_filter_never_contradicts_exact(lib, name):
    ids = _geom_ids()
    kind = ids[name]
    rng = np.random.default_rng(1234 + kind)
    n = 6000
    fall = {"surface": [0, 0], "random": [0, 0]}  # exact fallbacks / decisions of the realistic families
    for M in _transforms(rng, 100):
        inv12 = np.linalg.inv(M)[:3, :].reshape(-1)
        rays, lims = _rays(rng, kind, ids, M, n)
        exact, filt, t = _eval(lib, kind, inv12, rays, lims)
        for k, L in enumerate((lims, _tie_lims(t, lims, rng))):
            exact, filt, _ = _eval(lib, kind, inv12, rays, L)
            wrong = (filt >= 0) & (filt != exact)
            assert not wrong.any(), (f"{name}: {int(wrong.sum())} decisive filter answers contradict the exact test, "
                                     f"e.g. ray {rays[wrong][0].tolist()} lims {L[wrong][0].tolist()} "
                                     f"exact {exact[wrong][0]} filter {filt[wrong][0]}")
            if k == 0:
                fam = np.arange(len(filt)) // n
                for key, sel in (("surface", (fam == 0) & (L[:, 0] > 0)), ("random", fam == 3)):
                    fall[key][0] += int((filt[sel] < 0).sum())
                    fall[key][1] += int(sel.sum())
    # the filter must decide nearly every realistic case (hit points leaving a surface, rays through
    # the scene), or it saves nothing; the boundary-seeking families fall back by design
    for key, (x, m) in fall.items():
        assert x / m < 0.10, f"{name}: {x / m:.2%} of the {key} rays fell back to the exact test"


def test_filter_edge_rays(lib):
    """Hand-picked degenerate rays: zero direction components, origins exactly on faces, NaN / inf."""
    ids = _geom_ids()
    inv = np.eye(4)[:3].reshape(-1)
    rays = np.array([[0, 0, 0, 0, 0, 1], [0, 0, 0, 0, 0, 0], [0.5, 0.5, 0, 1, 0, 0], [1, 0, 0, 1, 0, 0],
                     [1, 1, 1, -1, -1, -1], [0, 0, 5, 0, 0, -1], [0, 0, 5, 1e-8, 0, -1], [np.nan, 0, 0, 0, 0, 1],
                     [np.inf, 0, 0, -1, 0, 0], [2, 0, 0, -1, 0, 0], [0, 0, 1e-30, 0, 0, -1e-30]], np.float32)
    for kind in ids.values():
        for lim in ([1e-4, 1.0, 1.0], [0.0, np.inf, np.inf], [1e-4, np.inf, 4.0]):
            lims = np.tile(lim, (len(rays), 1))
            exact, filt, _ = _eval(lib, kind, inv, rays, lims)
            assert not ((filt >= 0) & (filt != exact)).any(), (kind, lim, exact.tolist(), filt.tolist())
