"""The shadow cast's AABB any-hit filter (device_common.h box_any_f32), compiled for the host, against the
exact AABB.intersect (geometry.js:173-179, aabb_intersect: six correctly rounded f64 divisions) and World.cast's
acceptance minD < t < maxD: every decision it takes is the exact outcome, its distance estimate lies inside
(minD, maxD), and "too close to call" (the exact test runs) stays rare.  Cases: random boxes and rays, segments
ending on a face (t ~ 1), starting on a face (t ~ 0 and ~ minD), axis-parallel and near-1e-7 direction
components (the reference's per-axis skip), and non-finite inputs."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "box_any_host.hip")
OUT = os.path.join(ROOT, "tests", "native", "_build", "libbox_any_host.so")
HDRS = [os.path.join(ROOT, "jsraytracer_amd", "csrc", h) for h in ("device_common.h", "js_number.h", "fdlibm.h")]


@pytest.fixture(scope="module")
def lib():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(os.path.getmtime(f) for f in [SRC] + HDRS):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fno-fast-math", "-fPIC", "-shared", SRC, "-o", OUT + f".{os.getpid()}.tmp"], check=True)
        os.replace(OUT + f".{os.getpid()}.tmp", OUT)
    L = ctypes.CDLL(OUT)
    L.box_any.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_double, ctypes.c_double,
                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def _run(L, boxes, rays, minD, maxD):
    boxes = np.ascontiguousarray(boxes, np.float32)
    rays = np.ascontiguousarray(rays, np.float32)
    n = len(boxes)
    ex, dec, tf = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n)
    L.box_any(boxes.ctypes.data, rays.ctypes.data, n, minD, maxD, ex.ctypes.data, dec.ctypes.data, tf.ctypes.data)
    return ex, dec, tf


def _cases(seed, n=400_000):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-2, 2, (n, 3))
    h = rng.uniform(0.01, 2, (n, 3))
    o = rng.uniform(-6, 6, (n, 3))
    d = rng.normal(size=(n, 3)) * rng.uniform(0.1, 10, (n, 1))
    kind = rng.integers(0, 6, n)
    # a point on a random face of the box
    ax = rng.integers(0, 3, n)
    q = c + h * rng.uniform(-1, 1, (n, 3))
    sgn = rng.choice([-1.0, 1.0], n)
    q[np.arange(n), ax] = c[np.arange(n), ax] + sgn * h[np.arange(n), ax]
    q32 = q.astype(np.float32).astype(np.float64)
    # 1: segments ending on the face (t ~ 1)
    m = kind == 1
    d[m] = q32[m] - o[m]
    # 2: segments starting on the face (t ~ 0) or 1e-4 along the ray from it (t ~ minD)
    m = kind == 2
    o[m] = q32[m]
    m3 = kind == 3
    o[m3] = q32[m3] - 1e-4 * d[m3]
    # 4: axis-parallel / near-1e-7 components (the reference's |d_i| > 1e-7 skip)
    m = kind == 4
    comp = rng.integers(0, 3, n)
    vals = np.array([0.0, -0.0, 1e-7, -1e-7, np.nextafter(np.float32(1e-7), np.float32(1)),
                     np.nextafter(np.float32(1e-7), np.float32(0)), 1e-8, 2e-7])
    d[m, comp[m]] = rng.choice(vals, m.sum())
    # 5: rays through a box edge / corner region (grazing)
    m = kind == 5
    corner = c + h * rng.choice([-1.0, 1.0], (n, 3))
    d[m] = corner[m] - o[m] + rng.normal(scale=1e-6, size=(m.sum(), 3))
    boxes = np.concatenate([c, h], 1).astype(np.float32)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    return boxes, rays, kind


@pytest.mark.parametrize("maxD", [1.0, 5.0, np.inf])
@pytest.mark.parametrize("seed", [1, 2])
def test_box_any_decisions_are_exact(lib, seed, maxD):
    boxes, rays, kind = _cases(seed)
    minD = 1e-4
    ex, dec, tf = _run(lib, boxes, rays, minD, maxD)
    taken = dec >= 0
    assert (dec[taken] == ex[taken]).all(), np.flatnonzero(taken & (dec != ex))[:8]
    acc = dec == 1
    assert (tf[acc] > minD).all() and (tf[acc] < maxD).all()
    assert ex.sum() > 1000 and (ex == 0).sum() > 1000  # both outcomes exercised
    # "too close to call" is for comparisons within 2^-21 of a bound: the segments built to end on a face
    # (t = 1 up to the f32 rounding of the endpoint) and the rays aimed at a corner (tmin ~ tmax) defer often,
    # the ones starting 1e-4 along the ray from a face (t ~ minD) sometimes, the others almost never
    assert (dec[(kind == 1) | (kind == 5)] == -1).mean() > 0.1
    assert (dec[kind == 3] == -1).mean() < 0.05
    assert (dec[(kind == 0) | (kind == 2) | (kind == 4)] == -1).mean() < 1e-3


def test_box_any_random_rays_rarely_defer(lib):
    rng = np.random.default_rng(7)
    n = 400_000
    boxes = np.concatenate([rng.uniform(-2, 2, (n, 3)), rng.uniform(0.01, 2, (n, 3))], 1)
    rays = np.concatenate([rng.uniform(-6, 6, (n, 3)), rng.normal(size=(n, 3)) * 5], 1)
    ex, dec, _ = _run(lib, boxes, rays, 1e-4, 1.0)
    taken = dec >= 0
    assert (dec[taken] == ex[taken]).all()
    assert (dec == -1).mean() < 1e-4


def test_box_any_non_finite(lib):
    rows = []
    for o, d in [((np.nan, 0, 0), (1, 0, 0)), ((0, 0, 0), (np.nan, 1, 0)), ((np.inf, 0, 0), (-1, 0, 0)),
                 ((-5, 0, 0), (np.inf, 0, 0)), ((0, 0, 0), (0, 0, 0)), ((-5, 0.5, 0.5), (1e30, 0, 0)),
                 ((-5, 0, 0), (1e-30, 0, 0))]:
        rows.append((o, d))
    boxes = np.tile(np.array([0, 0, 0, 1, 1, 1], np.float32), (len(rows), 1))
    rays = np.array([list(o) + list(d) for o, d in rows], np.float32)
    for maxD in (1.0, np.inf):
        ex, dec, _ = _run(lib, boxes, rays, 1e-4, maxD)
        taken = dec >= 0
        assert (dec[taken] == ex[taken]).all(), (dec, ex)


def _planar_cases(seed, n=300_000):
    """Random similarity transforms (rotation x scale + translation) of the unit Square / Circle / Plane, rays
    aimed at random points of the primitive's plane inside and around its bounds (near the edges too), with
    segment ends before, at and beyond the plane."""
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.normal(size=(n, 3, 3)))
    scale = rng.uniform(0.2, 10, (n, 1, 1))
    M = q * scale  # world = M @ local + c
    c = rng.uniform(-5, 5, (n, 3))
    Minv = np.linalg.inv(M)
    inv = np.concatenate([Minv, (-Minv @ c[:, :, None])], 2)  # rows 0..2 of the inverse transform
    kinds = rng.choice([1, 2, 3], n)  # JSRT_GEOM_PLANE / SQUARE / CIRCLE (checked below)
    # a local point on the plane: inside, near the edge (|x| ~ 0.5 or r ~ 1), or outside
    loc = rng.uniform(-1.2, 1.2, (n, 3))
    edge = rng.random(n) < 0.3
    loc[edge, 0] = np.where(rng.random(edge.sum()) < 0.5, 0.5, -0.5) + rng.normal(scale=1e-6, size=edge.sum())
    loc[:, 2] = 0
    target = (M @ loc[:, :, None])[:, :, 0] + c
    o = target + rng.normal(size=(n, 3)) * rng.uniform(0.1, 20, (n, 1))
    frac = rng.choice([0.3, 0.9, 1.0, 1.1, 3.0, 1e-4, 2e-4], n)
    d = (target - o) / frac[:, None]
    rays = np.concatenate([o, d], 1).astype(np.float32)
    # the constructed boundary cases: the plane at t = 1 or t = minD, a hit point within 1e-6 of an edge
    boundary = edge | (frac == 1.0) | (frac == 1e-4)
    return np.ascontiguousarray(inv.reshape(n, 12)), kinds.astype(np.int32), rays, boundary


@pytest.mark.parametrize("maxD", [1.0, np.inf])
@pytest.mark.parametrize("seed", [3, 4])
def test_planar_any_decisions_are_exact(lib, seed, maxD):
    import ctypes as C
    L = lib
    L.planar_any.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_double, C.c_double, C.c_void_p,
                             C.c_void_p, C.c_void_p]
    inv, kinds, rays, boundary = _planar_cases(seed)
    n = len(kinds)
    ex, dec, tf = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n)
    L.planar_any(inv.ctypes.data, kinds.ctypes.data, rays.ctypes.data, n, 1e-4, maxD, ex.ctypes.data,
                 dec.ctypes.data, tf.ctypes.data)
    taken = dec >= 0
    bad = np.flatnonzero(taken & (dec != ex))
    assert len(bad) == 0, (bad[:8], kinds[bad[:8]])
    acc = dec == 1
    assert (tf[acc] > 1e-4).all() and (tf[acc] < maxD).all()
    for k in (1, 2, 3):
        assert ex[kinds == k].sum() > 1000 and (ex[kinds == k] == 0).sum() > 1000
    assert (dec[~boundary] == -1).mean() < 1e-3, (dec[~boundary] == -1).mean()


def _sphere_cases(seed, n=400_000):
    """Local rays against the unit sphere: random, aimed at surface points (segments ending on, before and
    beyond the surface), starting on the surface (t ~ 0) or at minD from it, and tangent rays."""
    rng = np.random.default_rng(seed)
    kind = rng.integers(0, 5, n)
    o = rng.normal(size=(n, 3)) * rng.uniform(0.5, 8, (n, 1))
    d = rng.normal(size=(n, 3)) * rng.uniform(0.1, 10, (n, 1))
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)  # a surface point
    frac = rng.choice([0.5, 0.999, 1.0, 1.001, 2.0], n)
    m = kind == 1
    d[m] = (u[m] - o[m]) / frac[m, None]
    m = kind == 2
    o[m] = u[m]
    m = kind == 3
    o[m] = u[m] - 1e-4 * d[m]
    m = kind == 4  # tangent: d perpendicular to the radius at u, o = u - s d
    t = rng.normal(size=(n, 3))
    t -= (t * u).sum(1, keepdims=True) * u
    d[m] = t[m]
    o[m] = u[m] - rng.uniform(0.1, 3, (m.sum(), 1)) * t[m] + rng.normal(scale=1e-7, size=(m.sum(), 3))
    rays = np.concatenate([o, d], 1).astype(np.float32)
    boundary = ((kind == 1) & (frac == 1.0)) | (kind == 3) | (kind == 4)
    return rays, boundary


@pytest.mark.parametrize("maxD", [1.0, np.inf])
@pytest.mark.parametrize("seed", [5, 6])
def test_sphere_any_decisions_are_exact(lib, seed, maxD):
    import ctypes as C
    L = lib
    L.sphere_any.argtypes = [C.c_void_p, C.c_long, C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]
    rays, boundary = _sphere_cases(seed)
    n = len(rays)
    ex, dec, tf = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n)
    L.sphere_any(rays.ctypes.data, n, 1e-4, maxD, ex.ctypes.data, dec.ctypes.data, tf.ctypes.data)
    taken = dec >= 0
    bad = np.flatnonzero(taken & (dec != ex))
    assert len(bad) == 0, bad[:8]
    acc = dec == 1
    assert (tf[acc] > 1e-4).all() and (tf[acc] < maxD).all()
    assert ex.sum() > 1000 and (ex == 0).sum() > 1000
    assert (dec[~boundary] == -1).mean() < 1e-3, (dec[~boundary] == -1).mean()


def _tri_cases(seed, n=400_000):
    """Random triangles (mesh-like sizes and slivers) and rays aimed at barycentric points inside, on the
    edges and vertices, and outside, with segments ending before, at and beyond the triangle."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-3, 3, (n, 1, 3))
    size = np.exp(rng.uniform(np.log(1e-3), np.log(2), (n, 1, 1)))
    v = c + rng.normal(size=(n, 3, 3)) * size
    sliver = rng.random(n) < 0.1
    v[sliver, 2] = v[sliver, 0] + (v[sliver, 1] - v[sliver, 0]) * rng.uniform(0, 1, (sliver.sum(), 1)) + \
        rng.normal(scale=1e-4, size=(sliver.sum(), 3)) * size[sliver, 0]
    bary = rng.dirichlet([1, 1, 1], n)
    kind = rng.integers(0, 4, n)
    m = kind == 1  # on an edge
    e = rng.integers(0, 3, n)
    bary[m, e[m]] = 0
    bary[m] /= bary[m].sum(1, keepdims=True)
    m = kind == 2  # outside
    bary[m] = bary[m] * 2 - 0.3
    m = kind == 3  # a vertex
    bary[m] = np.eye(3)[e[m]]
    target = (bary[:, :, None] * v).sum(1)
    o = target + rng.normal(size=(n, 3)) * rng.uniform(0.1, 10, (n, 1))
    frac = rng.choice([0.3, 0.9, 1.0, 1.1, 3.0, 1e-4], n)
    d = (target - o) / frac[:, None]
    verts = v.reshape(n, 9).astype(np.float32)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    boundary = (kind == 1) | (kind == 3) | (frac == 1.0) | (frac == 1e-4) | sliver
    return verts, rays, boundary


@pytest.mark.parametrize("maxD", [1.0, np.inf])
@pytest.mark.parametrize("seed", [8, 9])
def test_tri_any_decisions_are_exact(lib, seed, maxD):
    import ctypes as C
    L = lib
    L.tri_any.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_double, C.c_double, C.c_void_p, C.c_void_p,
                          C.c_void_p]
    verts, rays, boundary = _tri_cases(seed)
    n = len(rays)
    ex, dec, tf = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n)
    L.tri_any(verts.ctypes.data, rays.ctypes.data, n, 1e-4, maxD, ex.ctypes.data, dec.ctypes.data, tf.ctypes.data)
    taken = dec >= 0
    bad = np.flatnonzero(taken & (dec != ex))
    assert len(bad) == 0, bad[:8]
    acc = dec == 1
    assert (tf[acc] > 1e-4).all() and (tf[acc] < maxD).all()
    assert ex.sum() > 1000 and (ex == 0).sum() > 1000
    # (rays up to 30 units long against triangles down to 1e-3: the hit point bound is relative to the ray)
    assert (dec[~boundary] == -1).mean() < 0.1, (dec[~boundary] == -1).mean()


def test_f32_stable_bits(lib):
    """spherePick's stability test (device_common.h f32_stable_bits): a value it calls stable rounds to the same
    f32 as every value within 2^-44 of it (checked at the interval's ends and at random points of it), and it
    calls stable nearly every value the float rounding would (the exact interval test)."""
    import ctypes as C
    lib.stable_bits.argtypes = [C.c_void_p, C.c_long, C.c_void_p]
    rng = np.random.default_rng(11)
    n = 2_000_000
    d = rng.uniform(-1, 1, n) * np.exp2(-rng.integers(0, 24, n).astype(np.float64))
    mid = rng.random(n) < 0.3  # put some within a few 2^-44 of an f32 midpoint
    f = d[mid].astype(np.float32).astype(np.float64)
    up = np.nextafter(d[mid].astype(np.float32), np.float32(np.inf)).astype(np.float64)
    d[mid] = (f + up) / 2 + rng.normal(scale=2.0 ** -44, size=mid.sum()) * rng.choice([0.5, 1, 2, 8], mid.sum())
    out = np.empty(n, np.int32)
    lib.stable_bits(np.ascontiguousarray(d).ctypes.data, n, out.ctypes.data)
    e = 2.0 ** -44
    ref = (d - e).astype(np.float32) == (d + e).astype(np.float32)
    st = out == 1
    for delta in (-e, e, rng.uniform(-e, e, n)):
        assert ((d + delta).astype(np.float32)[st] == d.astype(np.float32)[st]).all()
    assert not (st & ~ref).any()
    assert (ref & ~st).mean() < 1e-4
    assert st.sum() > n // 2


def _closest_lims(rng, tref, n):
    """World.cast's closest-hit bound lim = min(maxD, the closest hit so far): random, +Infinity, and the exact
    distance itself and its neighbours (a hit tied with the current closest one is not taken: t < lim)."""
    lim = np.where(rng.random(n) < 0.3, np.inf, rng.uniform(0, 20, n))
    fin = np.isfinite(tref) & (tref > 0)
    pick = rng.integers(0, 5, n)
    near = np.select([pick == 0, pick == 1, pick == 2, pick == 3],
                     [tref, np.nextafter(tref, np.inf), np.nextafter(tref, -np.inf), tref * (1 + 1e-7)], tref * 2)
    return np.where(fin & (rng.random(n) < 0.5), near, lim)


def _check_closest(ex, tref, dec, tf, boundary, defer_max):
    taken = dec >= 0
    bad = np.flatnonzero(taken & (dec != ex))
    assert len(bad) == 0, bad[:8]
    acc = dec == 1
    # an accepted distance is the reference's, bit for bit (the filter's one division is the exact one's)
    assert np.array_equal(tf[acc].view(np.uint64), tref[acc].view(np.uint64)), np.flatnonzero(acc & (tf != tref))[:8]
    assert ex.sum() > 1000 and (ex == 0).sum() > 1000
    assert acc[~boundary].sum() > 0.99 * ex[~boundary].sum(), (acc[~boundary].sum(), ex[~boundary].sum())
    assert (dec[~boundary] == -1).mean() < defer_max, (dec[~boundary] == -1).mean()


@pytest.mark.parametrize("maxD", [1.0, np.inf])
@pytest.mark.parametrize("seed", [1, 2])
def test_box_closest_decisions_and_distances_are_exact(lib, seed, maxD):
    """box_closest_f32 (the closest-hit cast's AABB filter): its decisions are the exact acceptance minD < t < lim
    and an accepted distance is AABB.intersect's own, bit for bit."""
    import ctypes as C
    lib.box_closest.argtypes = [C.c_void_p] * 3 + [C.c_long, C.c_double, C.c_double] + [C.c_void_p] * 4
    boxes, rays, kind = _cases(seed)
    n = len(boxes)
    minD = 1e-4
    # the exact distances first (lim = +inf), then lims placed around them
    ex, tref, dec, tf = np.empty(n, np.int32), np.empty(n), np.empty(n, np.int32), np.empty(n)
    lims = np.full(n, np.inf)
    args = lambda lm: (boxes.ctypes.data, rays.ctypes.data, lm.ctypes.data, n, minD, maxD, ex.ctypes.data,
                       tref.ctypes.data, dec.ctypes.data, tf.ctypes.data)
    lib.box_closest(*args(lims))
    lims = _closest_lims(np.random.default_rng(seed + 100), tref.copy(), n)
    lib.box_closest(*args(lims))
    tie = (lims == tref) | (lims == np.nextafter(tref, np.inf)) | (lims == np.nextafter(tref, -np.inf)) | (lims == tref * (1 + 1e-7))
    _check_closest(ex, tref, dec, tf, (kind == 1) | (kind == 3) | (kind == 5) | tie, 1e-3)


@pytest.mark.parametrize("maxD", [1.0, np.inf])
@pytest.mark.parametrize("seed", [5, 6])
def test_sphere_closest_decisions_and_distances_are_exact(lib, seed, maxD):
    """sphere_closest_f32 (the closest-hit cast's Sphere filter), as test_box_closest for sphere_static."""
    import ctypes as C
    lib.sphere_closest.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_double, C.c_double] + [C.c_void_p] * 4
    rays, boundary = _sphere_cases(seed)
    n = len(rays)
    ex, tref, dec, tf = np.empty(n, np.int32), np.empty(n), np.empty(n, np.int32), np.empty(n)
    args = lambda lm: (rays.ctypes.data, lm.ctypes.data, n, 1e-4, maxD, ex.ctypes.data, tref.ctypes.data,
                       dec.ctypes.data, tf.ctypes.data)
    lims = np.full(n, np.inf)
    lib.sphere_closest(*args(lims))
    lims = _closest_lims(np.random.default_rng(seed + 100), tref.copy(), n)
    lib.sphere_closest(*args(lims))
    tie = (lims == tref) | (lims == np.nextafter(tref, np.inf)) | (lims == np.nextafter(tref, -np.inf)) | (lims == tref * (1 + 1e-7))
    _check_closest(ex, tref, dec, tf, boundary | tie, 1e-3)
