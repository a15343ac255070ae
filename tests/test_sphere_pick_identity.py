"""The phi estimates of the device's spherePick filter (jsraytracer_amd/csrc/device_common.h sin_cos_of_acos):
sin(phi) ~ sqrt((1 - a)(1 + a)) and cos(phi) ~ a for phi = acos(a), a = 2 r - 1 (math.js:180-185), against V8's
own sin(acos(a)) and cos(acos(a)) -- the oracle's fdlibm restatement (oracle/js_fdlibm.h), pinned bit for bit to
node by tests/test_oracle_trig.py.  The kernels keep an estimated pick only when every value within
SPHERE_PICK_EPS = 2^-44 of each product cos(theta) sin(phi), cos(phi), sin(theta) sin(phi) rounds to the same
f32; with OCML's theta terms within 2^-50 of V8's (tests/test_gpu_trig.py) and these within 2^-50, a product
is within 3 * 2^-50 + 2^-52 of V8's, inside the margin, so a kept pick is V8's bit for bit.  Host-only (the
identity is evaluated here in numpy with the device's operations: two exact-or-rounded f64 factors, one
product, a correctly rounded square root)."""
import ctypes

import numpy as np

BOUND = 2.0 ** -50
EPS = 2.0 ** -44


def _v8_trig(x):
    from oracle import pyoracle
    L = pyoracle.lib()
    L.jsrt_oracle_trig.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty((len(x), 3))
    L.jsrt_oracle_trig(x.ctypes.data, y.ctypes.data, len(x))
    return y  # sin, cos, acos


def _acos_args():
    rng = np.random.default_rng(20261018)
    # the generator's doubles: (hi * 2^26 + lo) * 2^-53 (keyed_rng.js), so a = 2 r - 1 is a multiple of 2^-52
    r = (rng.integers(0, 1 << 27, 4_000_000, dtype=np.int64) * (1 << 26) +
         rng.integers(0, 1 << 26, 4_000_000, dtype=np.int64)) * 2.0 ** -53
    a = 2.0 * r - 1.0
    k = np.arange(1, 53, dtype=np.float64)
    poles = np.concatenate([1 - 2.0 ** -k, -1 + 2.0 ** -k, 2.0 ** -k, -(2.0 ** -k), [-1.0, 0.0, 1.0, -0.0]])
    return np.concatenate([a, poles])


def test_sin_cos_of_acos_within_filter_margin():
    a = _acos_args()
    phi = _v8_trig(a)[:, 2]
    sc = _v8_trig(phi)
    v8_sin, v8_cos = sc[:, 0], sc[:, 1]
    est_sin = np.sqrt((1.0 - a) * (1.0 + a))  # device: sqrt((1.0 - a) * (1.0 + a)), each step one IEEE f64 op
    est_cos = a
    d_sin = np.abs(est_sin - v8_sin).max()
    d_cos = np.abs(est_cos - v8_cos).max()
    assert max(d_sin, d_cos) <= BOUND, (d_sin, d_cos)
    assert BOUND * 32 <= EPS
    # not the same function bit for bit: the filter (and the fdlibm fallback) is what makes it exact
    assert (est_sin != v8_sin).any() or (est_cos != v8_cos).any()
