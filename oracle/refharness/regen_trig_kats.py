"""Regenerates tests/golden/trig_v8.npz: node's (V8's) Math.sin / Math.cos / Math.acos on the seeded
arguments of trig_args() -- the angles the reference takes them of (2 pi r, acos(2 r - 1), r in [0, 1)),
wider ranges, the neighbours of multiples of pi/4 and pi/2, tiny and special values.  The fixture keeps a
subsample with its results and the SHA-256 of the full result arrays (test: tests/test_fdlibm.py).

    python oracle/refharness/regen_trig_kats.py        (needs node; run in the build container)
"""
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "tests", "golden", "trig_v8.npz")


def trig_args(seed=20261017):
    rng = np.random.default_rng(seed)
    r = rng.random(1_000_000)
    k = np.arange(-40, 41, dtype=np.float64)
    near = np.concatenate([k * (np.pi / 4), k * (np.pi / 2)])
    near = np.concatenate([near + d for d in (0.0, 1e-12, -1e-12, 1e-6, -1e-6)]
                          + [np.nextafter(near, np.inf), np.nextafter(near, -np.inf)])
    parts = [
        2.0 * np.pi * r,                              # spherePick theta (math.js:181)
        2.0 * rng.random(1_000_000) - 1.0,            # acos argument (math.js:182), phi's input
        np.arccos(2.0 * rng.random(500_000) - 1.0),   # sin / cos of phi
        rng.uniform(-10, 10, 500_000),
        np.exp(rng.uniform(np.log(1e-20), np.log(1e5), 300_000)) * rng.choice([-1.0, 1.0], 300_000),
        near,
        np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 2 ** -27, -2 ** -27, 2 ** -28, 2 ** -57, 2 ** -58, 1e-300,
                  np.nextafter(1.0, 0), np.nextafter(-1.0, 0), np.nextafter(0.5, 1), np.nextafter(-0.5, -1),
                  0.3, np.nextafter(0.3, 1), 0.78125, np.inf, -np.inf, np.nan, 2 ** 19 * np.pi / 2 * 0.999]),
    ]
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float64)


def digest(a):
    """SHA-256 of a result array with every NaN canonical (payloads are not part of the contract)."""
    a = np.array(a, dtype=np.float64)
    a[np.isnan(a)] = np.nan
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    x = trig_args()
    with tempfile.TemporaryDirectory() as t:
        fi, fo = os.path.join(t, "x.f64"), os.path.join(t, "y.f64")
        x.tofile(fi)
        subprocess.run(["node", os.path.join(HERE, "make_trig_kats.js"), fi, fo], check=True)
        y = np.fromfile(fo, dtype=np.float64).reshape(-1, 3)
    sub = np.arange(0, len(x), 97)
    np.savez_compressed(OUT, args_seed=np.array([20261017]), n=np.array([len(x)]),
                        sub_index=sub, sub_x=x[sub], sub_y=y[sub],
                        sha_sin=np.array(digest(y[:, 0])), sha_cos=np.array(digest(y[:, 1])),
                        sha_acos=np.array(digest(y[:, 2])))
    print(OUT, len(x), "arguments")


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
