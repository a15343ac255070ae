"""Regenerates tests/golden/uv_v8.npz: node's (V8's) Math.atan2(y, x) and Math.asin(x) on the seeded argument
pairs of uv_args() -- the components of f32 unit vectors (Vec.cartesianToSpherical's atan2(z, x) and asin(y),
math.js:189-193), points of a unit cylinder (geometry.js:479-487), wide random pairs and special values.  The
fixture keeps a subsample with its results and the SHA-256 of the full result arrays (tests/test_fdlibm.py,
tests/test_oracle_trig.py).

    python oracle/refharness/regen_uv_kats.py        (needs node; run in the build container)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "tests", "golden", "uv_v8.npz")
sys.path.insert(0, HERE)
from regen_trig_kats import digest  # noqa: E402


def uv_args(seed=20261018):
    rng = np.random.default_rng(seed)
    u = rng.normal(size=(1_500_000, 3))
    u = (u / np.linalg.norm(u, axis=1, keepdims=True)).astype(np.float32).astype(np.float64)
    sp = [np.stack([u[:, 0], u[:, 2]], 1), np.stack([u[:, 1], u[:, 0]], 1)]  # atan2(z, x) / asin(y)
    r = rng.uniform(-1, 1, (500_000, 2))
    wide = rng.normal(size=(500_000, 2)) * np.exp(rng.uniform(-40, 40, (500_000, 2)))
    axes = np.array([[0.0, 1.0], [0.0, -1.0], [-0.0, 1.0], [1.0, 0.0], [-1.0, 0.0], [1.0, -0.0], [-1.0, -0.0],
                     [0.0, 0.0], [-0.0, 0.0], [0.0, -0.0], [-0.0, -0.0], [np.inf, 1.0], [-np.inf, 1.0],
                     [np.inf, np.inf], [-np.inf, -np.inf], [1.0, np.inf], [np.nan, 1.0], [1.0, np.nan], [0.5, 0.5],
                     [-0.5, 0.5], [1e-300, 1.0], [1.0, 1e-300], [-1e-300, 1e300], [0.975, 0.1], [-0.975, 0.1],
                     [2 ** -28, 1.0], [2 ** -27, 1.0], [0.4375, 1.0], [1.1875, 1.0], [2.4375, 1.0]])
    return np.ascontiguousarray(np.concatenate(sp + [r, wide, axes]), dtype=np.float64)


def main():
    xy = uv_args()
    with tempfile.TemporaryDirectory() as t:
        fi, fo = os.path.join(t, "xy.f64"), os.path.join(t, "out.f64")
        xy.tofile(fi)
        subprocess.run(["node", os.path.join(HERE, "make_uv_kats.js"), fi, fo], check=True)
        y = np.fromfile(fo, dtype=np.float64).reshape(-1, 2)
    sub = np.arange(0, len(xy), 97)
    np.savez_compressed(OUT, args_seed=np.array([20261018]), n=np.array([len(xy)]), sub_xy=xy[sub], sub_y=y[sub],
                        sha_atan2=np.array(digest(y[:, 0])), sha_asin=np.array(digest(y[:, 1])))
    print("wrote", OUT, len(xy), "pairs")


if __name__ == "__main__":
    main()
