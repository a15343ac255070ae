"""Regenerates tests/golden/pow_v8.npz: node's (V8's) Math.pow(x, n) on seeded specular-term arguments -- x in
[0, 1 + 3e-7] (Math.max(L.dot(R), 0) of unit f32 vectors, materials.js:266) and the integer exponents the
reference scenes use as smoothness (tests/test_box_any.py-style seeded draws) -- for tests/test_pow_parity.py.

    python oracle/refharness/regen_pow_kats.py        (needs node; run in the build container)
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "tests", "golden", "pow_v8.npz")
JS = """'use strict';
const fs = require('fs');
const b = fs.readFileSync(process.argv[2]);
const a = new Float64Array(b.buffer, b.byteOffset, b.length / 8);
const out = new Float64Array(a.length / 2);
for (let i = 0; i < out.length; ++i) out[i] = Math.pow(a[2 * i], a[2 * i + 1]);
fs.writeFileSync(process.argv[3], Buffer.from(out.buffer));
"""


def pow_args(seed=20261019, n=150_000):
    rng = np.random.default_rng(seed)
    x = rng.random(n) * 1.0000003
    y = rng.choice([2.0, 3.0, 5.0, 10.0, 20.0, 50.0, 64.0, 100.0], n)
    return x, y


def main():
    x, y = pow_args()
    a = np.empty(2 * len(x))
    a[0::2], a[1::2] = x, y
    with tempfile.TemporaryDirectory() as t:
        js, fi, fo = os.path.join(t, "p.js"), os.path.join(t, "in.f64"), os.path.join(t, "out.f64")
        open(js, "w").write(JS)
        a.tofile(fi)
        subprocess.run(["node", js, fi, fo], check=True)
        v = np.fromfile(fo, dtype=np.float64)
    np.savez_compressed(OUT, seed=np.array([20261019]), n=np.array([len(x)]), v8=v)  # arguments: pow_args(seed)
    print("wrote", OUT, len(x))


if __name__ == "__main__":
    main()
