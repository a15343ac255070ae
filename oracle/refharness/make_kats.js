"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Known-answer vectors for the reference's scalar building blocks,
 * computed by the reference's own code in this Node realm:
 *   Math.fmod (src/math.js:27, toPrecision(8) rounding)  and the keyed RNG (keyed_rng.js).
 *   node oracle/refharness/make_kats.js > tests/golden/kats.json
 */
const { loadReference } = require("./load_reference");
const { keyedUniform, mix } = require("./keyed_rng");
loadReference();
let s = 0x1234567;
function r() { s = (Math.imul(s, 1103515245) + 12345) >>> 0; return s / 4294967296; }
const hex = (x) => { const b = Buffer.alloc(8); b.writeDoubleLE(x); return b.toString("hex"); };
const fmod = [];
const special = [[1.00390625, 7], [0.5, 2], [-0.5, 2], [3, 2], [-3, 2], [1e-9, 2], [-1e-9, 2], [1.0000000500000001, 2],
                 [5e-324, 2], [1e21, 7], [123456785, 1e12], [0, 2], [-0, 2], [Infinity, 2], [NaN, 2], [2.5, 0.1],
                 [1/3, 2], [2/3, 2], [-1/3, 2], [0.99999999999, 2], [1.99999999999, 2], [7.5e-16, 2], [1e-30, 3]];
for (const [a, b] of special) fmod.push([hex(a), hex(b), hex(Math.fmod(a, b))]);
for (let i = 0; i < 4000; ++i) {
    const e = Math.floor(r() * 30) - 12;
    const a = (r() * 2 - 1) * Math.pow(10, e), b = [2, 1, 3, 0.5, 2 / 3][i % 5];
    fmod.push([hex(a), hex(b), hex(Math.fmod(a, b))]);
}
for (let i = 0; i < 2000; ++i) { // Menger-like arguments: f32 point + size/2, size 2
    const p = Math.fround((r() * 2 - 1) * 3);
    fmod.push([hex(p + 1), hex(2), hex(Math.fmod(p + 1, 2))]);
}
const rng = [];
for (let i = 0; i < 500; ++i) {
    const k = [Math.floor(r() * 4294967296), Math.floor(r() * 4294967296), Math.floor(r() * 256), Math.floor(r() * 4294967296), Math.floor(r() * 64)];
    rng.push([k, hex(keyedUniform(...k))]);
}
const mixes = [];
for (let i = 0; i < 200; ++i) { const a = Math.floor(r() * 4294967296), b = Math.floor(r() * 4294967296); mixes.push([a, b, mix(a, b)]); }
process.stdout.write(JSON.stringify({ fmod, rng, mix: mixes }));
