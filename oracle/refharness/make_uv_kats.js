// Math.atan2 / Math.asin of node (V8, the reference's runtime) on the (x, y) float64 pairs in argv[2] (raw
// little-endian doubles, x0 y0 x1 y1 ...); writes argv[3]: per pair [atan2(y, x), asin(x)] (raw doubles).
// Used by regen_uv_kats.py to pin the fdlibm atan2 / asin of oracle/js_fdlibm.h and jsraytracer_amd/csrc/fdlibm.h.
'use strict';
const fs = require('fs');
const buf = fs.readFileSync(process.argv[2]);
const a = new Float64Array(buf.buffer, buf.byteOffset, buf.length / 8);
const n = a.length / 2;
const out = new Float64Array(n * 2);
for (let i = 0; i < n; ++i) {
    out[2 * i] = Math.atan2(a[2 * i + 1], a[2 * i]);
    out[2 * i + 1] = Math.asin(a[2 * i]);
}
fs.writeFileSync(process.argv[3], Buffer.from(out.buffer));
