// Math.sin / Math.cos / Math.acos of node (V8, the reference's runtime) on the float64 arguments in
// argv[2] (raw little-endian doubles); writes argv[3]: per argument [sin, cos, acos] (raw doubles).
// Used by regen_trig_kats.py to pin jsraytracer_amd/csrc/fdlibm.h to V8 bit for bit.
'use strict';
const fs = require('fs');
const buf = fs.readFileSync(process.argv[2]);
const x = new Float64Array(buf.buffer, buf.byteOffset, buf.length / 8);
const out = new Float64Array(x.length * 3);
for (let i = 0; i < x.length; ++i) {
    out[3 * i] = Math.sin(x[i]);
    out[3 * i + 1] = Math.cos(x[i]);
    out[3 * i + 2] = Math.acos(x[i]);
}
fs.writeFileSync(process.argv[3], Buffer.from(out.buffer));
