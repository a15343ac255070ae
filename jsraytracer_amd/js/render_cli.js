"use strict";
/*
 * render_cli.js — render one JSRT scene through HipRenderer (N-API -> libjsrt) and write the RGBA8
 * PixelBuffer bytes.  Used by the GPU tests to check the Node boundary end to end.
 *
 *   node render_cli.js <scene.jsrt[.gz]> <out.rgba> <width> <height> <spp> <depth> <kind> <seed>
 *                      [x_offset x_delt] [sync|async]
 */
const fs = require("fs");
const zlib = require("zlib");
const { HipRenderer, NodePixelBuffer } = require("./hip_renderer");

async function main() {
    const a = process.argv.slice(2);
    const [scene, out] = a;
    const [W, H, spp, depth, kind, seed] = a.slice(2, 8).map((x) => parseInt(x, 10));
    const xo = a[8] !== undefined ? parseInt(a[8], 10) : 0, xd = a[9] !== undefined ? parseInt(a[9], 10) : 1;
    const mode = a[10] || "sync";
    let b = fs.readFileSync(scene);
    if (scene.endsWith(".gz")) b = zlib.gunzipSync(b);
    const r = new HipRenderer(new Uint8Array(b.buffer, b.byteOffset, b.byteLength),
                              { samplesPerPixel: spp, maxRecursionDepth: depth, kind, seed });
    const img = new NodePixelBuffer(W, H);
    const progress = [];
    const cb = (st) => progress.push(st);
    if (mode === "async") await r.renderAsync(img, 1e-6, cb, xo, xd);
    else r.render(img, 1e-6, cb, xo, xd);
    fs.writeFileSync(out, Buffer.from(img.imgdata.data.buffer));
    console.log(JSON.stringify({ stats: r.stats, progress: progress.length }));
    r.destroy();
}
main().catch((e) => { console.error(e); process.exit(1); });
