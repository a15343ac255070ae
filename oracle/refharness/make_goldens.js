"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Generates the committed parity fixtures under tests/golden/ by running
 * the REFERENCE renderer itself (vm-loaded from /root/reference/src, see load_reference.js) with the
 * keyed RNG of keyed_rng.js substituted for Math.random.
 *
 *   node oracle/refharness/make_goldens.js <spec.json> <outdir>
 *
 * spec.json: {"scenes": {"<name>": {"renders": [{kind, width, height, spp, depth?, seed,
 *             x_offset?, x_delt?}]}}}
 *
 * Per scene it writes  <outdir>/scenes/<name>.jsrt  (scene blob, jsraytracer_amd/js/scene_blob.js)
 * and per render       <outdir>/images/<tag>.rgba   (the reference's ImageData bytes, pixelbuffer.js)
 *                      <outdir>/images/<tag>.f32    (last colour handed to PixelBuffer.setColor per
 *                                                    pixel, f32 x4, NaN-padded; pixelbuffer.js:39)
 * and <outdir>/index.json with the metadata (draw counts, World.color call counts, wall time).
 */
const fs = require("fs");
const path = require("path");
const { loadScene, refClass } = require("./load_reference");
const { installKeyedRng, sampleOrder } = require("./keyed_rng");
const { exportScene } = require("../../jsraytracer_amd/js/scene_blob");

const KIND_NAMES = ["simple", "incremental", "random"];

function makeRenderer(test, kind, spp, depth) {
    const R = test.renderer;
    const d = depth !== undefined ? depth : R.maxRecursionDepth;
    if (kind === 0) return new (refClass("SimpleRenderer"))(R.world, R.camera, d);
    if (kind === 1) return new (refClass("IncrementalMultisamplingRenderer"))(R.world, R.camera, spp, d);
    return new (refClass("RandomMultisamplingRenderer"))(R.world, R.camera, spp, d);
}

function tagOf(name, r) {
    const part = (r.x_delt && r.x_delt > 1) ? `_part${r.x_offset}of${r.x_delt}` : "";
    return `${name}_${KIND_NAMES[r.kind]}_${r.width}x${r.height}_s${r.spp}_d${r.depth}_seed${r.seed}${part}`;
}

async function main() {
    const spec = JSON.parse(fs.readFileSync(process.argv[2], "utf8"));
    const outdir = path.resolve(process.argv[3]);
    fs.mkdirSync(path.join(outdir, "scenes"), { recursive: true });
    fs.mkdirSync(path.join(outdir, "images"), { recursive: true });
    const indexPath = path.join(outdir, "index.json");
    const index = fs.existsSync(indexPath) ? JSON.parse(fs.readFileSync(indexPath, "utf8")) : { renders: {} };

    const PixelBuffer = refClass("PixelBuffer");
    for (const [name, sc] of Object.entries(spec.scenes)) {
        const t0 = Date.now();
        const test = await loadScene(name);
        const blob = exportScene(test);
        fs.writeFileSync(path.join(outdir, "scenes", name + ".jsrt"), blob);
        console.log(`${name}: scene exported (${blob.length} B, ${Date.now() - t0} ms)`);
        for (const r0 of sc.renders) {
            const r = Object.assign({ x_offset: 0, x_delt: 1 }, r0);
            if (r.depth === undefined) r.depth = test.renderer.maxRecursionDepth;
            const renderer = makeRenderer(test, r.kind, r.spp, r.depth);
            const W = r.width, H = r.height;
            const colors = new Float32Array(W * H * 4).fill(NaN);
            const lens = new Uint8Array(W * H);
            const pb = new PixelBuffer(W, H);
            const origSet = PixelBuffer.prototype.setColor;
            pb.setColor = function (x, y, color) {
                const i = y * W + x;
                for (let k = 0; k < 4; ++k) colors[4 * i + k] = k < color.length ? color[k] : NaN;
                lens[i] = color.length;
                return origSet.call(this, x, y, color);
            };
            const ctl = installKeyedRng(r.seed);
            ctl.startSequence(sampleOrder(r.kind, W, H, r.spp, r.x_offset, r.x_delt));
            const t1 = Date.now();
            renderer.render(pb, 0, false, r.x_offset, r.x_delt);
            const ms = Date.now() - t1;
            const tag = tagOf(name, r);
            fs.writeFileSync(path.join(outdir, "images", tag + ".rgba"), Buffer.from(pb.imgdata.data.buffer));
            fs.writeFileSync(path.join(outdir, "images", tag + ".f32"), Buffer.from(colors.buffer));
            index.renders[tag] = Object.assign({ scene: name, kind_name: KIND_NAMES[r.kind], draws: ctl.draws,
                                                 color_calls: ctl.colorCalls, ms, color_len: Math.max(...lens) }, r);
            console.log(`  ${tag}: ${ms} ms, ${ctl.draws} draws, ${ctl.colorCalls} World.color calls`);
        }
    }
    fs.writeFileSync(indexPath, JSON.stringify(index, null, 1));
}

main().catch(e => { console.error(e); process.exit(1); });
