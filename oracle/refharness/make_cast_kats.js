"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Known-answer vectors for World.cast (src/world.js:28-30), computed by
 * the reference itself (vm-loaded by load_reference.js): for each scene, batches of rays and the
 * reference's closest hit -- its distance (f64) and the hit Primitive, as its OBJS index in the scene
 * blob (jsraytracer_amd/js/scene_blob.js, the same blob as tests/golden/scenes/<name>.jsrt.gz).
 * They localise a parity failure to one cast (one primitive kind, one BVH, one SDF) instead of a
 * whole render:
 *   "primary"  -- Camera.getRayForPixel at a 16x16 grid of pixel centres (cameras.js:29-34): the
 *                 per-pixel primary-hit index (skipped for depth-of-field cameras, which draw);
 *   "random"   -- origins in the scene's finite bounding box (x1.5), directions uniform on the sphere,
 *                 World.cast(ray) (minD 0, maxD Infinity, transparent objects included);
 *   "shadow"   -- segments p -> q between such points, World.cast(ray, 0.0001, 1, false) as
 *                 materials.js:250-252 casts them (shadow-casting objects only).
 *
 *   node oracle/refharness/make_cast_kats.js <outdir> <scene>...
 * writes <outdir>/<scene>.json: {scene, blob_sha256, sets: [{name, minD, maxD, transp, n,
 *   rays: base64 f32 n x 6 (origin xyz w=1, direction xyz w=0), t: base64 f64 n, obj: base64 i32 n}]}
 */
const fs = require("fs");
const path = require("path");
const crypto = require("crypto");
const { loadScene, refClass } = require("./load_reference");
const { SceneBlobWriter } = require("../../jsraytracer_amd/js/scene_blob");

let s = 0x2468ace;
function r() { s = (Math.imul(s, 1103515245) + 12345) >>> 0; return s / 4294967296; }
const b64 = (typed) => Buffer.from(typed.buffer, typed.byteOffset, typed.byteLength).toString("base64");

async function main() {
    const outdir = path.resolve(process.argv[2]);
    fs.mkdirSync(outdir, { recursive: true });
    const Vec = refClass("Vec"), Ray = refClass("Ray");
    for (const name of process.argv.slice(3)) {
        const test = await loadScene(name);
        const w = new SceneBlobWriter();
        const blob = w.build(test);
        const world = test.renderer.world, cam = test.renderer.camera;
        const box = world.getFiniteBoundingBox();
        const lo = [0, 1, 2].map(i => box.center[i] - 1.5 * box.half_size[i]);
        const ext = [0, 1, 2].map(i => 3 * box.half_size[i]);
        const point = () => Vec.of(lo[0] + r() * ext[0], lo[1] + r() * ext[1], lo[2] + r() * ext[2], 1);
        const objOf = (o) => (o == null ? -1 : w.maps.obj.get(o));
        const sets = [];
        const run = (setName, rays, minD, maxD, transp) => {
            const n = rays.length;
            const R = new Float32Array(6 * n), T = new Float64Array(n), O = new Int32Array(n);
            rays.forEach((ray, k) => {
                for (let i = 0; i < 3; ++i) { R[6 * k + i] = ray.origin[i]; R[6 * k + 3 + i] = ray.direction[i]; }
                const h = world.cast(ray, minD, maxD, transp);
                T[k] = h.distance;
                O[k] = objOf(h.object);
            });
            sets.push({ name: setName, minD, maxD: isFinite(maxD) ? maxD : "Infinity", transp, n,
                        rays: b64(R), t: b64(T), obj: b64(O) });
        };
        const isDof = cam.constructor.name === "DepthOfFieldPerspectiveCamera";
        if (!isDof) {
            const rays = [];
            for (let j = 0; j < 16; ++j)
                for (let i = 0; i < 16; ++i) rays.push(cam.getRayForPixel(2 * (i + 0.5) / 16 - 1, 1 - 2 * (j + 0.5) / 16));
            run("primary", rays, 0, Infinity, true);
        }
        const rnd = [], sh = [];
        for (let k = 0; k < 512; ++k) {
            const th = 2 * Math.PI * r(), z = 2 * r() - 1, q = Math.sqrt(1 - z * z);
            rnd.push(new Ray(point(), Vec.of(q * Math.cos(th), q * Math.sin(th), z, 0)));
        }
        run("random", rnd, 0, Infinity, true);
        for (let k = 0; k < 256; ++k) {
            const p = point(), q = point();
            sh.push(new Ray(p, q.minus(p)));
        }
        run("shadow", sh, 0.0001, 1, false);
        const sha = crypto.createHash("sha256").update(blob).digest("hex");
        fs.writeFileSync(path.join(outdir, name + ".json"), JSON.stringify({ scene: name, blob_sha256: sha, sets }));
        console.log(`${name}: ${sets.map(x => x.name + " " + x.n).join(", ")}`);
    }
}
main().catch(e => { console.error(e); process.exit(1); });
