"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Known answers for the shading inputs of one hit, computed by the reference
 * itself (vm-loaded by load_reference.js):
 *
 *   material -- for the "primary" and "random" rays of tests/golden/casts/<scene>.json.gz, the
 *               material_data Primitive.color (src/world.js:125-137) hands to Material.color after
 *               Geometry.materialData (geometry.js:210-224, 249-254, 376-409, 449-455; sdf.js:41-47):
 *               the world normal (inv_transform.transposed().times(n).to4(0).normalized()), the world
 *               position, UV, the triangle's barycentric coordinates and the SDF basecolor.  Captured by
 *               replacing every Material class's color() with a recorder and calling
 *               World.color(ray, 1) (world.js:31-41) -- the reference's own code up to that call.
 *   sdf      -- for every SDFGeometry primitive: SDF.distance(p) of its root (sdf.js:53-74 and the tree
 *               of sdf.js:78-477) at points p in the primitive's local frame: random points in the root's
 *               bounding box (x1.25) and the local hit points of the material set's rays on it (the
 *               points sphere tracing and the forward-difference normal evaluate).
 *
 *   node oracle/refharness/make_material_kats.js <casts dir> <outdir> <scene>...
 * writes <outdir>/<scene>.json: {scene, blob_sha256, material: {n, rays (base64 f32 n x 6), t (f64),
 *   obj (i32), normal (f32 n x 4), position (f32 n x 4), uv (f32 n x 3), bary (f32 n x 3),
 *   basecolor (f32 n x 3)} (NaN where the field is absent), sdf: [{obj, n, points (f32 n x 4),
 *   distance (f64 n)}]}
 */
const fs = require("fs");
const path = require("path");
const zlib = require("zlib");
const crypto = require("crypto");
const { loadScene, refClass } = require("./load_reference");
const { SceneBlobWriter } = require("../../jsraytracer_amd/js/scene_blob");

let s = 0x13579bd;
function r() { s = (Math.imul(s, 1103515245) + 12345) >>> 0; return s / 4294967296; }
const b64 = (typed) => Buffer.from(typed.buffer, typed.byteOffset, typed.byteLength).toString("base64");
const unb64 = (str, T) => { const b = Buffer.from(str, "base64"); return new T(b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength)); };

function put(dst, k, width, v) {  // a Vec / number array (or undefined) into row k, NaN padded
    for (let i = 0; i < width; ++i) dst[width * k + i] = (v && i < v.length) ? v[i] : NaN;
}

async function main() {
    const castsDir = path.resolve(process.argv[2]), outdir = path.resolve(process.argv[3]);
    fs.mkdirSync(outdir, { recursive: true });
    const Vec = refClass("Vec"), Ray = refClass("Ray"), World = refClass("World");
    const materialClasses = ["SolidColorMaterial", "TransparentMaterial", "PositionalUVMaterial", "PhongMaterial",
                             "FresnelPhongMaterial", "PhongPathTracingMaterial"].map(refClass);
    for (const name of process.argv.slice(4)) {
        const test = await loadScene(name);
        const w = new SceneBlobWriter();
        const blob = w.build(test);
        const world = test.renderer.world;
        const kat = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(castsDir, name + ".json.gz"))));
        const rays = [];
        for (const set of kat.sets) {
            if (set.name !== "primary" && set.name !== "random") continue;
            const R = unb64(set.rays, Float32Array);
            for (let k = 0; k < set.n; ++k)
                rays.push(new Ray(Vec.of(R[6 * k], R[6 * k + 1], R[6 * k + 2], 1), Vec.of(R[6 * k + 3], R[6 * k + 4], R[6 * k + 5], 0)));
        }
        const n = rays.length;
        const RR = new Float32Array(6 * n), T = new Float64Array(n), O = new Int32Array(n);
        const NRM = new Float32Array(4 * n), POS = new Float32Array(4 * n), UV = new Float32Array(3 * n),
              BARY = new Float32Array(3 * n), BC = new Float32Array(3 * n);
        let captured = null;
        const saved = materialClasses.map(c => Object.getOwnPropertyDescriptor(c.prototype, "color"));
        for (const c of materialClasses) c.prototype.color = function (data) { captured = data; return Vec.of(0, 0, 0); };
        const hitsOn = new Map();  // SDF primitive -> local hit points
        try {
            rays.forEach((ray, k) => {
                for (let i = 0; i < 3; ++i) { RR[6 * k + i] = ray.origin[i]; RR[6 * k + 3 + i] = ray.direction[i]; }
                const h = world.cast(ray);
                T[k] = h.distance;
                O[k] = h.object == null ? -1 : w.maps.obj.get(h.object);
                captured = null;
                world.color(ray, 1);
                const d = captured || {};
                put(NRM, k, 4, d.normal);
                put(POS, k, 4, d.position);
                put(UV, k, 3, d.UV);
                put(BARY, k, 3, d.bary);
                put(BC, k, 3, d.basecolor);
                if (h.object != null && h.object.geometry && h.object.geometry.constructor.name === "SDFGeometry" &&
                    h.ancestors.length === 0) {
                    const lr = ray.getTransformed(h.object.getInvTransform());
                    if (!hitsOn.has(h.object)) hitsOn.set(h.object, []);
                    hitsOn.get(h.object).push(lr.getPoint(h.distance));
                }
            });
        } finally {
            materialClasses.forEach((c, i) => {
                if (saved[i]) Object.defineProperty(c.prototype, "color", saved[i]);
                else delete c.prototype.color;  // inherited before
            });
        }
        const sdf = [];
        for (const o of world.objects) {
            if (!o.geometry || o.geometry.constructor.name !== "SDFGeometry") continue;
            const root = o.geometry.root_sdf;
            const bb = root.getBoundingBox(refClass("Mat4").identity(), refClass("Mat4").identity());
            const pts = [];
            for (let k = 0; k < 256; ++k) {
                const p = [0, 1, 2].map(i => {
                    const c = isFinite(bb.center[i]) ? bb.center[i] : 0;
                    const h = isFinite(bb.half_size[i]) ? bb.half_size[i] : 4;
                    return c + (2 * r() - 1) * 1.25 * h;
                });
                pts.push(Vec.of(p[0], p[1], p[2], 1));
            }
            for (const p of (hitsOn.get(o) || []).slice(0, 256)) pts.push(p);
            const P = new Float32Array(4 * pts.length), D = new Float64Array(pts.length);
            pts.forEach((p, k) => { put(P, k, 4, p); D[k] = root.distance(p); });
            sdf.push({ obj: w.maps.obj.get(o), n: pts.length, points: b64(P), distance: b64(D) });
        }
        const sha = crypto.createHash("sha256").update(blob).digest("hex");
        if (sha !== kat.blob_sha256) throw new Error(`${name}: scene blob differs from the cast KATs' blob`);
        const material = { n, rays: b64(RR), t: b64(T), obj: b64(O), normal: b64(NRM), position: b64(POS), uv: b64(UV),
                           bary: b64(BARY), basecolor: b64(BC) };
        fs.writeFileSync(path.join(outdir, name + ".json"), JSON.stringify({ scene: name, blob_sha256: sha, material, sdf }));
        console.log(`${name}: ${n} material rays (${Array.from(O).filter(x => x >= 0).length} hits), ` +
                    `${sdf.map(x => x.n).join("+") || 0} SDF points`);
    }
}
main().catch(e => { console.error(e); process.exit(1); });
