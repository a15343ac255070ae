"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Fixtures for the native OBJ ingest + BVH builder
 * (jsraytracer_amd/csrc/mesh_build.cpp, include/jsrt_mesh.h), produced by the REFERENCE itself.
 *
 *   node oracle/refharness/make_mesh_fixtures.js <outdir> [scene ...]      (default: bunny dragon)
 *
 * Per mesh scene (tests/<scene>/test.mjs, which loads its OBJ through loadObjFile and builds a
 * BVHAggregate, objloader.js:224-231 / aggregates.js:33-41):
 *   <outdir>/<scene>.full.jsrt  the scene exported with the reference-built BVH (not committed for
 *                               the dragon: tests keep only its topology digest, see mesh_topology.py)
 *   <outdir>/<scene>.skel.jsrt  the same scene, but BVHAggregate.build handed only the FIRST
 *                               triangle: a one-leaf tree whose one Primitive is the template
 *                               (material, transform) jsrt_blob_attach_obj copies to every triangle
 *   <outdir>/<scene>.json       {obj, nodes, max_depth, triangles} from the reference's BVHAggregate
 */
const fs = require("fs");
const path = require("path");
const { loadScene, refClass, REF } = require("./load_reference");
const { exportScene } = require("../../jsraytracer_amd/js/scene_blob");

const OBJ_OF = { bunny: "assets/bunny2.obj", dragon: "assets/dragon.obj", bunny_path: "assets/bunny2.obj" };

async function main() {
    const outdir = path.resolve(process.argv[2]);
    const scenes = process.argv.length > 3 ? process.argv.slice(3) : ["bunny", "dragon"];
    fs.mkdirSync(outdir, { recursive: true });
    const BVH = refClass("BVHAggregate");
    const build = BVH.build;
    for (const name of scenes) {
        let stats = null;
        BVH.build = function (objects, ...rest) {
            const agg = build.call(this, objects, ...rest);
            stats = { triangles: objects.length, nodes: agg.nodeCount(), max_depth: agg.maxDepth() };
            return agg;
        };
        const full = await loadScene(name);
        fs.writeFileSync(path.join(outdir, name + ".full.jsrt"), exportScene(full));
        BVH.build = function (objects, ...rest) { return build.call(this, [objects[0]], ...rest); };
        const skel = await loadScene(name);
        fs.writeFileSync(path.join(outdir, name + ".skel.jsrt"), exportScene(skel));
        BVH.build = build;
        fs.writeFileSync(path.join(outdir, name + ".json"), JSON.stringify(Object.assign({ obj: OBJ_OF[name] }, stats)));
        console.log(name, JSON.stringify(stats));
    }
}

main().catch(e => { console.error(e); process.exit(1); });
