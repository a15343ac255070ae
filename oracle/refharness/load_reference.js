"use strict";
/*
 * TEST INFRASTRUCTURE ONLY (oracle side).  Loads the reference renderer's own source files
 * (/root/reference/src/*.js) into this Node realm so that fixtures can be generated from the
 * reference itself.  Nothing is copied: the files are read and evaluated at run time, the way
 * the reference's own offline tool does it (tests/test_to_json.js:8-23).  Only usable where
 * /root/reference exists (the dev container), never on the GPU box.
 *
 * Shims (SURVEY.md §8c): global fs / fspromise (objloader.js:24 textFetch reads files through
 * `fspromise` when not in a browser), ImageData (pixelbuffer.js:6).
 */
const fs = require("fs");
const path = require("path");
const vm = require("vm");

const REF = process.env.JSRT_REFERENCE || "/root/reference";

function loadReference() {
    if (global.__jsrt_reference_loaded) return REF;
    if (!fs.existsSync(path.join(REF, "src", "math.js")))
        throw new Error("reference sources not found under " + REF);
    global.fs = fs;
    global.fspromise = fs.promises;
    global.ImageData = class ImageData {
        constructor(w, h) { this.width = w; this.height = h; this.data = new Uint8ClampedArray(w * h * 4); }
    };
    // same order as src/worker.js:3-14 (+ serializer.js as in tests/test_to_json.js:20)
    for (const r of ["math", "world", "pixelbuffer", "geometry", "materials", "cameras", "renderers",
                     "lights", "objloader", "sdf", "aggregates", "serializer"]) {
        const fn = path.join(REF, "src", r + ".js");
        new vm.Script(fs.readFileSync(fn).toString(), { filename: fn }).runInThisContext();
    }
    global.__jsrt_reference_loaded = true;
    return REF;
}

// Resolve a test scene: returns a Promise of the {renderer, width, height} the test's
// configureTest(callback) produces (tests/<name>/test.mjs).
function loadScene(name) {
    loadReference();
    const testsDir = path.join(REF, "tests");
    process.chdir(testsDir); // objloader paths are relative ("../assets/...")
    return import(path.join(testsDir, name, "test.mjs")).then(m => new Promise((resolve, reject) => {
        try { m.configureTest(resolve); } catch (e) { reject(e); }
    }));
}

function refClass(name) { loadReference(); return (0, eval)(name); }

module.exports = { loadReference, loadScene, refClass, REF };
