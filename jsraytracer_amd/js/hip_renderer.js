"use strict";
/*
 * hip_renderer.js — the JS host side of the drop-in boundary.
 *
 * HipRenderer keeps the reference renderer contract (src/renderers.js:10 SimpleRenderer.render,
 * :70 IncrementalMultisamplingRenderer.render):
 *
 *     renderer.render(img, timelimit = 0, callback = false, x_offset = 0, x_delt = 1) -> img
 *
 * `img` is a PixelBuffer (src/pixelbuffer.js:1-50: img.imgdata = ImageData {width, height, data}),
 * columns px = x_offset, x_offset + x_delt, ... are written with the PixelBuffer.setColor rules, the
 * other columns are left untouched (as each reference worker leaves them, src/worker.js:26-38), and
 * callback({pass, completion}) fires no more often than every `timelimit` ms (renderers.js:28-37,
 * 103-112).  The render runs on the MI355X through libjsrt (include/jsrt.h) via the N-API addon
 * jsrt_node.node; render() blocks like the reference, renderAsync() returns a Promise.
 *
 * The scene crosses the boundary as a JSRT blob (include/jsrt_scene.h): either a prebuilt blob
 * (Buffer/Uint8Array) or a live reference renderer ({world, camera, samplesPerPixel,
 * maxRecursionDepth}), exported with scene_blob.js (in place of src/serializer.js).
 */
const path = require("path");

const ABI_VERSION = 4;  // include/jsrt.h JSRT_ABI_VERSION this wrapper is written against
let _addon = null;
function addon() {
    if (_addon) return _addon;
    const p = process.env.JSRT_NODE_ADDON || path.join(__dirname, "..", "_build", "jsrt_node.node");
    const a = require(p);  // throws if the addon was not built: there is no JS fallback renderer
    // a stale libjsrt (the .so travels to the GPU box separately) would misread the stats struct
    if (a.abiVersion() !== ABI_VERSION) throw `HipRenderer: libjsrt ABI ${a.abiVersion()}, expected ${ABI_VERSION}`;
    _addon = a;
    return _addon;
}

/*
 * The device a worker renders on: worker i of the reference's launcher (src/raytrace_launcher.js:65-101,
 * which spawns N workers over one CPU) goes to GPU i % deviceCount, so N workers spread over a node's
 * GPUs round-robin and each renders its interleaved columns (worker.js:30-32) on its own device.
 * deviceCount defaults to the devices HIP sees (0 without a GPU -> device 0).
 */
function deviceForWorker(workerIndex, deviceCount) {
    const n = deviceCount !== undefined ? deviceCount : addon().deviceCount();
    return n > 0 ? workerIndex % n : 0;
}

const KIND = { SimpleRenderer: 0, IncrementalMultisamplingRenderer: 1, RandomMultisamplingRenderer: 2 };

function blobFromLive(renderer, width, height) {
    const { exportScene } = require("./scene_blob");
    return exportScene({ renderer, width, height });
}

function readHeader(blob) {
    const dv = new DataView(blob.buffer, blob.byteOffset, blob.byteLength);
    if (dv.getUint32(0, true) !== 0x5452534A || dv.getUint32(4, true) !== 1) throw "HipRenderer: not a JSRT v1 scene blob";
    const nsec = dv.getUint32(8, true);
    for (let i = 0; i < nsec; ++i) {
        const o = 16 + 24 * i;
        if (dv.getUint32(o, true) === 0x52444E52) {  // 'RNDR'
            const off = Number(dv.getBigUint64(o + 8, true));
            return { kind: dv.getUint32(off, true), spp: dv.getUint32(off + 4, true),
                     maxDepth: dv.getUint32(off + 8, true), width: dv.getUint32(off + 12, true),
                     height: dv.getUint32(off + 16, true) };
        }
    }
    throw "HipRenderer: scene blob has no renderer record";
}

class HipRenderer {
    /*
     * scene: JSRT blob (Buffer / Uint8Array) or a live reference renderer object.
     * opts:  {device = 0, seed = 1, samplesPerPixel, maxRecursionDepth, kind, width, height,
     *         mode = "strict" (include/jsrt.h JSRT_MODE_*; "fast" is refused), deviceMask = 0 (jsrt_params)}
     *        (absent fields come from the scene's own renderer, as the reference's test.mjs sets them)
     */
    constructor(scene, opts = {}) {
        let blob = scene;
        if (!(scene instanceof Uint8Array)) {
            blob = blobFromLive(scene, opts.width || 600, opts.height || 600);
        }
        this.blob = blob;
        const h = readHeader(blob);
        this.kind = opts.kind !== undefined ? (typeof opts.kind === "string" ? KIND[opts.kind] : opts.kind) : h.kind;
        this.samplesPerPixel = opts.samplesPerPixel !== undefined ? opts.samplesPerPixel : h.spp;
        this.maxRecursionDepth = opts.maxRecursionDepth !== undefined ? opts.maxRecursionDepth : h.maxDepth;
        this.seed = opts.seed !== undefined ? opts.seed : 1;
        this.device = opts.device || 0;
        const MODES = { strict: 0, fast: 1 };
        this.mode = opts.mode === undefined ? 0 : (typeof opts.mode === "string" ? MODES[opts.mode] : opts.mode);
        if (this.mode === undefined) throw `HipRenderer: unknown numeric mode ${opts.mode}`;
        this.deviceMask = opts.deviceMask || 0;
        this.handle = addon().sceneCreate(blob, this.device);
    }
    static computePixelCount(img, x_offset, x_delt) {  // renderers.js:7-9
        return ((img.width() / x_delt) + Math.round(1 - x_offset / x_delt) * (img.width() % x_delt)) * img.height();
    }
    _params(img, timelimit, x_offset, x_delt, callback) {
        if (!(x_delt > 0)) throw "HipRenderer: x_delt must be positive";
        // With a callback the Incremental renderer reports per pass (renderers.js:103-112): one sample
        // per pixel per launch, so the callback sees each pass's running mean in img at the reference's
        // cadence.  Without one, the library's batch size renders the frame in as few launches as fit.
        const perPass = !!(timelimit && callback) && this.kind === KIND.IncrementalMultisamplingRenderer;
        return { width: img.width(), height: img.height(), samplesPerPixel: this.samplesPerPixel,
                 maxRecursionDepth: this.maxRecursionDepth, kind: this.kind, seed: this.seed,
                 x_offset, x_delt, device: this.device, timelimit: timelimit || 0,
                 samplesPerLaunch: perPass ? (this.samplesPerLaunch || 1) : 0, mode: this.mode,
                 deviceMask: this.deviceMask };
    }
    render(img, timelimit = 0, callback = false, x_offset = 0, x_delt = 1) {
        const p = this._params(img, timelimit, x_offset, x_delt, callback);
        const cb = (timelimit && callback) ? (pass, completion) => callback({ pass, completion }) : undefined;
        this.stats = addon().renderSync(this.handle, p, img.imgdata.data, cb);
        return img;
    }
    renderAsync(img, timelimit = 0, callback = false, x_offset = 0, x_delt = 1) {
        const p = this._params(img, timelimit, x_offset, x_delt, callback);
        const cb = (timelimit && callback) ? (pass, completion) => callback({ pass, completion }) : undefined;
        return addon().render(this.handle, p, img.imgdata.data, cb).then((st) => { this.stats = st; return img; });
    }
    destroy() {
        if (this.handle) addon().sceneDestroy(this.handle);
        this.handle = null;
    }
}

/* PixelBuffer stand-in for hosts without ImageData (Node): same fields pixelbuffer.js reads. */
class NodePixelBuffer {
    constructor(width, height) {
        this.imgdata = { width, height, data: new Uint8ClampedArray(width * height * 4) };
    }
    width() { return this.imgdata.width; }
    height() { return this.imgdata.height; }
    coord(x, y) { return y * (this.imgdata.width * 4) + x * 4; }
}

// loadObjFile(...) + BVHAggregate.build(...) natively (include/jsrt_mesh.h): splices the OBJ's triangles
// and their reference-identical BVH into the skeleton blob's one-leaf BVHAggregate (its template
// Primitive carries the material and transform loadObjFile would be given).
function attachObj(blob, objText, opts) { return addon().attachObj(blob, objText, opts || {}); }

module.exports = { HipRenderer, NodePixelBuffer, addon, readHeader, attachObj, deviceForWorker, ABI_VERSION };
