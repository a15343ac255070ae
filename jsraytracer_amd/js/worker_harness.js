"use strict";
/*
 * worker_harness.js — Node stand-in for the reference's browser worker host (src/worker.js:17-40,
 * src/raytrace_launcher.js:65-101) driving HipRenderer instead of the CPU renderers.
 *
 *   node worker_harness.js <scene.jsrt[.gz]> <workers> [out.rgba] [width height spp seed]
 *
 * Spawns <workers> worker_threads.  Each gets the reference's message [scenePath, workerIndex,
 * workerCount], takes GPU workerIndex % deviceCount (hip_renderer.js deviceForWorker), renders its
 * interleaved columns (x_offset = workerIndex, x_delt = workerCount) with
 * renderer.render(buffer, 1000, cb, workerIndex, workerCount) and posts [ImageData, workerIndex,
 * stats|null] ... then ["finished", workerIndex, null], exactly the reference protocol.  The main
 * thread composites like raytrace_launcher.js:92-97 (untouched pixels have alpha 0, so overlaying
 * every worker's full frame yields the image) and writes the RGBA8 bytes.
 */
const fs = require("fs");
const zlib = require("zlib");
const { Worker, isMainThread, parentPort, workerData } = require("worker_threads");
const { HipRenderer, NodePixelBuffer, deviceForWorker } = require("./hip_renderer");

function loadBlob(p) {
    let b = fs.readFileSync(p);
    if (p.endsWith(".gz")) b = zlib.gunzipSync(b);
    return new Uint8Array(b.buffer, b.byteOffset, b.byteLength);
}

if (!isMainThread) {
    parentPort.on("message", (msg) => {
        const [scenePath, workerIndex, workerCount] = msg;
        const o = workerData.overrides || {};
        // worker i on GPU i % deviceCount: the reference's workers spread over the node's GPUs
        const device = deviceForWorker(workerIndex);
        const renderer = new HipRenderer(loadBlob(scenePath), Object.assign({}, o, { device }));
        const W = o.width || renderer.width || 600, H = o.height || 600;
        const buffer = new NodePixelBuffer(W, H);
        const t0 = Date.now();
        renderer.render(buffer, 1000, (stats) => parentPort.postMessage([buffer.imgdata, workerIndex, stats]),
                        workerIndex, workerCount);
        parentPort.postMessage([buffer.imgdata, workerIndex, null]);
        parentPort.postMessage(["finished", workerIndex, { ms: Date.now() - t0, gpu: renderer.stats, device }]);
        renderer.destroy();
    });
} else {
    const [scenePath, nw = "1", out, w, h, spp, seed] = process.argv.slice(2);
    const N = parseInt(nw, 10);
    const overrides = {};
    if (w) overrides.width = parseInt(w, 10);
    if (h) overrides.height = parseInt(h, 10);
    if (spp) overrides.samplesPerPixel = parseInt(spp, 10);
    if (seed) overrides.seed = parseInt(seed, 10);
    const W = overrides.width || 600, H = overrides.height || 600;
    const composite = new Uint8ClampedArray(W * H * 4);
    let finished = 0;
    for (let i = 0; i < N; ++i) {
        const wk = new Worker(__filename, { workerData: { overrides } });
        wk.on("error", (e) => { console.error("worker", i, "failed:", e); process.exitCode = 1; });
        wk.on("message", ([img, idx, stats]) => {
            if (img === "finished") {
                console.error(`worker ${idx} on device ${stats.device} finished in ${stats.ms / 1000} s`);
                wk.terminate();
                if (++finished === N && out) fs.writeFileSync(out, Buffer.from(composite.buffer));
                return;
            }
            for (let k = 0; k < W * H; ++k)  // drawImage overlay: alpha-0 pixels are transparent
                if (img.data[4 * k + 3]) for (let c = 0; c < 4; ++c) composite[4 * k + c] = img.data[4 * k + c];
        });
        wk.postMessage([scenePath, i, N]);
    }
}
