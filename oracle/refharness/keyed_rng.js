"use strict";
/*
 * TEST INFRASTRUCTURE ONLY.  Deterministic, tree-addressed replacement for Math.random inside the
 * reference renderer (SURVEY.md §8c).  The reference draws from the unseeded global Math.random
 * (renderers.js:57-58,95-96; math.js:176-177,181-182; geometry.js:297-298,328-329;
 * materials.js:399,408,450,462), so parity with ANY other implementation requires substituting a
 * generator whose value depends only on *where* in the computation a draw happens:
 *
 *   key  = (seed, pixel = py*W + px, sample, node, call)
 *   node = ray-tree address of the World.color frame that is active when the draw happens:
 *          the pre-root frame has address 0 (it owns the camera jitter / DOF draws);
 *          each World.color call opens child = mix(parent.addr, ++parent.kids)  (depth-0 calls too)
 *   call = per-frame draw counter, in program order.
 *   h    = mix(mix(mix(mix(seed, pixel), sample), node), call)
 *   u    = ((mix(h, 0xA5A5A5A5) >>> 5) * 2^26 + (mix(h, 0x5A5A5A5A) >>> 6)) / 2^53   (53-bit double)
 *   mix(h, v): h = imul(h ^ v, 0x9E3779B1); h ^= h >>> 15; h = imul(h, 0x85EBCA77); h ^= h >>> 13
 *
 * The (pixel, sample) key advances after each root World.color returns, following the loop order of
 * the renderer in use (SimpleRenderer px-major renderers.js:21-23; Incremental iter-major
 * renderers.js:87-90; RandomMultisampling pixel-major with spp inner renderers.js:54).
 * Identical definitions: oracle/jsrt_oracle.c (jsrt_rng_*) and the HIP kernel (jsraytracer_amd/csrc).
 */

function mix(h, v) {
    h = Math.imul((h ^ v) | 0, 0x9E3779B1 | 0);
    h ^= h >>> 15;
    h = Math.imul(h, 0x85EBCA77 | 0);
    h ^= h >>> 13;
    return h >>> 0;
}

function keyedUniform(seed, pixel, sample, node, call) {
    const h = mix(mix(mix(mix(seed >>> 0, pixel >>> 0), sample >>> 0), node >>> 0), call >>> 0);
    const hi = mix(h, 0xA5A5A5A5 | 0) >>> 5;   // 27 bits
    const lo = mix(h, 0x5A5A5A5A | 0) >>> 6;   // 26 bits
    return (hi * 67108864 + lo) / 9007199254740992;
}

// Installs the keyed RNG + ray-tree addressing on the loaded reference classes.
// Returns a controller used by the golden renderer to set the sample sequence.
function installKeyedRng(seed) {
    const World = (0, eval)("World");
    const origColor = World.prototype.__jsrt_orig_color || World.prototype.color;
    World.prototype.__jsrt_orig_color = origColor;

    const ctl = {
        seed: seed >>> 0,
        stack: [{ addr: 0, calls: 0, kids: 0 }],
        seq: null,        // iterator of [pixel, sample]
        cur: [0, 0],
        draws: 0,
        colorCalls: 0,
        startSequence(iter) { this.seq = iter; this.advance(); },
        advance() {
            this.stack = [{ addr: 0, calls: 0, kids: 0 }];
            if (!this.seq) return;
            const n = this.seq.next();
            this.cur = n.done ? [0xFFFFFFFF, 0xFFFFFFFF] : n.value;
        },
    };

    World.prototype.color = function (ray, depth, minDistance) {
        const parent = ctl.stack[ctl.stack.length - 1];
        const frame = { addr: mix(parent.addr, ++parent.kids), calls: 0, kids: 0 };
        ctl.stack.push(frame);
        ctl.colorCalls++;
        let ret;
        try {
            ret = origColor.call(this, ray, depth, minDistance);
        } finally {
            ctl.stack.pop();
        }
        if (ctl.stack.length === 1) ctl.advance();
        return ret;
    };
    Math.random = function () {
        const f = ctl.stack[ctl.stack.length - 1];
        ctl.draws++;
        return keyedUniform(ctl.seed, ctl.cur[0], ctl.cur[1], f.addr, f.calls++);
    };
    return ctl;
}

// The (pixel, sample) order in which each renderer kind issues root World.color calls.
function* sampleOrder(kind, W, H, spp, x_offset = 0, x_delt = 1) {
    if (kind === 1) { // Incremental: renderers.js:87-90
        for (let it = 0; it < spp; ++it)
            for (let px = x_offset; px < W; px += x_delt)
                for (let py = 0; py < H; ++py) yield [py * W + px, it];
    } else if (kind === 2) { // RandomMultisampling: renderers.js:21-26 + :54
        for (let px = x_offset; px < W; px += x_delt)
            for (let py = 0; py < H; ++py)
                for (let s = 0; s < spp; ++s) yield [py * W + px, s];
    } else { // Simple: renderers.js:21-26
        for (let px = x_offset; px < W; px += x_delt)
            for (let py = 0; py < H; ++py) yield [py * W + px, 0];
    }
}

module.exports = { mix, keyedUniform, installKeyedRng, sampleOrder };
