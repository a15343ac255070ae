"use strict";
/*
 * scene_blob.js — host-side scene exporter for the drop-in boundary.
 *
 * Walks the reference's LIVE scene graph ({renderer, width, height} as produced by a test's
 * configureTest, e.g. tests/cornell_box_path/test.mjs:77-81) and writes the "JSRT" v1 binary blob
 * defined in include/jsrt_scene.h.  It replaces the role src/serializer.js:12-60 plays for the
 * worker path, without its lossy cases (Triangle.serialize drops vertex normals,
 * geometry.js:355-357; PhongPathTracingMaterial.deserialize builds a Fresnel material,
 * materials.js:394-396; Infinity -> JSON null).
 *
 * Class lookup is by name in the global scope of the realm the reference's src/*.js were loaded
 * into (importScripts in src/worker.js:3-14, or vm.runInThisContext under Node), so this file
 * imports nothing from the reference.
 */

const SEC = {};
function fourcc(s) { return s.charCodeAt(0) | (s.charCodeAt(1) << 8) | (s.charCodeAt(2) << 16) | (s.charCodeAt(3) << 24) >>> 0; }
for (const t of ["RNDR", "CAMR", "MCOL", "MATL", "GEOM", "OBJS", "MATS", "ROOT", "CHLD", "BVHN", "TRIS", "LITE", "SDFN", "SDFG"])
    SEC[t] = fourcc(t) >>> 0;

const K = {
    RENDERER_SIMPLE: 0, RENDERER_INCREMENTAL: 1, RENDERER_RANDOM: 2,
    CAMERA_PERSPECTIVE: 0, CAMERA_DOF: 1,
    MC_SOLID: 1, MC_SCALED_SCALAR: 2, MC_SCALED_VEC: 3, MC_CHECKER: 4,
    MAT_PHONG: 1, MAT_FRESNEL: 2, MAT_PATH: 3, MAT_SOLID: 4, MAT_TRANSPARENT: 5,
    GEOM_PLANE: 1, GEOM_SQUARE: 2, GEOM_CIRCLE: 3, GEOM_SPHERE: 4, GEOM_CYLINDER: 5, GEOM_AABB: 6,
    GEOM_TRIANGLE: 7, GEOM_SDF: 8,
    OBJ_PRIMITIVE: 1, OBJ_AGGREGATE: 2, OBJ_BVH: 3, OBJ_TRANSFORMED: 4,
    LIGHT_POINT: 1, LIGHT_AREA: 2,
    SDF_UNION: 1, SDF_INTERSECTION: 2, SDF_DIFFERENCE: 3, SDF_SMOOTH_UNION: 4, SDF_SMOOTH_INTERSECTION: 5,
    SDF_SMOOTH_DIFFERENCE: 6, SDF_ROUND: 7, SDF_SPHERE: 8, SDF_BOX: 9, SDF_TETRAHEDRON: 10,
    SDF_TRANSFORM: 11, SDF_RECURSIVE_UNION: 12,
    SDFT_SEQUENCE: 20, SDFT_RECURSIVE: 21, SDFT_MATRIX: 22, SDFT_REFLECTION: 23, SDFT_REPETITION: 24,
};

const REC_SIZE = { RNDR: 48, CAMR: 168, MCOL: 40, MATL: 64, GEOM: 48, OBJS: 32, MATS: 256, ROOT: 4, CHLD: 4,
                   BVHN: 64, TRIS: 256, LITE: 304, SDFN: 336, SDFG: 64 };

function cls(name) {
    try { return (0, eval)(name); } catch (e) { return undefined; }
}
function isA(obj, name) {
    const C = cls(name);
    return C !== undefined && obj instanceof C;
}

// A little record writer: each record is written field by field into a DataView at known offsets.
class Rec {
    constructor(size) { this.buf = new ArrayBuffer(size); this.dv = new DataView(this.buf); }
    u32(off, v) { this.dv.setUint32(off, v >>> 0, true); return this; }
    i32(off, v) { this.dv.setInt32(off, v | 0, true); return this; }
    f32(off, v) { this.dv.setFloat32(off, v, true); return this; }
    f64(off, v) { this.dv.setFloat64(off, v, true); return this; }
    vec(off, v, n = 4) { // copies Vec (Float32Array) bits; missing components 0
        for (let i = 0; i < n; ++i) this.f32(off + 4 * i, (v && i < v.length) ? v[i] : 0);
        return this;
    }
    mat(off, m) { // Mat rows (float64), 4x4 row-major
        for (let r = 0; r < 4; ++r) for (let c = 0; c < 4; ++c) this.f64(off + 8 * (4 * r + c), m[r][c]);
        return this;
    }
}

function assertVec(v, what) {
    if (!(v instanceof Float32Array)) throw "scene_blob: " + what + " is not a Vec";
    if (v.length > 4) throw "scene_blob: " + what + " has length " + v.length;
    return v;
}
function asF32Vec(v, what) {
    if (v instanceof Float32Array) return assertVec(v, what);
    if (v instanceof Array) {
        const f = Float32Array.from(v);
        for (let i = 0; i < v.length; ++i)
            if (!Object.is(f[i], v[i])) throw "scene_blob: " + what + " has non-f32 entries";
        return f;
    }
    throw "scene_blob: " + what + " is not a vector";
}

class SceneBlobWriter {
    constructor() {
        this.sec = {};
        for (const t of Object.keys(REC_SIZE)) this.sec[t] = [];
        this.maps = { mc: new Map(), mat: new Map(), geom: new Map(), obj: new Map(), bvh: new Map(), matrix: new Map(),
                      matrixBytes: new Map(), sdf: new Map(), sdfgeom: new Map() };
    }
    push(tag, rec) { this.sec[tag].push(rec); return this.sec[tag].length - 1; }

    matrixIndex(m, inv) {
        const key1 = this.maps.matrix.get(m);
        if (key1 && key1.has(inv)) return key1.get(inv);
        const r = new Rec(256).mat(0, m).mat(128, inv);
        const bytesKey = Buffer.from(r.buf).toString("base64");
        let idx = this.maps.matrixBytes.get(bytesKey);
        if (idx === undefined) {
            idx = this.push("MATS", r);
            this.maps.matrixBytes.set(bytesKey, idx);
        }
        if (!key1) this.maps.matrix.set(m, new Map([[inv, idx]]));
        else key1.set(inv, idx);
        return idx;
    }

    mcIndex(mc) {
        if (mc === undefined || mc === null) return -1;
        if (this.maps.mc.has(mc)) return this.maps.mc.get(mc);
        const r = new Rec(40);
        if (isA(mc, "SolidMaterialColor")) {
            const v = assertVec(mc._color, "SolidMaterialColor._color");
            r.u32(0, K.MC_SOLID).i32(4, -1).i32(8, -1).u32(12, v.length).vec(16, v);
        } else if (isA(mc, "ScaledMaterialColor")) {
            const a = this.mcIndex(mc._mc);
            if (typeof mc._scale === "number")
                r.u32(0, K.MC_SCALED_SCALAR).i32(4, a).i32(8, -1).u32(12, 0).f64(32, mc._scale);
            else {
                const v = asF32Vec(mc._scale, "ScaledMaterialColor._scale");
                r.u32(0, K.MC_SCALED_VEC).i32(4, a).i32(8, -1).u32(12, v.length).vec(16, v);
            }
        } else if (isA(mc, "CheckerboardMaterialColor")) {
            r.u32(0, K.MC_CHECKER).i32(4, this.mcIndex(mc.color1)).i32(8, this.mcIndex(mc.color2));
        } else
            throw "scene_blob: unsupported MaterialColor " + (mc.constructor && mc.constructor.name);
        const idx = this.push("MCOL", r);
        this.maps.mc.set(mc, idx);
        return idx;
    }

    matIndex(m) {
        if (this.maps.mat.has(m)) return this.maps.mat.get(m);
        const r = new Rec(64);
        let kind;
        if (isA(m, "PhongPathTracingMaterial")) kind = K.MAT_PATH;
        else if (isA(m, "FresnelPhongMaterial")) kind = K.MAT_FRESNEL;
        else if (isA(m, "PhongMaterial")) kind = K.MAT_PHONG;
        else if (isA(m, "SolidColorMaterial")) kind = K.MAT_SOLID;
        else if (isA(m, "TransparentMaterial")) kind = K.MAT_TRANSPARENT;
        else throw "scene_blob: unsupported Material " + (m && m.constructor && m.constructor.name);
        r.u32(0, kind);
        for (let i = 1; i < 8; ++i) r.i32(4 * i, -1);
        if (kind === K.MAT_SOLID || kind === K.MAT_TRANSPARENT) {
            r.i32(28, this.mcIndex(m._color));
            r.f64(56, kind === K.MAT_TRANSPARENT ? m._opacity : 0);
        } else {
            r.i32(4, this.mcIndex(m.baseColor)).i32(8, this.mcIndex(m.ambient)).i32(12, this.mcIndex(m.diffusivity))
             .i32(16, this.mcIndex(m.specularity)).i32(20, this.mcIndex(m.reflectivity))
             .i32(24, this.mcIndex(m.transmissivity));
            r.f64(32, m.smoothness);
            r.f64(40, kind === K.MAT_PHONG ? 1 : m.refractiveIndexRatio);
            r.f64(48, kind === K.MAT_PATH ? m.mirrorProbability : 0);
        }
        const idx = this.push("MATL", r);
        this.maps.mat.set(m, idx);
        return idx;
    }

    triIndex(t) {
        const r = new Rec(256);
        for (let k = 0; k < 3; ++k) r.vec(16 * k, assertVec(t.ps[k], "Triangle.ps"));
        if (t.ps.some(p => p.length !== 4)) throw "scene_blob: Triangle vertices must be 4-vectors";
        r.vec(48, t.v0).vec(64, t.v1).vec(80, t.normal);
        r.f64(96, t.delta).f64(104, t.d00).f64(112, t.d11).f64(120, t.d01).f64(128, t.denom).f64(136, t.area);
        const pd = t.psdata || {};
        for (const k of Object.keys(pd))
            if (k !== "normal" && k !== "UV") throw "scene_blob: unsupported Triangle psdata key " + k;
        if (pd.normal) {
            r.u32(144, 1);
            for (let k = 0; k < 3; ++k) r.vec(160 + 16 * k, assertVec(pd.normal[k], "Triangle normal"));
            if (pd.normal.some(v => v.length !== 4)) throw "scene_blob: vertex normals must be 4-vectors";
        }
        if (pd.UV) {
            r.u32(148, 1).u32(152, pd.UV[0].length);
            for (let k = 0; k < 3; ++k) r.vec(208 + 16 * k, assertVec(pd.UV[k], "Triangle UV"));
        }
        return this.push("TRIS", r);
    }

    geomIndex(g) {
        if (this.maps.geom.has(g)) return this.maps.geom.get(g);
        const r = new Rec(48);
        if (isA(g, "AABB")) // includes UnitBox (geometry.js:230)
            r.u32(0, K.GEOM_AABB).vec(16, assertVec(g.center, "AABB.center")).vec(32, assertVec(g.half_size, "AABB.half"));
        else if (isA(g, "Square")) r.u32(0, K.GEOM_SQUARE);
        else if (isA(g, "Circle")) r.u32(0, K.GEOM_CIRCLE);
        else if (isA(g, "SimplePlane")) r.u32(0, K.GEOM_PLANE); // SimplePlane and Plane
        else if (isA(g, "Sphere")) r.u32(0, K.GEOM_SPHERE);
        else if (isA(g, "Cylinder")) r.u32(0, K.GEOM_CYLINDER);
        else if (isA(g, "Triangle")) r.u32(0, K.GEOM_TRIANGLE).i32(4, this.triIndex(g));
        else if (isA(g, "SDFGeometry")) r.u32(0, K.GEOM_SDF).i32(4, this.sdfGeomIndex(g));
        else throw "scene_blob: unsupported Geometry " + (g && g.constructor && g.constructor.name);
        const idx = this.push("GEOM", r);
        this.maps.geom.set(g, idx);
        return idx;
    }

    sdfGeomIndex(g) {
        if (this.maps.sdfgeom.has(g)) return this.maps.sdfgeom.get(g);
        const r = new Rec(64);
        r.i32(0, this.sdfIndex(g.root_sdf)).i32(4, g.max_samples);
        r.f64(8, g.distance_epsilon).f64(16, g.max_trace_distance).f64(24, g.normal_step_size);
        r.vec(32, assertVec(g.aabb.center, "SDF aabb")).vec(48, assertVec(g.aabb.half_size, "SDF aabb"));
        const idx = this.push("SDFG", r);
        this.maps.sdfgeom.set(g, idx);
        return idx;
    }

    sdfList(list) {
        const idx = list.map(c => this.sdfIndex(c));
        const first = this.sec.CHLD.length;
        for (const i of idx) this.push("CHLD", new Rec(4).i32(0, i));
        return [first, idx.length];
    }

    sdfIndex(s) {
        if (this.maps.sdf.has(s)) return this.maps.sdf.get(s);
        const r = new Rec(336);
        r.i32(4, -1).i32(8, -1).i32(12, -1).i32(16, 0).i32(20, 0);
        const bc = (v) => { const b = assertVec(v || Float32Array.of(1, 1, 1), "basecolor"); r.vec(48, b).u32(64, b.length); };
        if (isA(s, "UnionSDF") || isA(s, "IntersectionSDF")) {
            const [f, n] = this.sdfList(s.children);
            r.u32(0, isA(s, "UnionSDF") ? K.SDF_UNION : K.SDF_INTERSECTION).i32(12, f).i32(16, n);
        } else if (isA(s, "DifferenceSDF"))
            r.u32(0, K.SDF_DIFFERENCE).i32(4, this.sdfIndex(s.positive)).i32(8, this.sdfIndex(s.negative));
        else if (isA(s, "SmoothUnionSDF") || isA(s, "SmoothIntersectionSDF"))
            r.u32(0, isA(s, "SmoothUnionSDF") ? K.SDF_SMOOTH_UNION : K.SDF_SMOOTH_INTERSECTION)
             .i32(4, this.sdfIndex(s.childA)).i32(8, this.sdfIndex(s.childB)).f64(24, s.k);
        else if (isA(s, "SmoothDifferenceSDF"))
            r.u32(0, K.SDF_SMOOTH_DIFFERENCE).i32(4, this.sdfIndex(s.positive)).i32(8, this.sdfIndex(s.negative)).f64(24, s.k);
        else if (isA(s, "RoundSDF"))
            r.u32(0, K.SDF_ROUND).i32(4, this.sdfIndex(s.child_sdf)).f64(24, s.rounding);
        else if (isA(s, "SphereSDF")) { r.u32(0, K.SDF_SPHERE).f64(24, s.radius); bc(s.basecolor); }
        else if (isA(s, "BoxSDF")) { r.u32(0, K.SDF_BOX).vec(32, assertVec(s.size, "BoxSDF.size")); bc(s.basecolor); }
        else if (isA(s, "TetrahedronSDF")) { r.u32(0, K.SDF_TETRAHEDRON); bc(s.basecolor); }
        else if (isA(s, "TransformSDF"))
            r.u32(0, K.SDF_TRANSFORM).i32(4, this.sdfIndex(s.child_sdf)).i32(8, this.sdfIndex(s.transformer));
        else if (isA(s, "RecursiveTransformUnionSDF"))
            r.u32(0, K.SDF_RECURSIVE_UNION).i32(4, this.sdfIndex(s.sdf)).i32(8, this.sdfIndex(s.transformer)).i32(20, s.iterations);
        else if (isA(s, "SDFTransformerSequence")) {
            const [f, n] = this.sdfList(s.transformers);
            r.u32(0, K.SDFT_SEQUENCE).i32(12, f).i32(16, n);
        } else if (isA(s, "SDFRecursiveTransformer"))
            r.u32(0, K.SDFT_RECURSIVE).i32(4, this.sdfIndex(s.transformer)).i32(20, s.iterations);
        else if (isA(s, "SDFMatrixTransformer"))
            r.u32(0, K.SDFT_MATRIX).f64(24, s._scale).mat(80, s._transform).mat(208, s._inv_transform);
        else if (isA(s, "SDFReflectionTransformer"))
            r.u32(0, K.SDFT_REFLECTION).f64(24, s.delta).vec(32, assertVec(s.normal, "reflection normal"));
        else if (isA(s, "SDFInfiniteRepetitionTransformer"))
            r.u32(0, K.SDFT_REPETITION).vec(32, assertVec(s.sizes, "repetition sizes"));
        else throw "scene_blob: unsupported SDF node " + (s && s.constructor && s.constructor.name);
        // record the node before returning so shared subtrees map to one index
        const idx = this.push("SDFN", r);
        this.maps.sdf.set(s, idx);
        return idx;
    }

    bvhIndex(node) {
        // `new BVHAggregate(objs, other.kdtree, T)` instances share one tree (tests/starwars/test.mjs)
        if (this.maps.bvh.has(node)) return this.maps.bvh.get(node);
        const r = new Rec(64);
        const idx = this.push("BVHN", r);
        this.maps.bvh.set(node, idx);
        r.vec(0, assertVec(node.aabb.center, "BVH aabb")).vec(16, assertVec(node.aabb.half_size, "BVH aabb"));
        r.u32(32, node.isLeaf ? 1 : 0).i32(36, -1).i32(40, -1).i32(44, 0).i32(48, 0).i32(52, node.depth);
        if (node.isLeaf) {
            const ids = node.objects.map(o => this.objIndex(o));
            r.i32(44, this.sec.CHLD.length).i32(48, ids.length);
            for (const i of ids) this.push("CHLD", new Rec(4).i32(0, i));
        } else {
            r.i32(36, this.bvhIndex(node.lesser_node));
            r.i32(40, this.bvhIndex(node.greater_node));
        }
        return idx;
    }

    objIndex(o) {
        if (this.maps.obj.has(o)) return this.maps.obj.get(o);
        const r = new Rec(32);
        r.i32(4, -1).i32(8, -1).i32(16, -1).i32(20, 0).i32(24, -1);
        r.i32(28, this.matrixIndex(o.transform, o.inv_transform));
        if (isA(o, "Primitive")) {
            r.u32(0, K.OBJ_PRIMITIVE).i32(4, this.geomIndex(o.geometry)).i32(8, this.matIndex(o.material))
             .u32(12, o.does_cast_shadow ? 1 : 0);
        } else if (isA(o, "BVHAggregate")) {
            r.u32(0, K.OBJ_BVH).i32(24, this.bvhIndex(o.kdtree));
        } else if (isA(o, "Aggregate")) {
            const ids = o.objects.map(c => this.objIndex(c));
            r.u32(0, K.OBJ_AGGREGATE).i32(16, this.sec.CHLD.length).i32(20, ids.length);
            for (const i of ids) this.push("CHLD", new Rec(4).i32(0, i));
        } else if (isA(o, "TransformedWorldObject")) {
            const c = this.objIndex(o.object);
            r.u32(0, K.OBJ_TRANSFORMED).i32(16, this.sec.CHLD.length).i32(20, 1);
            this.push("CHLD", new Rec(4).i32(0, c));
        } else throw "scene_blob: unsupported WorldObject " + (o && o.constructor && o.constructor.name);
        const idx = this.push("OBJS", r);
        this.maps.obj.set(o, idx);
        return idx;
    }

    light(l) {
        const r = new Rec(304);
        r.i32(4, this.mcIndex(l.color_mc));
        if (isA(l, "SimplePointLight")) {
            const p = assertVec(l.position, "light position");
            r.u32(0, K.LIGHT_POINT).u32(12, 1).vec(16, p).u32(32, p.length);
        } else if (isA(l, "RandomSampleAreaLight")) {
            const g = l.surface_geometry;
            let gk;
            if (isA(g, "Square")) gk = K.GEOM_SQUARE;
            else if (isA(g, "Circle")) gk = K.GEOM_CIRCLE;
            else if (isA(g, "Sphere")) gk = K.GEOM_SPHERE;
            else throw "scene_blob: unsupported area-light geometry " + (g && g.constructor && g.constructor.name);
            r.u32(0, K.LIGHT_AREA).u32(8, gk).u32(12, l.samples).mat(48, l.transform).mat(176, l.inv_transform);
        } else throw "scene_blob: unsupported Light " + (l && l.constructor && l.constructor.name);
        this.push("LITE", r);
    }

    // test: {renderer, width, height}; over: optional {width, height, spp, kind, maxDepth}
    build(test, over = {}) {
        const R = test.renderer;
        let kind = K.RENDERER_SIMPLE;
        if (isA(R, "IncrementalMultisamplingRenderer")) kind = K.RENDERER_INCREMENTAL;
        else if (isA(R, "RandomMultisamplingRenderer")) kind = K.RENDERER_RANDOM;
        if (over.kind !== undefined) kind = over.kind;
        const spp = over.spp !== undefined ? over.spp : (R.samplesPerPixel || 1);
        const depth = over.maxDepth !== undefined ? over.maxDepth : R.maxRecursionDepth;
        const W = over.width !== undefined ? over.width : test.width;
        const H = over.height !== undefined ? over.height : test.height;
        const bg = assertVec(R.world.bg_color, "bg_color");
        const rr = new Rec(48);
        rr.u32(0, kind).u32(4, spp).u32(8, depth).u32(12, W).u32(16, H).u32(20, bg.length).vec(24, bg);
        this.push("RNDR", rr);

        const C = R.camera;
        const cr = new Rec(168);
        const dof = isA(C, "DepthOfFieldPerspectiveCamera");
        if (!dof && !isA(C, "PerspectiveCamera")) throw "scene_blob: unsupported camera";
        cr.u32(0, dof ? K.CAMERA_DOF : K.CAMERA_PERSPECTIVE).mat(8, C.transform).f64(136, C.tan_fov).f64(144, C.aspect);
        if (dof) cr.f64(152, C.focus_distance).f64(160, C.sensor_size);
        this.push("CAMR", cr);

        for (const o of R.world.objects) this.push("ROOT", new Rec(4).i32(0, this.objIndex(o)));
        for (const l of R.world.lights) this.light(l);
        return this.serialize();
    }

    serialize() {
        const tags = Object.keys(REC_SIZE);
        const header = 16 + 24 * tags.length;
        let off = (header + 7) & ~7;
        const descs = [];
        for (const t of tags) {
            const bytes = this.sec[t].length * REC_SIZE[t];
            descs.push([t, this.sec[t].length, off, bytes]);
            off += (bytes + 7) & ~7;
        }
        const out = Buffer.alloc(off);
        out.writeUInt32LE(0x5452534A, 0);
        out.writeUInt32LE(1, 4);
        out.writeUInt32LE(tags.length, 8);
        out.writeUInt32LE(0, 12);
        descs.forEach(([t, n, o, b], i) => {
            const p = 16 + 24 * i;
            out.writeUInt32LE(SEC[t], p);
            out.writeUInt32LE(n, p + 4);
            out.writeBigUInt64LE ? out.writeBigUInt64LE(BigInt(o), p + 8) : out.writeUInt32LE(o, p + 8);
            out.writeBigUInt64LE ? out.writeBigUInt64LE(BigInt(b), p + 16) : out.writeUInt32LE(b, p + 16);
            let q = o;
            for (const rec of this.sec[t]) { Buffer.from(rec.buf).copy(out, q); q += REC_SIZE[t]; }
        });
        return out;
    }
}

function exportScene(test, overrides = {}) {
    return new SceneBlobWriter().build(test, overrides);
}

if (typeof module !== "undefined")
    module.exports = { exportScene, SceneBlobWriter, K, SEC };
