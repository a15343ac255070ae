// render.hip — wavefront (breadth-first) evaluation of the reference's ray tree on MI355X.
//
// The reference evaluates World.color recursively, depth first (world.js:31-41 ->
// materials.js:271-333).  Two facts make a breadth-first schedule produce bit-identical results:
//   1. every random draw is keyed by the ray-tree address of its World.color frame
//      (DESIGN.md §2.3), never by global call order;
//   2. the only cross-node arithmetic is surface.plus(child.times(col).times(w).times(k)) in child
//      order, which k_reduce performs bottom-up with the same f32 roundings.
// So each kernel processes one bounce level of ALL paths of a batch:
//   k_gen      camera rays (renderers.js:95-96 jitter, cameras.js:29-52)                -> level 0
//   k_extend   closest hit per ray (World.cast, world.js:28-30), culled world loop
//   k_shade    Primitive.color + materialData + getBaseFactors + light samples + scatter;
//              children appended to the next level with wave-aggregated atomics
//   k_shadow   the shadow casts of a node's light samples + colorFromLights' sums
//   k_reduce   levels deepest -> 0: surface + children, into the parent's child slot
//   k_accum    per pixel, samples in order: the renderer's f32 accumulation
//   k_final    running mean + PixelBuffer.setColor rules -> RGBA8 (+ f32 colour)
// Every kernel is small and converged (all lanes run the same stage) with its own register
// budget; batches are (pixels x samples) with ray SoA buffers in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "device_common.h"
#include "render_kernel.h"

#ifndef JSRT_SHADE_OCC  // min waves per SIMD requested for k_shade (register budget)
#define JSRT_SHADE_OCC 2
#endif
#ifndef JSRT_SHADOW_OCC
#define JSRT_SHADOW_OCC 1
#endif
#ifndef JSRT_EXTEND_OCC
#define JSRT_EXTEND_OCC 1
#endif

namespace jsrt {

const char *const KT_NAMES[KT_N] = {"k_gen", "k_extend", "k_shade", "k_shadow", "k_reduce", "k_accum", "k_final",
                                    "k_lightsum"};
constexpr uint32_t NO_PARENT = 0xFFFFFFFFu;  // camera ray: its result is the path's root colour
constexpr uint32_t DEAD_RAY = 0xFFFFFFFEu;   // level-0 slot of a path outside the image (no result)

// block-aggregated append (one atomic per block: same-address atomics serialise device-wide).
// Every thread of the block must call it.
template <int NT>
__device__ __forceinline__ uint32_t block_append(uint32_t *counter, int n) {
    constexpr int NW = NT / 64;
    __shared__ uint32_t s_off[NW + 1];
    const uint64_t b1 = __ballot(n >= 1), b2 = __ballot(n >= 2);
    const int lane = (int)__lane_id(), wid = (int)(threadIdx.x >> 6);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t pre = (uint32_t)(__popcll(b1 & lt) + __popcll(b2 & lt));
    if (lane == 0) s_off[wid] = (uint32_t)(__popcll(b1) + __popcll(b2));
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = s_off[w];
            s_off[w] = acc;
            acc += c;
        }
        s_off[NW] = acc ? atomicAdd(counter, acc) : 0u;
    }
    __syncthreads();
    return s_off[NW] + s_off[wid] + pre;
}

__device__ __forceinline__ void write_result(const WArgs &W, uint32_t i, F3 c) {
    const uint32_t p = W.parent[i];
    if (p == DEAD_RAY) return;
    float *dst = (p == NO_PARENT) ? W.root + 3 * (size_t)W.path[i] : W.slot + 3 * (size_t)p;
    dst[0] = c.x;
    dst[1] = c.y;
    dst[2] = c.z;
}

// patch-ordered owned pixel index -> (owned column c, row py, image column px)
__device__ __forceinline__ bool pixel_of(const RenderArgs &A, uint32_t p, int &c, int &py, int &px) {
    const int patch = (int)(p >> 6), lane = (int)(p & 63);
    c = (patch % A.patches_x) * 8 + (lane & 7);
    py = (patch / A.patches_x) * 8 + (lane >> 3);
    if (c >= A.ncols || py >= A.H) return false;
    px = owned_to_px(c, A.x_offset, A.x_delt, A.col_block);
    return px < A.W;
}

__device__ __forceinline__ F3 pick(bool f, F3 a, F3 b) { return f3(f ? a.x : b.x, f ? a.y : b.y, f ? a.z : b.z); }
__device__ __forceinline__ Child pick(bool f, const Child &a, const Child &b) {
    return Child{pick(f, a.dir, b.dir), pick(f, a.col, b.col), pick(f, a.w, b.w), f ? a.k : b.k};
}

// World.color hit branch up to the shadow casts: Primitive.color (world.js:125-137) +
// Geometry.materialData + Material.color (materials.js).  Writes the node (info, ambient / surface,
// shadow hand-off of its light samples) and returns its children (0..2) in evaluation order.
template <int PF>
__device__ __forceinline__ int shade_node(const DScene &S, const WArgs &W, uint32_t i, uint32_t tt, const Hit &h, F3 o, F3 d,
                          uint32_t addr, uint32_t key, Child &ch0, Child &ch1, F3 &pos) {
    const DPrim &P = S.prims[h.prim];
    // inv_transform = prim.inv x ancestorInvTransform (float64, math.js:399-409); the host
    // precomputed it (same operations) for identity prims and for the top-level context
    double inv[16];
    {
        const int ps = S.prim_shade[h.prim];
        if (ps < 0 || h.ctx == 0) {
            const double *src = ps < 0 ? S.shadeI + 16 * h.ctx : S.shade0 + 16 * ps;
#pragma unroll
            for (int k = 0; k < 16; ++k) inv[k] = src[k];
        } else {
            const double *C = S.ctx + 16 * h.ctx;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const double a0 = r < 3 ? P.inv[4 * r + 0] : 0.0, a1 = r < 3 ? P.inv[4 * r + 1] : 0.0,
                                 a2 = r < 3 ? P.inv[4 * r + 2] : 0.0, a3 = r < 3 ? P.inv[4 * r + 3] : 1.0;
                    double s = 0;
                    s += a0 * C[c];
                    s += a1 * C[4 + c];
                    s += a2 * C[8 + c];
                    s += a3 * C[12 + c];
                    inv[4 * r + c] = s;
                }
        }
    }
    const bool need_uv = (S.mat_flags[P.material] & MATF_UV) != 0;
    const F3 lo = xf_point(inv, o), ld = xf_dir(inv, d);
    const F3 pl = ray_point(lo, ld, h.t);  // base_data.position (local)
    F3 nrm = f3(0, 0, 0);
    float nrm_w = 0.0f;
    float u = 0, v = 0;
    F3 basecolor = f3(1, 1, 1);
    switch (P.gkind) {
    case JSRT_GEOM_PLANE:
    case JSRT_GEOM_SQUARE:
    case JSRT_GEOM_CIRCLE:  // SimplePlane.materialData (geometry.js:249-254)
        nrm = f3(0, 0, 1);
        u = pl.x;
        v = pl.y;
        break;
    case JSRT_GEOM_SPHERE: {  // geometry.js:449-455: position.normalized() includes w = 1
        const double nn = sqrt(dot3(pl, pl) + 1.0);
        nrm = pl;
        nrm_w = 1.0f;
        if (nn > 0.00001) { nrm = scale(pl, 1 / nn); nrm_w = (float)(1.0 * (1 / nn)); }
        if (need_uv) cart_to_sph(nrm, u, v);
        break;
    }
    case JSRT_GEOM_CYLINDER:  // geometry.js:479-487
        nrm = normalized(f3(pl.x, pl.y, 0));
        if (need_uv) {
            u = (float)(0.5 + atan2((double)pl.y, (double)pl.x) / (2 * JS_PI));
            v = (float)(0.5 + (double)pl.z);
        }
        break;
    case JSRT_GEOM_AABB: {  // geometry.js:210-224
        double norm_dist = 0;
        const float pc[3] = {pl.x, pl.y, pl.z};
        float nn[3] = {0, 0, 0};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double comp = ((double)pc[i] - (double)P.center[i]) / (double)P.half[i];
            const double ac = fabs(comp);
            if (ac > norm_dist) {
                norm_dist = ac;
                nn[0] = nn[1] = nn[2] = 0;
                nn[i] = (float)js_sign(comp);
            }
        }
        nrm = f3(nn[0], nn[1], nn[2]);
        break;
    }
    case JSRT_GEOM_TRIANGLE: {  // geometry.js:376-409
        if (!(PF & PF_TRI)) break;
        const DTri &T = S.tris[P.gindex];
        nrm = f3(T.n[0], T.n[1], T.n[2]);
        if (T.shade >= 0) {
            const DTriShade &TS = S.trish[T.shade];
            const F3 v2 = f3(pl.x - T.p0[0], pl.y - T.p0[1], pl.z - T.p0[2]);
            const double d20 = dot3(v2, f3(T.v0[0], T.v0[1], T.v0[2])), d21 = dot3(v2, f3(T.v1[0], T.v1[1], T.v1[2]));
            const double bv = (T.d11 * d20 - T.d01 * d21) / T.denom, bw = (T.d00 * d21 - T.d01 * d20) / T.denom;
            const float b0 = (float)(1 - bv - bw), b1 = (float)bv, b2 = (float)bw;
            if (TS.has_uv) {
                u = (TS.uv[0][0] * b0 + TS.uv[1][0] * b1) + TS.uv[2][0] * b2;
                v = (TS.uv[0][1] * b0 + TS.uv[1][1] * b1) + TS.uv[2][1] * b2;
            }
            if (TS.has_normal) {
                nrm = f3((TS.vn[0][0] * b0 + TS.vn[1][0] * b1) + TS.vn[2][0] * b2,
                         (TS.vn[0][1] * b0 + TS.vn[1][1] * b1) + TS.vn[2][1] * b2,
                         (TS.vn[0][2] * b0 + TS.vn[1][2] * b1) + TS.vn[2][2] * b2);
                nrm_w = (TS.vn[0][3] * b0 + TS.vn[1][3] * b1) + TS.vn[2][3] * b2;
            }
        }
        break;
    }
    case JSRT_GEOM_SDF: {  // SDFGeometry.materialData (sdf.js:41-47)
        if (!(PF & PF_SDF)) break;
        const jsrt_rec_sdfgeom &G = S.sdfg[P.gindex];
        const double dist0 = sdf_node_dist(S, G.root, pl);
        const float step = (float)G.normal_step;
        const float nx = (float)((sdf_node_dist(S, G.root, f3(pl.x + step, pl.y + 0.0f, pl.z + 0.0f)) - dist0) / G.normal_step);
        const float ny = (float)((sdf_node_dist(S, G.root, f3(pl.x + 0.0f, pl.y + step, pl.z + 0.0f)) - dist0) / G.normal_step);
        const float nz = (float)((sdf_node_dist(S, G.root, f3(pl.x + 0.0f, pl.y + 0.0f, pl.z + step)) - dist0) / G.normal_step);
        const SdfMD md = sdf_material(S, G.root, pl);
        if (md.has_bc) basecolor = md.bc;
        if (md.has_uv) { u = md.u; v = md.v; }
        nrm = normalized(f3(nx, ny, nz));
        break;
    }
    default: break;
    }
    // normal = inv_transform.transposed().times(normal).to4(0).normalized()  (world.js:133-134)
    F3 N;
    {
        const float wx = (float)((((double)nrm.x * inv[0] + (double)nrm.y * inv[4]) + (double)nrm.z * inv[8]) + (double)nrm_w * inv[12]);
        const float wy = (float)((((double)nrm.x * inv[1] + (double)nrm.y * inv[5]) + (double)nrm.z * inv[9]) + (double)nrm_w * inv[13]);
        const float wz = (float)((((double)nrm.x * inv[2] + (double)nrm.y * inv[6]) + (double)nrm.z * inv[10]) + (double)nrm_w * inv[14]);
        N = normalized(f3(wx, or0(wy), or0(wz)));
    }
    ShadeData sd;
    sd.pos = ray_point(o, d, h.t);  // material_data.position = ray.getPoint(distance)
    pos = sd.pos;
    const jsrt_rec_material &M = S.mat[P.material];
    const int mkind = (int)M.kind;
    Rng rng{key, addr, 0};
    if (mkind == JSRT_MAT_SOLID) {
        const F3 c = mc_eval(S, M.color, u, v);
        W.sx[i] = c.x; W.sy[i] = c.y; W.sz[i] = c.z;
        W.info[i] = INFO_HIT;
        return 0;
    }
    if (mkind == JSRT_MAT_TRANSPARENT) {  // materials.js:169-173
        const F3 a = scale(mc_eval(S, M.color, u, v), M.opacity);
        W.sx[i] = a.x; W.sy[i] = a.y; W.sz[i] = a.z;
        ch0 = Child{d, f3(1, 1, 1), f3(1, 1, 1), 1 - M.opacity};
        W.info[i] = INFO_HIT | (1u << INFO_NCHILD_SHIFT);
        return 1;
    }
    // getBaseFactors (materials.js:210-238)
    sd.V = neg(normalized(d));
    F3 Nn = normalized(N);
    sd.backside = false;
    double vdotn = dot3(sd.V, Nn);
    if (vdotn < 0) {
        Nn = neg(Nn);
        sd.backside = true;
        vdotn = -vdotn;
    }
    sd.N = Nn;
    sd.vdotn = vdotn;
    sd.R = normalized(sub(scale(Nn, 2 * vdotn), sd.V));
    sd.ambient = mul(basecolor, mc_eval(S, M.ambient, u, v));
    sd.diff = mul(basecolor, mc_eval(S, M.diffuse, u, v));
    sd.spec = mc_eval(S, M.specular, u, v);
    sd.refl = mc_eval(S, M.reflect, u, v);
    sd.trans = mc_eval(S, M.transmit, u, v);
    sd.smoothness = M.smoothness;
    sd.kr = 1;
    sd.has_refr = false;
    sd.refr = f3(0, 0, 0);
    if (mkind != JSRT_MAT_PHONG) {
        const double ratio = M.ratio;
        // fresnelReflectionFactor (materials.js:366-386)
        double kr;
        if (!__builtin_isfinite(ratio)) kr = 1;
        else {
            const double ni = sd.backside ? ratio : 1, nt = sd.backside ? 1 : ratio;
            const double cosi = vdotn, sint = ni / nt * sqrt(js_max(0, 1 - cosi * cosi));
            if (sint >= 1) kr = 1;
            else {
                const double cost = sqrt(js_max(0, 1 - sint * sint));
                const double Rs = ((nt * cosi) - (ni * cost)) / ((nt * cosi) + (ni * cost));
                const double Rp = ((ni * cosi) - (nt * cost)) / ((ni * cosi) + (nt * cost));
                kr = (Rs * Rs + Rp * Rp) / 2;
            }
        }
        sd.kr = kr;
        // getRefractionDirection (materials.js:358-364)
        const double r = sd.backside ? ratio : 1 / ratio, k = 1 - r * r * (1 - vdotn * vdotn);
        if (!(k < 0)) {
            sd.has_refr = true;
            sd.refr = add(scale(neg(sd.V), r), scale(Nn, r * vdotn - sqrt(k)));
        }
    }
    // colorFromLights (materials.js:240-259): k_shadow evaluates the light samples (one lane each,
    // RNG calls [0, light_draws) of this frame) from the material data handed off here; the
    // scatter draws below follow them (calls light_draws, ...)
    W.sx[i] = sd.ambient.x; W.sy[i] = sd.ambient.y; W.sz[i] = sd.ambient.z;
    uint32_t info = INFO_HIT;
    if (W.ns > 0) {
        info |= INFO_LIT;
        W.sox[tt] = sd.pos.x; W.soy[tt] = sd.pos.y; W.soz[tt] = sd.pos.z;
        W.fnx[tt] = sd.N.x; W.fny[tt] = sd.N.y; W.fnz[tt] = sd.N.z;
        W.frx[tt] = sd.R.x; W.fry[tt] = sd.R.y; W.frz[tt] = sd.R.z;
        W.ftx[tt] = sd.refr.x; W.fty[tt] = sd.refr.y; W.ftz[tt] = sd.refr.z;
        W.fdx[tt] = sd.diff.x; W.fdy[tt] = sd.diff.y; W.fdz[tt] = sd.diff.z;
        W.fsx[tt] = sd.spec.x; W.fsy[tt] = sd.spec.y; W.fsz[tt] = sd.spec.z;
        W.fkr[tt] = sd.kr;
        W.fmat[tt] = P.material;
        rng.calls = (uint32_t)S.light_draws;
    }
    int n = 0;
    auto push = [&](const Child &c) {  // unconditional selects keep both slots in registers
        const bool first = n == 0;
        ch0 = pick(first, c, ch0);
        ch1 = pick(first, ch1, c);
        ++n;
    };
    if (mkind == JSRT_MAT_PHONG) {  // materials.js:277-288
        if (dot3(sd.refl, sd.refl) > 0) push(Child{sd.R, f3(1, 1, 1), sd.refl, 1.0});
        if (dot3(sd.trans, sd.trans) > 0) push(Child{normalized(d), f3(1, 1, 1), sd.trans, 1.0});
    } else {  // materials.js:315-330
        if (sd.kr > 0) {
            F3 dir = sd.R, col = f3(1, 1, 1);
            bool ok = true;
            if (mkind == JSRT_MAT_PATH) ok = path_scatter(M.mirror_prob, true, sd.R, Nn, sd, rng, dir, col);
            if (ok) push(Child{dir, col, sd.refl, sd.kr});
        }
        if (sd.kr < 1) {
            F3 dir = sd.refr, col = f3(1, 1, 1);
            bool ok = sd.has_refr;
            if (mkind == JSRT_MAT_PATH) ok = path_scatter(M.mirror_prob, sd.has_refr, sd.refr, neg(Nn), sd, rng, dir, col);
            if (ok) push(Child{dir, col, sd.trans, 1 - sd.kr});
        }
    }
    W.info[i] = info | ((uint32_t)n << INFO_NCHILD_SHIFT);
    return n;
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gen(DScene S, RenderArgs A, WArgs W) {
    // level 0 holds one camera ray per path of the batch at slot q (no append); paths whose pixel
    // lies outside the image (edge patches) get a DEAD_RAY slot that misses and writes nothing
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;  // path index in the batch
    if (q >= W.npaths) return;
    int c = 0, py = 0, px = 0;
    const uint32_t pl = q % W.npix, sl = q / W.npix;  // sample-major: neighbours are neighbour pixels
    const uint32_t smp = W.s0 + sl;
    const bool valid = pixel_of(A, W.p0 + pl, c, py, px);
    if (A.max_depth <= 0) {  // World.color(ray, 0) = black; no level is traced
        W.root[3 * q] = W.root[3 * q + 1] = W.root[3 * q + 2] = 0.0f;
        return;
    }
    W.path[q] = q;
    if (!valid) {
        W.parent[q] = DEAD_RAY;
        return;
    }
    const uint32_t pixel = (uint32_t)(py * A.W + px);
    const uint32_t key = mix32(mix32(A.seed, pixel), smp);
    Rng pre{key, 0u, 0u};  // pre-root frame (address 0): jitter, then DOF draws
    double x = 2 * ((double)px / A.W) - 1, y = -2 * ((double)py / A.H) + 1;  // renderers.js:22-25
    if (A.kind != JSRT_RENDERER_SIMPLE) {
        const double jx = x + (2.0 / A.W) * (pre.next() - 0.5);  // renderers.js:95-96
        const double jy = y + (2.0 / A.H) * (pre.next() - 0.5);
        x = jx;
        y = jy;
    }
    F3 o, d;
    camera_ray(S.cam, x, y, pre, o, d);
    W.ox[q] = o.x; W.oy[q] = o.y; W.oz[q] = o.z;
    W.dx[q] = d.x; W.dy[q] = d.y; W.dz[q] = d.z;
    W.addr[q] = mix32(0u, 1u);
    W.key[q] = key;
    W.parent[q] = NO_PARENT;
}

template <int PF>
__global__ __launch_bounds__(256, JSRT_EXTEND_OCC) void k_extend(DScene S, WArgs W, uint32_t base, uint32_t count, double minD) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint32_t i = base + t;
    if (W.parent[i] == DEAD_RAY) {
        W.prim[i] = -1;
        return;
    }
    const F3 o = f3(W.ox[i], W.oy[i], W.oz[i]), d = f3(W.dx[i], W.dy[i], W.dz[i]);
    const Hit h = world_cast<PF, false>(S, o, d, minD, DINF, true);
    W.t[i] = h.t;
    W.prim[i] = h.prim;
    W.ctx[i] = h.ctx;
}

template <int PF>
__global__ __launch_bounds__(256, JSRT_SHADE_OCC) void k_shade(DScene S, WArgs W, uint32_t base, uint32_t count, int child_depth) {
    const uint32_t tt = blockIdx.x * 256 + threadIdx.x;
    const bool in = tt < count;
    const uint32_t i = base + (in ? tt : 0u);
    int nchild = 0;
    Child ch0, ch1;
    F3 pos = f3(0, 0, 0);
    uint32_t addr = 0, key = 0;
    bool hit = false;
    if (in) {
        const int prim = W.prim[i];
        if (prim < 0) {  // miss: World.color returns bg_color (world.js:35-36)
            write_result(W, i, f3(S.bg[0], S.bg[1], S.bg[2]));
            W.info[i] = 0;
        } else {
            hit = true;
            const F3 o = f3(W.ox[i], W.oy[i], W.oz[i]), d = f3(W.dx[i], W.dy[i], W.dz[i]);
            addr = W.addr[i];
            key = W.key[i];
            const Hit h{W.t[i], prim, W.ctx[i]};
            nchild = shade_node<PF>(S, W, i, tt, h, o, d, addr, key, ch0, ch1, pos);
        }
    }
    // children: World.color(child, depth - 1); at depth 0 they are black without a cast
    const uint32_t at = block_append<256>(W.counter, child_depth > 0 ? nchild : 0);
    if (!hit) return;
    const uint32_t path = W.path[i];
    auto emit = [&](const Child &c, uint32_t j) {
        const uint32_t sl = 2 * i + j;
        W.ccol[3 * sl] = c.col.x; W.ccol[3 * sl + 1] = c.col.y; W.ccol[3 * sl + 2] = c.col.z;
        W.cw[3 * sl] = c.w.x; W.cw[3 * sl + 1] = c.w.y; W.cw[3 * sl + 2] = c.w.z;
        W.ck[sl] = c.k;
        if (child_depth > 0) {
            const uint32_t r = at + j;
            W.ox[r] = pos.x; W.oy[r] = pos.y; W.oz[r] = pos.z;
            W.dx[r] = c.dir.x; W.dy[r] = c.dir.y; W.dz[r] = c.dir.z;
            W.addr[r] = mix32(addr, j + 1);
            W.key[r] = key;
            W.path[r] = path;
            W.parent[r] = sl;
        } else {
            W.slot[3 * sl] = W.slot[3 * sl + 1] = W.slot[3 * sl + 2] = 0.0f;
        }
    };
    if (nchild > 0) emit(ch0, 0);
    if (nchild > 1) emit(ch1, 1);
}

// One light sample of a lit node per lane (lane e = level index * ns + sample): the sample
// (lights.js sampleIterator), its shadow cast (materials.js:250-252) and, when unshadowed,
// colorFromLightSample (materials.js:261-269, 340-356); shadowed samples contribute 0.
template <int PF>
__global__ __launch_bounds__(256, JSRT_SHADOW_OCC) void k_shadow(DScene S, WArgs W, uint32_t base, uint32_t count) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ns = (uint32_t)W.ns;
    if (e >= count * ns) return;
    const uint32_t tt = e / ns, s = e - tt * ns, i = base + tt;
    if (!(W.info[i] & INFO_LIT)) return;
    const F3 P = f3(W.sox[tt], W.soy[tt], W.soz[tt]);
    const DLight &Lt = S.lights[S.sample_light[s]];
    Rng rng{W.key[i], W.addr[i], (uint32_t)S.sample_call[s]};
    F3 delta, L, lcol;
    light_sample(S, Lt, P, rng, delta, L, lcol);
#ifdef JSRT_AB_NOCAST
    const Hit sh{DINF, -1, 0};
#else
    const Hit sh = world_cast<PF, true>(S, P, delta, 0.0001, 1, false);
#endif
    F3 c = f3(0, 0, 0);
    if (!(sh.prim >= 0 && sh.t > 0 && sh.t < 1)) {
        ShadeData sd;
        sd.N = f3(W.fnx[tt], W.fny[tt], W.fnz[tt]);
        sd.R = f3(W.frx[tt], W.fry[tt], W.frz[tt]);
        sd.refr = f3(W.ftx[tt], W.fty[tt], W.ftz[tt]);
        sd.diff = f3(W.fdx[tt], W.fdy[tt], W.fdz[tt]);
        sd.spec = f3(W.fsx[tt], W.fsy[tt], W.fsz[tt]);
        sd.kr = W.fkr[tt];
        const jsrt_rec_material &M = S.mat[W.fmat[tt]];
        sd.smoothness = M.smoothness;
#ifdef JSRT_AB_NOCOLOR
        c = lcol;
#else
        c = light_sample_color((int)M.kind, sd, L, lcol);
#endif
    }
    W.scx[e] = c.x;
    W.scy[e] = c.y;
    W.scz[e] = c.z;
}

// colorFromLights' sums (materials.js:244-257): per light, its samples in order (a shadowed
// sample adds +0, which never changes an f32 running sum that starts at +0), times 1/samples.
__global__ __launch_bounds__(256) void k_lightsum(DScene S, WArgs W, uint32_t base, uint32_t count) {
    const uint32_t tt = blockIdx.x * 256 + threadIdx.x;
    if (tt >= count) return;
    const uint32_t i = base + tt;
    if (!(W.info[i] & INFO_LIT)) return;
    F3 ret = f3(W.sx[i], W.sy[i], W.sz[i]);  // ambient
    size_t e = (size_t)tt * W.ns;
    for (int li = 0; li < S.n_lights; ++li) {
        const DLight &Lt = S.lights[li];
        const int ns = Lt.kind == JSRT_LIGHT_POINT ? 1 : Lt.samples;
        F3 light_color = f3(0, 0, 0);
        for (int k = 0; k < ns; ++k, ++e) light_color = add(light_color, f3(W.scx[e], W.scy[e], W.scz[e]));
        if (ns > 0) ret = add(ret, scale(light_color, 1.0 / ns));
    }
    W.sx[i] = ret.x;
    W.sy[i] = ret.y;
    W.sz[i] = ret.z;
}

// surface.plus(child.times(col).times(w).times(k)) for the children in order (materials.js:277-330)
__global__ __launch_bounds__(256) void k_reduce(WArgs W, uint32_t base, uint32_t count) {
    const uint32_t tt = blockIdx.x * 256 + threadIdx.x;
    if (tt >= count) return;
    const uint32_t i = base + tt;
    const uint32_t info = W.info[i];
    if (!(info & INFO_HIT)) return;
    F3 c = f3(W.sx[i], W.sy[i], W.sz[i]);
    const int n = (int)((info >> INFO_NCHILD_SHIFT) & 3);
    for (int j = 0; j < n; ++j) {
        const uint32_t sl = 2 * i + (uint32_t)j;
        const F3 v = f3(W.slot[3 * sl], W.slot[3 * sl + 1], W.slot[3 * sl + 2]);
        const F3 col = f3(W.ccol[3 * sl], W.ccol[3 * sl + 1], W.ccol[3 * sl + 2]);
        const F3 w = f3(W.cw[3 * sl], W.cw[3 * sl + 1], W.cw[3 * sl + 2]);
        c = add(c, scale(mul(mul(v, col), w), W.ck[sl]));
    }
    write_result(W, i, c);
}

// per pixel, the batch's samples in order (renderers.js:93-97, 52-61)
__global__ __launch_bounds__(256) void k_accum(RenderArgs A, WArgs W) {
    const uint32_t pl = blockIdx.x * 256 + threadIdx.x;
    if (pl >= W.npix) return;
    int c, py, px;
    if (!pixel_of(A, W.p0 + pl, c, py, px)) return;
    const size_t oi = (size_t)c * A.H + py;
    F3 acc = f3(A.accum[4 * oi], A.accum[4 * oi + 1], A.accum[4 * oi + 2]);
    const uint32_t nsb = W.npaths / W.npix;
    for (uint32_t sl = 0; sl < nsb; ++sl) {
        const uint32_t q = sl * W.npix + pl;
        const F3 col = f3(W.root[3 * q], W.root[3 * q + 1], W.root[3 * q + 2]);
        if (A.kind == JSRT_RENDERER_RANDOM) acc = add(acc, scale(col, 1.0 / A.spp));
        else if (A.kind == JSRT_RENDERER_INCREMENTAL)
            acc = f3(acc.x + col.x, acc.y + or0(col.y), acc.z + or0(col.z));  // buffer.plus(c.to4(true))
        else acc = col;
    }
    A.accum[4 * oi] = acc.x;
    A.accum[4 * oi + 1] = acc.y;
    A.accum[4 * oi + 2] = acc.z;
}

__global__ __launch_bounds__(256) void k_final(RenderArgs A) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= (uint32_t)A.ncols * A.H) return;
    const F3 acc = f3(A.accum[4 * p], A.accum[4 * p + 1], A.accum[4 * p + 2]);
    const F3 out = (A.kind == JSRT_RENDERER_INCREMENTAL) ? scale(acc, 1.0 / A.spp) : acc;  // times(1/(iter+1))
    A.rgba[p] = set_color_rgba(out);
    if (A.colors) {
        A.colors[4 * p] = out.x;
        A.colors[4 * p + 1] = out.y;
        A.colors[4 * p + 2] = out.z;
        A.colors[4 * p + 3] = 1.0f;
    }
}

// ---------------------------------------------------------------------------------------------
// host orchestration
namespace {
inline unsigned grid(size_t n) { return (unsigned)((n + 255) / 256); }

template <class T>
T *carve(uint8_t *&p, size_t n) {
    T *r = reinterpret_cast<T *>(p);
    p += (n * sizeof(T) + 255) & ~(size_t)255;
    return r;
}
size_t need(size_t n, size_t sz) { return (n * sz + 255) & ~(size_t)255; }
}  // namespace

void EventPairs::begin(hipStream_t s) {
    if (used == b.size()) {
        hipEvent_t x, y;
        (void)hipEventCreate(&x);
        (void)hipEventCreate(&y);
        b.push_back(x);
        e.push_back(y);
    }
    (void)hipEventRecord(b[used], s);
}
void EventPairs::end(hipStream_t s) { (void)hipEventRecord(e[used++], s); }
double EventPairs::total_ms() const {
    double ms = 0;
    for (size_t k = 0; k < used; ++k) {
        float x = 0;
        if (hipEventElapsedTime(&x, b[k], e[k]) == hipSuccess) ms += x;
    }
    return ms;
}
EventPairs::~EventPairs() {
    for (auto x : b) (void)hipEventDestroy(x);
    for (auto x : e) (void)hipEventDestroy(x);
}

hipError_t Wavefront::reserve(size_t pool, size_t level_cap, int ns) {
    if (mem && pool <= cap_pool && level_cap <= cap_level && ns <= cap_ns) return hipSuccess;
    size_t bytes = 0;
    bytes += 10 * need(pool, 4) + need(pool, 8) + 2 * need(pool, 4);  // rays + hits
    bytes += 4 * need(pool, 4);                                      // info + surface
    bytes += 3 * need(6 * pool, 4) + need(2 * pool, 8);              // ccol cw slot + ck
    bytes += 18 * need(level_cap, 4) + need(level_cap, 8) + need(level_cap, 4) + 3 * need(level_cap * (size_t)ns, 4);
    bytes += need(3 * level_cap, 4) + 256;
    if (mem) (void)hipFree(mem);
    mem = nullptr;
    cap_pool = cap_level = 0;
    hipError_t e = hipMalloc(&mem, bytes);
    if (e != hipSuccess) return e;
    cap_bytes = bytes;
    cap_pool = pool;
    cap_level = level_cap;
    cap_ns = ns;
    uint8_t *p = static_cast<uint8_t *>(mem);
    WArgs &w = args;
    w.ox = carve<float>(p, pool); w.oy = carve<float>(p, pool); w.oz = carve<float>(p, pool);
    w.dx = carve<float>(p, pool); w.dy = carve<float>(p, pool); w.dz = carve<float>(p, pool);
    w.addr = carve<uint32_t>(p, pool); w.key = carve<uint32_t>(p, pool);
    w.path = carve<uint32_t>(p, pool); w.parent = carve<uint32_t>(p, pool);
    w.t = carve<double>(p, pool); w.prim = carve<int32_t>(p, pool); w.ctx = carve<int32_t>(p, pool);
    w.info = carve<uint32_t>(p, pool);
    w.sx = carve<float>(p, pool); w.sy = carve<float>(p, pool); w.sz = carve<float>(p, pool);
    w.ccol = carve<float>(p, 6 * pool); w.cw = carve<float>(p, 6 * pool); w.slot = carve<float>(p, 6 * pool);
    w.ck = carve<double>(p, 2 * pool);
    w.sox = carve<float>(p, level_cap); w.soy = carve<float>(p, level_cap); w.soz = carve<float>(p, level_cap);
    w.fnx = carve<float>(p, level_cap); w.fny = carve<float>(p, level_cap); w.fnz = carve<float>(p, level_cap);
    w.frx = carve<float>(p, level_cap); w.fry = carve<float>(p, level_cap); w.frz = carve<float>(p, level_cap);
    w.ftx = carve<float>(p, level_cap); w.fty = carve<float>(p, level_cap); w.ftz = carve<float>(p, level_cap);
    w.fdx = carve<float>(p, level_cap); w.fdy = carve<float>(p, level_cap); w.fdz = carve<float>(p, level_cap);
    w.fsx = carve<float>(p, level_cap); w.fsy = carve<float>(p, level_cap); w.fsz = carve<float>(p, level_cap);
    w.fkr = carve<double>(p, level_cap);
    w.fmat = carve<int32_t>(p, level_cap);
    const size_t se = level_cap * (size_t)ns;
    w.scx = carve<float>(p, se); w.scy = carve<float>(p, se); w.scz = carve<float>(p, se);
    w.root = carve<float>(p, 3 * level_cap);
    w.counter = carve<uint32_t>(p, 64);
    return hipSuccess;
}

Wavefront::~Wavefront() {
    if (mem) (void)hipFree(mem);
}

namespace {
template <int PF>
hipError_t run_batch(const DScene &S, const RenderArgs &A, const WArgs &W, hipStream_t st, KernelTimes *kt,
                     uint32_t *h_counter, bool &overflow) {
    auto timed = [&](int which, auto launch) {
        if (kt) kt->ev[which].begin(st);
        launch();
        if (kt) kt->ev[which].end(st);
    };
    std::vector<uint32_t> lvl_base, lvl_count;
    overflow = false;
    hipError_t e;
    timed(KT_GEN, [&] { hipLaunchKernelGGL(k_gen, dim3(grid(W.npaths)), dim3(256), 0, st, S, A, W); });
    uint32_t base = 0, count = A.max_depth > 0 ? W.npaths : 0;
    for (int L = 0; L < A.max_depth && count > 0; ++L) {
        const uint32_t next = base + count;
        const int child_depth = A.max_depth - L - 1;
        if ((size_t)count > W.level_cap || (child_depth > 0 && (size_t)next + 2 * (size_t)count > W.pool)) {
            overflow = true;
            return hipSuccess;
        }
        lvl_base.push_back(base);
        lvl_count.push_back(count);
        timed(KT_EXTEND, [&] {
            hipLaunchKernelGGL(k_extend<PF>, dim3(grid(count)), dim3(256), 0, st, S, W, base, count,
                               L == 0 ? 0.0 : 0.0001);
        });
        *h_counter = next;
        if ((e = hipMemcpyAsync(W.counter, h_counter, 4, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
        timed(KT_SHADE, [&] {
            hipLaunchKernelGGL(k_shade<PF>, dim3(grid(count)), dim3(256), 0, st, S, W, base, count, child_depth);
        });
        if (W.ns > 0) {
            timed(KT_SHADOW, [&] {
                hipLaunchKernelGGL(k_shadow<PF>, dim3(grid((size_t)count * W.ns)), dim3(256), 0, st, S, W, base, count);
            });
            timed(KT_LIGHTSUM, [&] {
                hipLaunchKernelGGL(k_lightsum, dim3(grid(count)), dim3(256), 0, st, S, W, base, count);
            });
        }
        if ((e = hipMemcpyAsync(h_counter, W.counter, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        base = next;
        count = *h_counter - next;
    }
    for (int L = (int)lvl_base.size() - 1; L >= 0; --L)
        timed(KT_REDUCE, [&] {
            hipLaunchKernelGGL(k_reduce, dim3(grid(lvl_count[L])), dim3(256), 0, st, W, lvl_base[L], lvl_count[L]);
        });
    timed(KT_ACCUM, [&] { hipLaunchKernelGGL(k_accum, dim3(grid(W.npix)), dim3(256), 0, st, A, W); });
    return hipGetLastError();
}
}  // namespace

hipError_t render_frame(const DScene &S, const RenderArgs &A, int ns, Wavefront &wf, hipStream_t st, KernelTimes *kt,
                        size_t max_paths, const std::function<bool(int, double)> &progress) {
    if (!A.accum) return hipErrorInvalidValue;
    const uint32_t npix_total = (uint32_t)A.patches * 64u;
    if (ns > 4) max_paths = max_paths * 4 / (size_t)ns;  // the per-sample hand-off scales with ns
    if (max_paths < 64) max_paths = 64;
    uint32_t npix = npix_total, nsb = 1;  // batch: [p0, p0 + npix) pixels x [s0, s0 + nsb) samples
    if ((size_t)npix > max_paths) npix = (uint32_t)(max_paths & ~(size_t)63);
    else nsb = (uint32_t)std::max<size_t>(1, std::min<size_t>(max_paths / npix, (size_t)A.spp));
    // ray pool for all levels of a batch; one level may hold up to half of it (Fresnel / glass
    // materials spawn two children per hit).  A one-patch batch that still overflows grows it.
    size_t pool = (size_t)npix * nsb * 8, level_cap = pool / 2;
    hipError_t e = wf.reserve(pool, level_cap, ns > 0 ? ns : 1);
    if (e != hipSuccess) return e;
    WArgs W = wf.args;
    W.ns = ns;
    W.pool = pool;
    W.level_cap = level_cap;
    if ((e = hipMemsetAsync(A.accum, 0, (size_t)A.ncols * A.H * 4 * sizeof(float), st)) != hipSuccess) return e;
    uint32_t *h_counter = nullptr;
    if ((e = hipHostMalloc((void **)&h_counter, 16, 0)) != hipSuccess) return e;
    const uint64_t total = (uint64_t)npix_total * A.spp;
    uint64_t done = 0;
    for (uint32_t s0 = 0; s0 < (uint32_t)A.spp && e == hipSuccess; s0 += nsb) {
        const uint32_t nb = std::min<uint32_t>(nsb, (uint32_t)A.spp - s0);
        for (uint32_t p0 = 0; p0 < npix_total && e == hipSuccess; p0 += npix) {
            // halve the pixel range until the batch fits (branching materials grow the levels)
            std::vector<std::pair<uint32_t, uint32_t>> todo{{p0, std::min(npix, npix_total - p0)}};
            while (!todo.empty() && e == hipSuccess) {
                const auto job = todo.back();
                todo.pop_back();
                W.p0 = job.first;
                W.npix = job.second;
                W.s0 = s0;
                W.npaths = job.second * nb;
                bool overflow = false;
                switch (S.profile) {
                case PF_ANALYTIC: e = run_batch<PF_ANALYTIC>(S, A, W, st, kt, h_counter, overflow); break;
                case PF_MESH: e = run_batch<PF_MESH>(S, A, W, st, kt, h_counter, overflow); break;
                case PF_SDF: e = run_batch<PF_SDF>(S, A, W, st, kt, h_counter, overflow); break;
                default: e = run_batch<PF_ALL>(S, A, W, st, kt, h_counter, overflow); break;
                }
                if (e != hipSuccess) break;
                if (overflow) {
                    if (job.second <= 64) {  // cannot split further: grow the pool and retry
                        if (pool > ((size_t)1 << 31)) { e = hipErrorOutOfMemory; break; }
                        if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
                        pool *= 2;
                        level_cap = pool / 2;
                        if ((e = wf.reserve(pool, level_cap, ns > 0 ? ns : 1)) != hipSuccess) break;
                        const WArgs keep = W;
                        W = wf.args;
                        W.ns = ns;
                        W.pool = pool;
                        W.level_cap = level_cap;
                        W.p0 = keep.p0; W.npix = keep.npix; W.s0 = keep.s0; W.npaths = keep.npaths;
                        todo.push_back(job);
                        continue;
                    }
                    const uint32_t half = ((job.second / 2) + 63) & ~63u;
                    todo.push_back({job.first + half, job.second - half});
                    todo.push_back({job.first, half});
                    continue;
                }
                done += (uint64_t)job.second * nb;
            }
        }
        if (e == hipSuccess && progress && !progress((int)(s0 + nb - 1), (double)done / (double)total)) break;
    }
    (void)hipHostFree(h_counter);
    if (e != hipSuccess) return e;
    if (kt) kt->ev[KT_FINAL].begin(st);
    hipLaunchKernelGGL(k_final, dim3(grid((size_t)A.ncols * A.H)), dim3(256), 0, st, A);
    if (kt) kt->ev[KT_FINAL].end(st);
    return hipGetLastError();
}

#ifdef JSRT_DBG_COUNT
extern "C" int jsrt_debug_counters(unsigned long long *out, int n) {
    if (n > 256) n = 256;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long zero[256] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace jsrt
