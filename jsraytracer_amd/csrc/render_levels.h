// render_levels.h — the per-level kernels of the wavefront renderer (render.hip) and the batch
// launcher that enqueues them, templated on the kernel profile PF (device_scene.h).  render_pf.hip
// instantiates them once per profile (-DJSRT_PF=...), so the four profiles compile as separate
// translation units in parallel; render.hip holds the profile-independent kernels and the frame loop.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "device_common.h"
#include "render_kernel.h"

#ifndef JSRT_SHADE_OCC  // min waves per SIMD requested for k_shade: 4 (SDF 167 -> 128 VGPRs) = Menger +5 %, r03_s34
#define JSRT_SHADE_OCC 4
#endif
#ifndef JSRT_SHADE_OCC_SDF  // SDF profiles: 3 waves (round 6, after the four-distance normal: Menger k_shade 28.5 ->
#define JSRT_SHADE_OCC_SDF 3  // 25.1 ms, 5 waves 34.9; profiles/r06_s25_shade_occ_menger.txt)
#endif
#ifndef JSRT_SHADE_OCC_FLAT  // analytic profile: 5 waves (95 VGPRs, 8 spilled) beat 4 (105): cornell +2.4 %, r03_s14
#define JSRT_SHADE_OCC_FLAT 5
#endif
// k_shadow / k_extend: at least 6 / 5 waves per SIMD.  Their casts are latency-bound (BVH node and
// scene loads on a dependent chain), so more resident waves beat the registers the compiler would
// otherwise keep (A/B on MI355X: cornell +3 %, bunny +15 %, dragon +4 % against no bound; 8 waves
// for k_shadow spills and loses 11 % on cornell).
#ifndef JSRT_SHADOW_OCC
#define JSRT_SHADOW_OCC 6
#endif
#ifndef JSRT_SHADOW_OCC_FLAT  // analytic profile: 8 waves (64 VGPRs, 15 spilled): cornell k_shadow 41.9 -> 41.5 ms and
// every interleaved 8-step pair faster (round 6, profiles/r06_s5_ab.txt); 7 waves (72 VGPRs) before
#define JSRT_SHADOW_OCC_FLAT 8
#endif
#ifndef JSRT_EXTEND_OCC
#define JSRT_EXTEND_OCC 5
#endif
#ifndef JSRT_MARCH_OCC  // min waves per SIMD of the persistent SDF marches (k_extend_q, k_shadow_cast)
#define JSRT_MARCH_OCC 1
#endif
#ifndef JSRT_EXTEND_OCC_FLAT  // analytic profile: 8 waves (round 6: k_extend 30.37 -> 29.74 ms, 5 waves 30.35,
#define JSRT_EXTEND_OCC_FLAT 8   // profiles/r06_s21_occ_cornell.txt; round 2 had 6 beat 5, r02_s20)
#endif
// optional waves-per-EU window (min, max) per kernel for A/B occupancy experiments
#ifdef JSRT_SHADOW_WPE
#define SHADOW_ATTR __attribute__((amdgpu_waves_per_eu(JSRT_SHADOW_WPE)))
#else
#define SHADOW_ATTR
#endif
#ifdef JSRT_SHADE_WPE
#define SHADE_ATTR __attribute__((amdgpu_waves_per_eu(JSRT_SHADE_WPE)))
#else
#define SHADE_ATTR
#endif

namespace jsrt {

#ifdef JSRT_X_STAMPS
// (timing experiment only) per-phase shader-clock cycles of k_shade: every 16th block's waves add each phase's
// cycles into their own slot (no atomics: same-address atomics from many waves would serialise and swamp the
// kernel), g_xst[slot][k] and the count in [slot][8 + k]; jsrt_x_stamps (render_pf.hip) sums the slots
constexpr int XST_SLOTS = 32768;
static __device__ unsigned long long g_xst[XST_SLOTS][16];
template <class T>
__device__ __forceinline__ void xst(int k, uint64_t &t, const T &dep) {
    asm volatile("" ::"v"(dep));  // the phase ends when `dep` is available
    const uint64_t now = __builtin_amdgcn_s_memtime();
    const uint32_t slot = (blockIdx.x >> 4) * 4 + (threadIdx.x >> 6);
    if (__lane_id() == 0 && (blockIdx.x & 15) == 0 && slot < XST_SLOTS) {
        g_xst[slot][k] += (unsigned long long)(now - t);
        g_xst[slot][8 + k] += 1ull;
    }
    t = now;
}
#define XST_BEGIN uint64_t xst_t = __builtin_amdgcn_s_memtime();
#define XST(k, dep) xst(k, xst_t, dep)
#else
#define XST_BEGIN
#define XST(k, dep)
#endif

constexpr uint32_t NO_PARENT = 0xFFFFFFFFu;  // camera ray: its result is the path's root colour
constexpr uint32_t DEAD_RAY = 0xFFFFFFFEu;   // level-0 slot of a path outside the image (no result)
constexpr int32_t NO_RAY = -2;                // W.prim of a slot that holds no ray to trace

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

// Two block-aggregated appends at once, one 64-bit atomic per block on a counter pair (ctr[0], ctr[1]):
// n0 (0..2) entries on the low word and n1 (0..1) on the high one (two atomics on one L2 line serialise:
// measured, k_shade 2.6 -> 7.9 ms per cornell launch).  Every thread of the block must call it; o0 / o1 =
// this thread's first offsets.
__device__ __forceinline__ void block_append2(uint32_t *ctr, int n0, int n1, uint32_t &o0, uint32_t &o1) {
    constexpr int NW = 256 / 64;
    __shared__ uint32_t s0[NW + 1], s1[NW + 1];
    const uint64_t a1 = __ballot(n0 >= 1), a2 = __ballot(n0 >= 2), b1 = __ballot(n1 >= 1);
    const int lane = (int)__lane_id(), wid = (int)(threadIdx.x >> 6);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t p0 = (uint32_t)(__popcll(a1 & lt) + __popcll(a2 & lt)), p1 = (uint32_t)__popcll(b1 & lt);
    if (lane == 0) {
        s0[wid] = (uint32_t)(__popcll(a1) + __popcll(a2));
        s1[wid] = (uint32_t)__popcll(b1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x0 = 0, x1 = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = s0[w], d = s1[w];
            s0[w] = x0;
            s1[w] = x1;
            x0 += c;
            x1 += d;
        }
        const unsigned long long old =
            (x0 | x1) ? atomicAdd(reinterpret_cast<unsigned long long *>(ctr), ((unsigned long long)x1 << 32) | x0) : 0ull;
        s0[NW] = (uint32_t)old;
        s1[NW] = (uint32_t)(old >> 32);
    }
    __syncthreads();
    o0 = s0[NW] + s0[wid] + p0;
    o1 = s1[NW] + s1[wid] + p1;
}

// Block-aggregated append with the block's children grouped by a 3-bit key (the direction octant): one
// atomic per block on the level counter; o0 / o1 = the offsets of this thread's children in the block's
// range (children of one key contiguous, in no particular order within a key).  Every thread of the
// block must call it.
__device__ __forceinline__ uint32_t block_append_keyed(uint32_t *counter, int n, int k0, int k1, uint32_t &o0,
                                                       uint32_t &o1) {
    __shared__ uint32_t s_cnt[8], s_base[9];
    if (threadIdx.x < 8) s_cnt[threadIdx.x] = 0u;
    __syncthreads();
    const int lane = (int)__lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    uint32_t r[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bool has = n > j;
        const int k = j == 0 ? k0 : k1;
        uint64_t todo = __ballot(has);
        while (todo) {  // one LDS atomic per distinct key of the wave
            const int first = __builtin_ctzll(todo);
            const int kv = __builtin_amdgcn_readlane(k, first);
            const uint64_t m = __ballot(has && k == kv);
            uint32_t b = 0;
            if (lane == first) b = atomicAdd(&s_cnt[kv], (uint32_t)__popcll(m));
            b = __shfl(b, first);
            if (has && k == kv) r[j] = b + (uint32_t)__popcll(m & lt);
            todo &= ~m;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < 8; ++k) {
            s_base[k] = acc;
            acc += s_cnt[k];
        }
        s_base[8] = acc ? atomicAdd(counter, acc) : 0u;
    }
    __syncthreads();
    o0 = s_base[k0 & 7] + r[0];
    o1 = s_base[k1 & 7] + r[1];
    return s_base[8];
}
__device__ __forceinline__ int octant(F3 d) { return (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0); }

// Grid cell of a hit point (DScene::grid_*), grid_cells when outside the grid (or not finite)
__device__ __forceinline__ int grid_cell(const DScene &S, F3 p) {
    const float fx = (p.x - S.grid_lo[0]) * S.grid_inv[0], fy = (p.y - S.grid_lo[1]) * S.grid_inv[1],
                fz = (p.z - S.grid_lo[2]) * S.grid_inv[2];
    if (!(fx >= 0.0f && fx < (float)S.grid_dim[0] && fy >= 0.0f && fy < (float)S.grid_dim[1] && fz >= 0.0f &&
          fz < (float)S.grid_dim[2]))
        return S.grid_cells;
    return (int)fx + S.grid_dim[0] * ((int)fy + S.grid_dim[1] * (int)fz);
}


__device__ __forceinline__ void write_result(const WArgs &W, uint32_t i, F3 c) {  // tree schedule
    const uint32_t p = W.parent[i];
    if (p == DEAD_RAY) return;
    if (p == NO_PARENT) {
        float *dst = W.root + 3 * (size_t)W.path[i];
        dst[0] = c.x;
        dst[1] = c.y;
        dst[2] = c.z;
    } else {
        W.slot[(size_t)(p & 1u) * W.nstride + (p >> 1)] = make_float4(c.x, c.y, c.z, 0.0f);
    }
}

// patch-ordered owned pixel index -> (owned column c, row py, image column px).  8 x 8-pixel patches in raster order,
// or (A.tile_p > 0) in raster order within tiles of tile_p x tile_p patches taken in raster order, the last tile
// row and column partial: the pixels of consecutive indices, and so the rays a batch has in flight, then cover a
// compact region of the image rather than a band as wide as it (the BVH working set of their casts)
__device__ __forceinline__ bool pixel_of(const RenderArgs &A, uint32_t p, int &c, int &py, int &px) {
    int patch = (int)(p >> 6);
    const int lane = (int)(p & 63);
    if (A.tile_p > 0) {
        const int T = A.tile_p, pxn = A.patches_x, pyn = A.patches / A.patches_x;
        const int ty = patch / (pxn * T), r = patch - ty * pxn * T;  // (every tile row but the last is full)
        const int h = min(T, pyn - ty * T);
        const int tx = r / (T * h), r2 = r - tx * T * h;  // (every tile of the row but the last is full)
        const int w = min(T, pxn - tx * T);
        patch = (ty * T + r2 / w) * pxn + tx * T + r2 % w;
    }
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

// Tree schedule: level L of the batch occupies pool slots [base, base + count).  Counts live on
// the device (k_gen writes level 0, k_shade appends level L + 1), so the host enqueues every level
// without reading them back; an overflowed batch reads as empty everywhere and is redone.
struct LevelRange {
    uint32_t base, count;
};
__device__ __forceinline__ LevelRange level_range(const WArgs &W, int L) {
    if (W.lvl[LVL_FLAG]) return LevelRange{0u, 0u};
    uint32_t b = 0;
    for (int j = 0; j < L; ++j) b += W.lvl[j];
    return LevelRange{b, W.lvl[L]};
}
// Chain schedule: level L's node records start at L * cap.  It visits count chains: every path (level 0,
// and every level without side chains), else the hybrid chain's live chains of level L: the chains that
// continue from level L - 1 (listed, lvl[2L]) and then the side chains that start at L (lvl[2L + 1], ids
// contiguous).  Keeping the new side chains out of the list keeps every wave's slots in one run: a side
// chain interleaved with its parent's neighbours cost each 4-B SoA store of its wave a cache line more.
__device__ __forceinline__ LevelRange chain_level(const WArgs &W, int L) {
    const uint32_t base = (uint32_t)L * W.cap;
    if (!W.hybrid) return LevelRange{base, W.npaths};
    if (W.lvl[LVL_FLAG]) return LevelRange{base, 0u};
    return LevelRange{base, W.lvl[2 * L] + W.lvl[2 * L + 1]};
}
// the first id of the side chains that start at level L (ids of earlier starts below it)
__device__ __forceinline__ uint32_t side_base(const WArgs &W, int L) {
    uint32_t c = W.npaths;
    for (int j = 1; j < L; ++j) c += as_const(W.lvl)[2 * j + 1];  // (words no kernel of level >= L changes)
    return c;
}
// the chain slot of level L's t-th visited chain
__device__ __forceinline__ uint32_t chain_slot(const WArgs &W, int L, uint32_t t) {
    if (!W.hybrid || L == 0) return t;
    const uint32_t nc = as_const(W.lvl)[2 * L];
    return t < nc ? ((L & 1) ? W.list1 : W.list0)[t] : side_base(W, L) + (t - nc);
}

// shadow hand-off plane flags (store_hand)
constexpr uint32_t HAND_KR = 0x80000000u;    // planes 3 .w and 5: kr != 1 (and refr)
constexpr uint32_t HAND_DIFF = 0x40000000u;  // plane 2: diff is not the material's constant
constexpr uint32_t HAND_R = 0x20000000u;     // plane 3: the specular term needs R
constexpr uint32_t HAND_SPEC = 0x10000000u;  // plane 4: spec is not the material's constant
constexpr uint32_t HAND_MAT = 0x0FFFFF00u;   // mat << 8
constexpr int HAND_PLANES = 6;

// The material data k_shade hands to k_shadow for one lit node (after getBaseFactors), plus the
// node's RNG frame (its light-sample draws come first, materials.js:244-257).
struct Handoff {
    F3 pos, N, R, refr, diff, spec;
    double kr;
    int32_t mkind, mat;
    uint32_t addr, key;
    uint32_t node;   // the node's level index / chain slot (bucketed hand-off: where k_shadow writes its colour)
    uint32_t mask;   // shadow-root mask index (DScene::grid_mask) of the node's hit point
    uint32_t flags;  // HAND_*: the optional planes this node stores
};
struct NodeOut {
    F3 surf;        // surface colour: the final colour of an unlit node, the ambient term of a lit one
    uint32_t info;  // INFO_* bits + child count

    Handoff h;      // h.pos (the hit point) is set for every hit; the rest for lit nodes
};

// Primitive.color (world.js:125-137) up to Material.color: Geometry.materialData of the hit (per kind,
// geometry.js / sdf.js:41-47) and the world normal inv_transform.transposed().times(n).to4(0)
// .normalized().  ALL (the material-data known answers, jsrt_material_data): UV of every kind that has
// one and a triangle's barycentric coordinates, whether or not the material reads them.
struct Surface {
    F3 N;          // world normal (w = 0)
    float u, v;    // UV (when has_uv, or when the material reads it)
    F3 basecolor;  // SDF basecolor, else (1, 1, 1)
    F3 bary;       // ALL: a triangle's barycentric coordinates
    int has_uv, has_bc, has_bary;
};
template <int PF, bool ALL>
__device__ __forceinline__ void surface_data(const DScene &S, const Hit &h, F3 o, F3 d, bool need_uv, Surface &sf) {
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
    if (ALL) need_uv = true;
    const F3 lo = xf_point(inv, o), ld = xf_dir(inv, d);
    const F3 pl = ray_point(lo, ld, h.t);  // base_data.position (local)
    F3 nrm = f3(0, 0, 0);
    float nrm_w = 0.0f;
    float u = 0, v = 0;
    F3 basecolor = f3(1, 1, 1);
    int has_uv = 0, has_bc = 0, has_bary = 0;
    F3 bary = f3(0, 0, 0);
    switch (P.gkind) {
    case JSRT_GEOM_PLANE:
    case JSRT_GEOM_SQUARE:
    case JSRT_GEOM_CIRCLE:  // SimplePlane.materialData (geometry.js:249-254)
        nrm = f3(0, 0, 1);
        u = pl.x;
        v = pl.y;
        has_uv = 1;
        break;
    case JSRT_GEOM_SPHERE: {  // geometry.js:449-455: position.normalized() includes w = 1
        const double nn = sqrt(dot3(pl, pl) + 1.0);
        nrm = pl;
        nrm_w = 1.0f;
        if (nn > 0.00001) { nrm = scale(pl, 1 / nn); nrm_w = (float)(1.0 * (1 / nn)); }
        if (need_uv) cart_to_sph(nrm, u, v);
        has_uv = 1;
        break;
    }
    case JSRT_GEOM_CYLINDER:  // geometry.js:479-487
        nrm = normalized(f3(pl.x, pl.y, 0));
        if (need_uv) {
            u = (float)(0.5 + fdlibm::atan2((double)pl.y, (double)pl.x) / (2 * JS_PI));
            v = (float)(0.5 + (double)pl.z);
        }
        has_uv = 1;
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
        if (ALL || T.shade >= 0) {  // toBarycentric (geometry.js:389-396)
            const F3 v2 = f3(pl.x - T.p0[0], pl.y - T.p0[1], pl.z - T.p0[2]);
            const double d20 = dot3(v2, f3(T.v0[0], T.v0[1], T.v0[2])), d21 = dot3(v2, f3(T.v1[0], T.v1[1], T.v1[2]));
            const double bv = (T.d11 * d20 - T.d01 * d21) / T.denom, bw = (T.d00 * d21 - T.d01 * d20) / T.denom;
            const float b0 = (float)(1 - bv - bw), b1 = (float)bv, b2 = (float)bw;
            bary = f3(b0, b1, b2);
            has_bary = 1;
            if (T.shade >= 0) {  // Triangle.blend of the psdata (geometry.js:397-409)
                const DTriShade &TS = S.trish[T.shade];
                if (TS.has_uv) {
                    u = (TS.uv[0][0] * b0 + TS.uv[1][0] * b1) + TS.uv[2][0] * b2;
                    v = (TS.uv[0][1] * b0 + TS.uv[1][1] * b1) + TS.uv[2][1] * b2;
                    has_uv = 1;
                }
                if (TS.has_normal) {
                    nrm = f3((TS.vn[0][0] * b0 + TS.vn[1][0] * b1) + TS.vn[2][0] * b2,
                             (TS.vn[0][1] * b0 + TS.vn[1][1] * b1) + TS.vn[2][1] * b2,
                             (TS.vn[0][2] * b0 + TS.vn[1][2] * b1) + TS.vn[2][2] * b2);
                    nrm_w = (TS.vn[0][3] * b0 + TS.vn[1][3] * b1) + TS.vn[2][3] * b2;
                }
            }
        }
        break;
    }
    case JSRT_GEOM_SDF: {  // SDFGeometry.materialData (sdf.js:41-47)
        if (!(PF & PF_SDF)) break;
        const jsrt_rec_sdfgeom &G = S.sdfg[P.gindex];
        // the distance at pl and at the three offset points (sdf.js:41-47), from one evaluation site in
        // a loop: the form's straight-line code or the VM is emitted once, not four times (Menger k_shade
        // 72 -> 64 ms, r03_s14)
        const float step = (float)G.normal_step;
        double dd[4] = {0, 0, 0, 0};
        bool four = false;  // the Menger form's four distances together (sdf_forms.h sdf_form_normal4)
        double hab[2] = {0, 0};
        if (S.sdf_all_forms) {
            const int pc = S.sdf_range[2 * G.root];
            for (;;) {  // waterfall over the lanes' programs (uniform pc)
                const int pcu = uni(pc);
                if (pc == pcu) {
                    four = sdf_form_normal4(as_const(S.sdf_const), as_const(S.sdf_insn), pcu, pl, step, dd, hab);
                    break;
                }
            }
        }
#pragma unroll 1
        for (int k = 0; k < (four ? 0 : 4); ++k) {
            const F3 q = f3(pl.x + (k == 1 ? step : 0.0f), pl.y + (k == 2 ? step : 0.0f), pl.z + (k == 3 ? step : 0.0f));
            const double r = S.sdf_all_forms ? sdf_form_dist(S, G.root, q) : sdf_node_dist(S, G.root, q);
            dd[0] = k == 0 ? r : dd[0];
            dd[1] = k == 1 ? r : dd[1];
            dd[2] = k == 2 ? r : dd[2];
            dd[3] = k == 3 ? r : dd[3];
        }
        const double dist0 = dd[0];
        const float nx = (float)((dd[1] - dist0) / G.normal_step);
        const float ny = (float)((dd[2] - dist0) / G.normal_step);
        const float nz = (float)((dd[3] - dist0) / G.normal_step);
        const SdfMD md = sdf_material(S, G.root, pl, four ? hab : nullptr);
        if (md.has_bc) { basecolor = md.bc; has_bc = 1; }
        if (md.has_uv) { u = md.u; v = md.v; has_uv = 1; }
        nrm = normalized(f3(nx, ny, nz));
        break;
    }
    default: break;
    }
    // normal = inv_transform.transposed().times(normal).to4(0).normalized()  (world.js:133-134)
    {
        const float wx = (float)((((double)nrm.x * inv[0] + (double)nrm.y * inv[4]) + (double)nrm.z * inv[8]) + (double)nrm_w * inv[12]);
        const float wy = (float)((((double)nrm.x * inv[1] + (double)nrm.y * inv[5]) + (double)nrm.z * inv[9]) + (double)nrm_w * inv[13]);
        const float wz = (float)((((double)nrm.x * inv[2] + (double)nrm.y * inv[6]) + (double)nrm.z * inv[10]) + (double)nrm_w * inv[14]);
        sf.N = normalized(f3(wx, or0(wy), or0(wz)));
    }
    sf.u = u;
    sf.v = v;
    sf.basecolor = basecolor;
    sf.bary = bary;
    sf.has_uv = has_uv;
    sf.has_bc = has_bc;
    sf.has_bary = has_bary;
}

// World.color hit branch up to the shadow casts: Primitive.color (world.js:125-137) +
// Geometry.materialData + Material.color (materials.js).  Fills the node (info, ambient / surface,
// shadow hand-off of its light samples) and returns its children (0..2) in evaluation order.
// A child whose diffuse direction came from an unstable spherePick (path_scatter's fix) sets INFO_FIX (never
// stored) and leaves in LDS, in column threadIdx.x of `fixl` [5][256]: fix0, fix1 (1 + the pick's RNG call,
// bit 31 = scattered about -N, the refraction side; 0 = none) and the node's N.  k_shade recomputes those
// directions at its tail (fix_child_dirs), so nothing of it is live in registers through the stores.
constexpr uint32_t INFO_FIX = 1u << 30;
template <int PF>
__device__ __forceinline__ int shade_node(const DScene &S, bool lit, const Hit &h, F3 o, F3 d, uint32_t addr,
                                          uint32_t key, NodeOut &out, Child &ch0, Child &ch1, uint32_t *fixl,
                                          bool force_fix) {
    const DPrim &P = S.prims[h.prim];
    Surface sf;
    surface_data<PF, false>(S, h, o, d, (S.mat_flags[P.material] & MATF_UV) != 0, sf);
    const F3 N = sf.N, basecolor = sf.basecolor;
    const float u = sf.u, v = sf.v;
    ShadeData sd;
    sd.pos = ray_point(o, d, h.t);  // material_data.position = ray.getPoint(distance)
    out.h.pos = sd.pos;
    out.h.addr = addr;
    out.h.key = key;
    const jsrt_rec_material &M = S.mat[P.material];
    const int mkind = (int)M.kind;
    Rng rng{key, addr, 0};
    if (mkind == JSRT_MAT_SOLID) {
        out.surf = mc_eval(S, M.color, u, v);
        out.info = INFO_HIT;
        return 0;
    }
    if (mkind == JSRT_MAT_TRANSPARENT) {  // materials.js:169-173
        out.surf = scale(mc_eval(S, M.color, u, v), M.opacity);
        ch0 = Child{d, f3(1, 1, 1), f3(1, 1, 1), 1 - M.opacity};
        out.info = INFO_HIT | (1u << INFO_NCHILD_SHIFT);
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
    out.surf = sd.ambient;
    uint32_t info = INFO_HIT;
    if (lit) {
        info |= INFO_LIT;
        out.h.N = sd.N;
        out.h.R = sd.R;
        out.h.refr = sd.refr;
        out.h.diff = sd.diff;
        out.h.spec = sd.spec;
        out.h.kr = sd.kr;
        out.h.mkind = mkind;
        out.h.mat = P.material;
        // the planes k_shadow needs beyond P, N (store_hand): a colour the material does not hold as a
        // constant, R unless the specular term is provably +0 (light_sample_color spec_zero), kr / refr
        // where kr != 1 (colorFromLightSample never reads refr with kr == 1, materials.js:349-354)
        const int32_t mf = S.mat_flags[P.material];
        uint32_t fl = 0;
        if (!(mf & MATF_DIFF_CONST) || sf.has_bc) fl |= HAND_DIFF;  // diff = basecolor x the diffuse chain
        if (!(mf & MATF_SPEC_CONST)) fl |= HAND_SPEC;
        if (mkind != JSRT_MAT_PHONG && sd.kr != 1.0) fl |= HAND_KR | HAND_R;
        if (!(mf & MATF_SPEC_ZERO) || !(__builtin_isfinite(sd.R.x) && __builtin_isfinite(sd.R.y) && __builtin_isfinite(sd.R.z)))
            fl |= HAND_R;
        out.h.flags = fl;
        rng.calls = (uint32_t)S.light_draws;
    }
    int n = 0;
    uint32_t fix0 = 0u, fix1 = 0u;
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
            uint32_t fx = 0;
            if (mkind == JSRT_MAT_PATH) ok = path_scatter(M.mirror_prob, true, sd.R, Nn, sd, rng, dir, col, fx, force_fix);
            if (ok) {
                fix0 = fx;  // the first child
                push(Child{dir, col, sd.refl, sd.kr});
            }
        }
        if (sd.kr < 1) {
            F3 dir = sd.refr, col = f3(1, 1, 1);
            bool ok = sd.has_refr;
            uint32_t fx = 0;
            if (mkind == JSRT_MAT_PATH) ok = path_scatter(M.mirror_prob, sd.has_refr, sd.refr, neg(Nn), sd, rng, dir, col, fx, force_fix);
            if (ok) {
                if (fx) {  // child n (0 when the reflection side pushed none)
                    if (n == 0) fix0 = fx | 0x80000000u;
                    else fix1 = fx | 0x80000000u;
                }
                push(Child{dir, col, sd.trans, 1 - sd.kr});
            }
        }
    }
    if (__builtin_expect((fix0 | fix1) != 0u, 0)) {
        const uint32_t t = threadIdx.x;
        fixl[t] = fix0;
        fixl[256 + t] = fix1;
        fixl[512 + t] = __float_as_uint(Nn.x);
        fixl[768 + t] = __float_as_uint(Nn.y);
        fixl[1024 + t] = __float_as_uint(Nn.z);
        info |= INFO_FIX;
    }
    out.info = info | ((uint32_t)n << INFO_NCHILD_SHIFT);
    return n;
}

// ---------------------------------------------------------------------------------------------
// Node / hand-off storage (AoS float4 records: one or two 16-B accesses per lane)
__device__ __forceinline__ float u2f(uint32_t x) { return __uint_as_float(x); }
__device__ __forceinline__ uint32_t f2u(float x) { return __float_as_uint(x); }

__device__ __forceinline__ void store_node(const WArgs &W, uint32_t i, F3 c, uint32_t info) {
    W.node[i] = make_float4(c.x, c.y, c.z, u2f(info));
}
__device__ __forceinline__ bool unit_child(const Child &c) {
    return c.w.x == 1.0f && c.w.y == 1.0f && c.w.z == 1.0f && c.k == 1.0;
}
__device__ __forceinline__ void store_child(const WArgs &W, uint32_t i, uint32_t j, const Child &c) {
    float4 *x = W.child + (size_t)(2 * j) * W.nstride + i;
    x[0] = make_float4(c.col.x, c.col.y, c.col.z, c.w.x);
    if (!unit_child(c))
        x[W.nstride] = make_float4(c.w.y, c.w.z, u2f((uint32_t)__double2loint(c.k)), u2f((uint32_t)__double2hiint(c.k)));
}
// ((v * col) * w) * k added to c: surface.plus(child.times(col).times(w).times(k)) (materials.js:277-330).
// info: the node's INFO_* word (INFO_UNIT0 / INFO_UNIT1: w = (1, 1, 1), k = 1, so the product is v * col).
__device__ __forceinline__ F3 add_child(const WArgs &W, uint32_t i, uint32_t j, F3 c, F3 v, uint32_t info,
                                       const float4 *first = nullptr) {  // first: the record's plane 0, if loaded
    const float4 *x = W.child + (size_t)(2 * j) * W.nstride + i;
    const float4 a = first ? *first : x[0];
    if (info & (j == 0 ? INFO_UNIT0 : INFO_UNIT1)) return add(c, mul(v, f3(a.x, a.y, a.z)));
    const float4 b = x[W.nstride];
    const double k = __hiloint2double((int)f2u(b.w), (int)f2u(b.z));
    return add(c, scale(mul(mul(v, f3(a.x, a.y, a.z)), f3(a.w, b.x, b.y)), k));
}
// Hand-off record of a lit node: float4 planes (plane stride hstride), two always and the rest as the
// node's material needs them (Handoff::flags, in the tag), plus the node index where the hand-off is
// bucketed (hnode[h], k_shadow's write-back address):
//   0 {P, h0 = mix(key, addr)}  1 {N, tag = mat << 8 | mask | HAND_*}
//   2 {diff} HAND_DIFF  3 {R, hi(kr)} HAND_R  4 {spec} HAND_SPEC  5 {refr, lo(kr)} HAND_KR
// A colour without its plane is the material's constant (S.mc_const); the material's kind and smoothness
// come from its record (S.mat).  cornell's walls need 36 B (80 B until round 4), its floor 68 B.
__device__ __forceinline__ void store_hand(const WArgs &W, uint32_t h, const Handoff &o) {
    float4 *p = W.hand + h;
    const size_t hs = W.hstride;
    const uint32_t fl = o.flags;
    const uint32_t tag = ((uint32_t)o.mat << 8) | (o.mask & 0xFFu) | fl;
    p[0] = make_float4(o.pos.x, o.pos.y, o.pos.z, u2f(mix32(o.key, o.addr)));
    p[hs] = make_float4(o.N.x, o.N.y, o.N.z, u2f(tag));
    if (fl & HAND_DIFF) p[2 * hs] = make_float4(o.diff.x, o.diff.y, o.diff.z, 0.0f);
    if (fl & HAND_R) p[3 * hs] = make_float4(o.R.x, o.R.y, o.R.z, u2f((uint32_t)__double2hiint(o.kr)));
    if (fl & HAND_SPEC) p[4 * hs] = make_float4(o.spec.x, o.spec.y, o.spec.z, 0.0f);
    if (fl & HAND_KR) p[5 * hs] = make_float4(o.refr.x, o.refr.y, o.refr.z, u2f((uint32_t)__double2loint(o.kr)));
    if (W.bucket) W.hnode[h] = o.node;
}

// per pixel, the renderer's f32 accumulation of one sample (renderers.js:93-97, 52-61)
__device__ __forceinline__ F3 accumulate(const RenderArgs &A, F3 acc, F3 col) {
    if (A.kind == JSRT_RENDERER_RANDOM) return add(acc, scale(col, 1.0 / A.spp));
    if (A.kind == JSRT_RENDERER_INCREMENTAL) return f3(acc.x + col.x, acc.y + or0(col.y), acc.z + or0(col.z));  // buffer.plus(c.to4(true))
    return col;
}

// ---------------------------------------------------------------------------------------------
// profile-independent kernels (render.hip) launched by run_batch
__global__ __launch_bounds__(256) void k_gen(DScene S, RenderArgs A, WArgs W);
__global__ __launch_bounds__(256) void k_reduce(WArgs W, int L);
__global__ __launch_bounds__(256) void k_accum(RenderArgs A, WArgs W);
__global__ __launch_bounds__(256) void k_resolve(RenderArgs A, WArgs W);
__global__ __launch_bounds__(256) void k_resolve_side(RenderArgs A, WArgs W, int s);
__global__ __launch_bounds__(256) void k_resolve_paths(RenderArgs A, WArgs W);

// Grid of a persistent kernel: as many 256-thread blocks as the device keeps resident (occupancy x
// CUs), never more than the work needs (render.hip).
unsigned persistent_grid(const void *kernel, size_t work);
inline unsigned grid(size_t n) { return (unsigned)((n + 255) / 256); }
inline unsigned grid_ub(size_t n) { return (unsigned)std::max<size_t>(1, (n + 255) / 256); }

// Bucketed shadow hand-off (WArgs::bucket = shift + 1): the lit nodes of level L are written grouped
// by hit primitive (bucket prim >> shift: one primitive each in a flat scene, runs of consecutive
// triangles in a mesh; within a bucket by slice), so the 64 lanes of a k_shadow wave serve nodes on
// one surface: their shadow rays cull the same objects and walk the same BVH nodes, and their
// materials take the same branches.  Only the order k_shadow visits nodes in changes.
static_assert(BKT_N == 64, "k_extend's last wave flushes one bucket per lane");
// The bucketed hand-off (and the block appends' 64-bit ballots) assume 64-lane waves (gfx950).
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "the wavefront renderer needs wave64 (build for gfx950)"
#endif
__device__ __forceinline__ int bucket_key(const WArgs &W, int bucket) {  // counter of (bucket, this block's slice)
    return bucket * BKT_S + (int)(blockIdx.x % BKT_S);
}

// Closest hit (World.cast, world.js:28-30).  Chain: ray q of the batch; tree: level L's range.
template <int PF, bool CHAIN>
__global__ __launch_bounds__(256, PF == PF_ANALYTIC ? JSRT_EXTEND_OCC_FLAT : JSRT_EXTEND_OCC) void k_extend(DScene S, WArgs W, int L,
                                                                                                 double minD) {
    __shared__ uint32_t hist[BKT_N], waves_done;  // bucketed hand-off: the block's lit hits per bucket
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t i = t;
    bool live = true;
    {
        // chain: ray slot t of the level's live slots; tree: level L's range of the pool
        const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
        const uint32_t rbase = CHAIN ? 0u : R.base;
        if ((!CHAIN || W.hybrid) && t == 0 && R.count > gridDim.x * 256u) W.lvl[LVL_UNDER] = 1u;  // launch bound too small
        if (!W.bucket) {
            if (t >= R.count) return;
        } else {  // every wave of a live block reaches the count below
            if (blockIdx.x * 256u >= R.count) return;  // block-uniform
            if (threadIdx.x < BKT_N) hist[threadIdx.x] = 0u;
            if (threadIdx.x == 0) waves_done = 0u;
            __syncthreads();
            live = t < R.count;
        }
        i = rbase + (live ? t : 0u);
        if (CHAIN) i = live ? chain_slot(W, L, t) : 0u;
    }
    int hp = -1, b = 0;  // b: the hit's bucket
    // the ray is loaded together with its prim word (one memory round trip, not two dependent ones)
    const int32_t pin = W.prim[i];
    const F3 o = f3(W.ox[i], W.oy[i], W.oz[i]), d = f3(W.dx[i], W.dy[i], W.dz[i]);
    if (live && pin != NO_RAY) {
        const Hit h = world_cast<PF, false>(S, o, d, minD, DINF, true);
        W.t[i] = h.t;
        W.prim[i] = h.prim;
        W.ctx[i] = h.ctx;
        hp = h.prim;
        // grid bucket: the cell of the hit point in f32 (within ~1e-6 of material_data.position, which
        // scene_load.cpp shadow_grid's grown cells cover; k_shade reads the bucket back from brank)
        if (W.bucket && hp >= 0) {
            const float tf = (float)h.t;
            b = W.bucket_grid ? grid_cell(S, f3(fmaf(d.x, tf, o.x), fmaf(d.y, tf, o.y), fmaf(d.z, tf, o.z)))
                              : hp >> (W.bucket - 1);
        }
    }
    if (W.bucket) {
        // Bucketed hand-off: ranks every lit hit (S.prim_lit: shade_node lights every hit but Solid /
        // Transparent) among the block's hits in its bucket (wave-aggregated LDS atomics); the
        // block's last wave adds the histogram to the level's per-key counters (one global atomic per
        // bucket per block, keys spread over BKT_S slices) and keeps the block's bases.  No barrier
        // waits for the block's slowest cast, and the atomics overlap other blocks' casts (as a
        // separate pass they cost cornell 30 ms per frame, r02_s16).
        const bool lit = hp >= 0 && S.prim_lit[hp] != 0;
        const int lane = (int)__lane_id();
        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        // one LDS atomic per distinct bucket of the wave (a few hot buckets would serialise), issued by the bucket's
        // first lane: the loop only finds each lane's leader and rank (no memory operation in it), then the leaders'
        // atomics go out as ONE instruction to distinct addresses and each lane reads its leader's base (round 6:
        // the loop had waited for one atomic's return per distinct bucket, ~25 per wave of scattered hits)
        uint64_t todo = __ballot(lit);
        int leader = lane;
        uint32_t rk = 0, cnt = 0;
        while (todo) {
            const int first = __builtin_ctzll(todo);
            const int bv = __builtin_amdgcn_readlane(b, first);
            const uint64_t m = __ballot(lit && b == bv);
            if (lit && b == bv) {
                leader = first;
                rk = (uint32_t)__popcll(m & lt);
            }
            if (lane == first) cnt = (uint32_t)__popcll(m);
            todo &= ~m;
        }
        uint32_t base = 0;
        if (lit && lane == leader) base = atomicAdd(&hist[b], cnt);
        base = (uint32_t)__shfl((int)base, leader);
        if (lit) W.brank[i] = ((uint32_t)b << 16) | (base + rk);
        __threadfence_block();
        uint32_t done = 0;
        if (lane == 0) done = atomicAdd(&waves_done, 1u);
        if (__shfl(done, 0) == 256u / 64u - 1u) {  // the block's last wave: BKT_N == 64 lanes flush
            __threadfence_block();
            const uint32_t c = hist[lane];
            if (c) W.bbase[(size_t)blockIdx.x * BKT_N + lane] = atomicAdd(W.bkt + (size_t)L * BKT_LEVEL + bucket_key(W, lane), c);
        }
    }
}

// Offsets of the level's hand-off keys: an exclusive prefix over the k_extend counts (key order =
// bucket-major), and the level's lit-node total.  One block.
__global__ __launch_bounds__(256) void k_bucket_offsets(WArgs W, int L);

// World.color at level L (world.js:31-41): a miss is bg_color, a hit is shaded (shade_node).
// Chain schedule (every node has <= 1 child): node L*P + q, its child ray replaces ray q.
// Tree schedule: node = pool slot; children are appended to level L + 1 (block-aggregated).
// A node with unstable spherePicks (INFO_FIX): its record for k_fix_dirs (rare: about one pick in 10^5), with
// the ray slots its children's directions went to.  Out of records (never: fixcap is 1/8 of the level's
// slots), the frame is redone with a larger pool, as for any other capacity.
__device__ __forceinline__ void fix_record(const WArgs &W, const uint32_t *fixl, uint32_t key, uint32_t addr,
                                           int nchild, uint32_t d0, uint32_t d1) {
    const uint32_t t = threadIdx.x;
    const uint32_t k = atomicAdd(W.fixctr, 1u);
    if (k >= W.fixcap) {
        W.lvl[LVL_FLAG] = 1u;
        return;
    }
    uint4 *r = W.fixrec + 3 * (size_t)k;
    r[0] = make_uint4(d0, d1, key, addr);
    r[1] = make_uint4(fixl[t], fixl[256 + t], (uint32_t)nchild, 0u);
    r[2] = make_uint4(fixl[512 + t], fixl[768 + t], fixl[1024 + t], 0u);
}

// The child directions of the level's unstable spherePicks, recomputed with V8's sin / cos / acos (fdlibm.h)
// from each pick's own draws and stored over the OCML direction k_shade wrote: a separate one-block kernel
// after k_shade, so the fdlibm code is not part of k_shade (inline there it cost ~50 spilled VGPRs, as a call
// a 416-B stack frame per lane; either slowed k_shade 25 % to 4x, profiles/r04_s10_ab.txt, r04_s11_ab.txt).
__global__ __launch_bounds__(256) void k_fix_dirs(WArgs W);

// DScene::stab: the per-hit tables in LDS (`lds`, a copy of the image or of k_shadow's prefix of it) bound in the
// kernel's own DScene copy in place of the global ones
__device__ __forceinline__ void stab_bind(DScene &SL, const uint4 *lds, bool shade) {
    const char *sb = reinterpret_cast<const char *>(lds);
    SL.mat = reinterpret_cast<const jsrt_rec_material *>(sb + SL.stab_off[STAB_MAT]);
    SL.mat_flags = reinterpret_cast<const int32_t *>(sb + SL.stab_off[STAB_MAT_FLAGS]);
    SL.mc = reinterpret_cast<const jsrt_rec_mcolor *>(sb + SL.stab_off[STAB_MC]);
    SL.mc_const = reinterpret_cast<const float *>(sb + SL.stab_off[STAB_MC_CONST]);
    SL.sample_call = reinterpret_cast<const int32_t *>(sb + SL.stab_off[STAB_SAMPLE_CALL]);
    SL.sample_light = reinterpret_cast<const int32_t *>(sb + SL.stab_off[STAB_SAMPLE_LIGHT]);
    if (!shade) return;
    SL.prims = reinterpret_cast<const DPrim *>(sb + SL.stab_off[STAB_PRIMS]);
    SL.prim_shade = reinterpret_cast<const int32_t *>(sb + SL.stab_off[STAB_PRIM_SHADE]);
    SL.shade0 = reinterpret_cast<const double *>(sb + SL.stab_off[STAB_SHADE0]);
    SL.shadeI = reinterpret_cast<const double *>(sb + SL.stab_off[STAB_SHADEI]);
    SL.prim_lit = reinterpret_cast<const int32_t *>(sb + SL.stab_off[STAB_PRIM_LIT]);
}

// STAGE (flat scenes whose shading tables fit, DScene::stab): the tables are copied into LDS by every block, so a
// hit's dependent record chain (prim -> shading matrix / material -> colour constants) is LDS round trips
template <int PF, bool CHAIN, bool STAGE>
__global__ __launch_bounds__(256, PF == PF_ANALYTIC ? JSRT_SHADE_OCC_FLAT
                                                    : (PF & PF_SDF) ? JSRT_SHADE_OCC_SDF : JSRT_SHADE_OCC) SHADE_ATTR void k_shade(
    DScene S, WArgs W, int L, int child_depth) {
    XST_BEGIN
    const uint32_t t0 = blockIdx.x * 256, tt = t0 + threadIdx.x;
    const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
    const uint32_t count = R.count, base = R.base, next_base = CHAIN ? 0u : R.base + R.count;
    if (!CHAIN || W.hybrid || STAGE) {
        if (t0 >= count) return;  // block-uniform: every thread of a live block reaches block_append / the barrier
    } else if (tt >= count) {
        return;
    }
#ifdef JSRT_SHADE_SORT
    // (A/B) the block's nodes permuted by hit primitive through LDS (a counting sort on min(prim, 62), misses
    // and idle lanes last), so a wave shades nodes of one or two primitives: one geometry branch, one material
    __shared__ uint32_t s_cnt[64], s_perm[256];
    uint32_t tq = tt;
    if (!CHAIN || W.hybrid) {  // (kernel argument: block-uniform; the plain chain returns per thread above)
        uint32_t key = 63u;
        if (tt < count) {
            const uint32_t s0 = CHAIN ? chain_slot(W, L, tt) : tt;
            const int p0 = W.prim[CHAIN ? s0 : base + tt];
            key = p0 >= 0 ? (uint32_t)(p0 < 62 ? p0 : 62) : 63u;
        }
        if (threadIdx.x < 64) s_cnt[threadIdx.x] = 0u;
        __syncthreads();
        const uint32_t rank = atomicAdd(&s_cnt[key], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the 64 counts in one wave
            const uint32_t c = s_cnt[threadIdx.x];
            uint32_t x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o);
                if ((int)threadIdx.x >= o) x += y;
            }
            s_cnt[threadIdx.x] = x - c;
        }
        __syncthreads();
        s_perm[s_cnt[key] + rank] = threadIdx.x;
        __syncthreads();
        tq = t0 + s_perm[threadIdx.x];
    }
    const bool in = tq < count;
    const uint32_t q = in ? tq : 0u;                          // level index
#else
    const bool in = tt < count;
    const uint32_t q = in ? tt : 0u;                          // level index
#endif
    const uint32_t slot = CHAIN && in ? chain_slot(W, L, q) : q;  // chain: the chain's slot
    const uint32_t i = base + (CHAIN ? slot : q);             // node index (chain: L * cap + slot)
    const uint32_t r = CHAIN ? slot : i;                      // ray index
    int nchild = 0;
    Child ch0, ch1;
    NodeOut out;
    __shared__ uint32_t fixl[5 * 256];  // shade_node's unstable spherePicks (INFO_FIX)
    const int prim = in ? W.prim[r] : NO_RAY;
    const bool hit = prim >= 0;
    // STAGE: the ray (and its hit) loaded before the staging barrier, so the two latencies overlap (without it
    // the loads stay under `hit`: hoisted there they cost the mesh / SDF k_shade ~40 spilled VGPRs)
    F3 ro = f3(0, 0, 0), rd = f3(0, 0, 0);
    double rt = 0;
    int32_t rctx = 0;
    uint32_t raddr = 0, rkey = 0;
    if (STAGE && in) {
        ro = f3(W.ox[r], W.oy[r], W.oz[r]);
        rd = f3(W.dx[r], W.dy[r], W.dz[r]);
        rt = W.t[r];
        rctx = W.ctx[r];
        raddr = W.addr[r];
        rkey = W.key[r];
    }
    DScene SL = S;
    if constexpr (STAGE) {
        extern __shared__ uint4 stab_lds[];
        const uint4 *src = reinterpret_cast<const uint4 *>(S.stab);
        for (int k = (int)threadIdx.x; k < S.stab_words; k += 256) stab_lds[k] = src[k];
        __syncthreads();
        stab_bind(SL, stab_lds, true);
    }
    XST(0, prim);
    // Every load, and the children's append (a returning atomic), is issued before the node's first
    // store: vmcnt counts stores too, in issue order, so a load or atomic issued behind the node's
    // ~20 HBM stores would wait for all of them to complete.
    uint32_t parent = 0, path = 0, hslot = ~0u;
    if (!CHAIN && prim != NO_RAY) {
        parent = W.parent[r];
        path = W.path[r];
    }
    if (hit) {
        if (!STAGE) {
            ro = f3(W.ox[r], W.oy[r], W.oz[r]);
            rd = f3(W.dx[r], W.dy[r], W.dz[r]);
            rt = W.t[r];
            rctx = W.ctx[r];
            raddr = W.addr[r];
            rkey = W.key[r];
        }
        const Hit h{rt, prim, rctx};
        nchild = shade_node<PF>(SL, W.ns > 0, h, ro, rd, raddr, rkey, out, ch0, ch1, fixl, W.force_fix != 0);
        out.h.node = CHAIN ? slot : q;  // (k_shadow: node base + this)
        out.h.mask = (uint32_t)S.grid_cells;  // every root
        if (W.bucket && (out.info & INFO_LIT)) {  // the lit node's hand-off slot, ranked by k_extend
            const uint32_t br = W.brank[r];      // bucket << 16 | rank in the block's bucket
            const int b = (int)(br >> 16);
            const uint32_t *B = W.bkt + (size_t)L * BKT_LEVEL;
            hslot = B[2 * BKT_K + bucket_key(W, b)] + W.bbase[(size_t)blockIdx.x * BKT_N + b] + (br & 0xFFFFu);
            if (hslot >= B[3 * BKT_K]) hslot = ~0u;  // (never: k_extend counted this node)
            if (W.bucket_grid) out.h.mask = (uint32_t)b;
        }
    }
    XST(1, out.info);
    // tree: children append to level L + 1; at depth 0 they are black without a cast
    // W.child_sort: a block's children grouped by direction octant, so a wave of the next level's k_extend
    // casts rays of one or two octants that walk the same BVH subtrees (WArgs::child_sort)
    uint32_t co[2] = {0u, 1u};  // offsets of the children from `at`
    uint32_t at = 0, side_at = 0;
    if (!CHAIN) {
        const int nc = child_depth > 0 ? nchild : 0;
        if (W.child_sort)  // (kernel argument: block-uniform, every thread reaches the barriers)
            at = block_append_keyed(W.lvl + L + 1, nc, nchild > 0 ? octant(ch0.dir) : 0, nchild > 1 ? octant(ch1.dir) : 0,
                                    co[0], co[1]);
        else
            at = block_append<256>(W.lvl + L + 1, nc);
    } else if (W.hybrid) {
        // the chain continues into level L + 1 (its first child: an entry in level L + 1's list), and a
        // second child starts a side chain, the next id of the side chains started at L + 1 (after npaths and
        // those started at levels 1..L: read here, before the first store, as a load behind the stores would
        // wait for all of them)
        const int side = (child_depth > 0 && nchild > 1) ? 1 : 0, cont = (child_depth > 0 && nchild > 0) ? 1 : 0;
        block_append2(W.lvl + 2 * (L + 1), cont, side, at, side_at);
        side_at += side_base(W, L + 1);
    }
    XST(2, side_at);
    // unstable spherePicks: the record for k_fix_dirs, with the slots the children's rays go to below (written
    // before the node's stores, behind which the returning atomic would wait for all of them)
    if (__builtin_expect(hit && (out.info & INFO_FIX) != 0u, 0) && child_depth > 0) {
        if (CHAIN) fix_record(W, fixl, out.h.key, out.h.addr, W.hybrid ? nchild : 1, r, side_at);
        else fix_record(W, fixl, out.h.key, out.h.addr, nchild, next_base + at + co[0], next_base + at + co[1]);
    }
    // ---- stores ----
    if (prim == NO_RAY) {
        if (in) store_node(W, i, f3(0, 0, 0), 0u);
        if (CHAIN && W.hybrid && in) W.endl[r] = (uint8_t)L;
        return;
    }
    if (!hit) {  // miss: World.color returns bg_color (world.js:35-36)
        const F3 bg = f3(S.bg[0], S.bg[1], S.bg[2]);
        if (CHAIN) {
            store_node(W, i, bg, INFO_MISS);
            W.prim[r] = NO_RAY;
            if (W.hybrid) W.endl[r] = (uint8_t)L;
        } else {
            if (parent == NO_PARENT) {  // write_result with the preloaded parent / path
                float *dst = W.root + 3 * (size_t)path;
                dst[0] = bg.x;
                dst[1] = bg.y;
                dst[2] = bg.z;
            } else if (parent != DEAD_RAY) {
                W.slot[(size_t)(parent & 1u) * W.nstride + (parent >> 1)] = make_float4(bg.x, bg.y, bg.z, 0.0f);
            }
            store_node(W, i, bg, 0u);
        }
        return;
    }
    if (nchild > 0 && unit_child(ch0)) out.info |= INFO_UNIT0;
    if (nchild > 1 && unit_child(ch1)) out.info |= INFO_UNIT1;
    // (JSRT_X_*: timing-only experiments that drop one class of k_shade's stores; the image is wrong)
#ifndef JSRT_X_NONODE
    store_node(W, i, out.surf, out.info & ~INFO_FIX);
#endif
#ifndef JSRT_X_NOHAND
    // (The record at the node's own index -- coalesced 16-B stores -- with k_shadow gathering it through hnode:
    // k_shade -1.5 ms, k_shadow +2.9 ms per cornell frame, profiles/r05_s5_s6_ab.txt; the scatter stays here.)
    if (out.info & INFO_LIT) {
        if (!W.bucket) store_hand(W, q, out.h);
        else if (hslot != ~0u) store_hand(W, hslot, out.h);
    }
#endif
#ifndef JSRT_X_NONODE
    if (nchild > 0) store_child(W, i, 0, ch0);
    if (nchild > 1) store_child(W, i, 1, ch1);
#endif
    if (CHAIN) {  // the child ray (World.color(child, depth - 1)) takes over slot q
        uint32_t *next = (L & 1) ? W.list0 : W.list1;  // level L + 1's list
        if (child_depth > 0 && nchild > 0) {
#ifndef JSRT_X_NORAY
            W.ox[r] = out.h.pos.x; W.oy[r] = out.h.pos.y; W.oz[r] = out.h.pos.z;
            W.dx[r] = ch0.dir.x; W.dy[r] = ch0.dir.y; W.dz[r] = ch0.dir.z;
            W.addr[r] = mix32(out.h.addr, 1u);
#endif
            if (W.hybrid) next[at] = r;
        } else {
            W.prim[r] = NO_RAY;  // no child, or children black without a cast (depth 0)
            if (W.hybrid) W.endl[r] = (uint8_t)L;
        }
        if (W.hybrid && child_depth > 0 && nchild > 1) {  // the second child's side chain
            const uint32_t c = side_at;  // npaths + side(< L + 1) + this chain's offset
            if (c >= W.cap) {
                W.lvl[LVL_FLAG] = 1u;  // out of chain slots: the host redoes the frame with more
                return;
            }
            W.ox[c] = out.h.pos.x; W.oy[c] = out.h.pos.y; W.oz[c] = out.h.pos.z;
            W.dx[c] = ch1.dir.x; W.dy[c] = ch1.dir.y; W.dz[c] = ch1.dir.z;
            W.addr[c] = mix32(out.h.addr, 2u);
            W.key[c] = out.h.key;
            W.parent[c] = i;
            W.prim[c] = -1;
        }
#ifdef JSRT_X_STAMPS
        __builtin_amdgcn_s_waitcnt(0);  // (the stores retired)
        XST(3, r);
#endif
        return;
    }
    if (nchild == 0) return;
    if (child_depth == 0) {
        W.slot[i] = make_float4(0, 0, 0, 0);
        if (nchild > 1) W.slot[W.nstride + i] = make_float4(0, 0, 0, 0);
        return;
    }
    const uint32_t last = at + (nchild > 1 ? (co[0] > co[1] ? co[0] : co[1]) : co[0]);
    if ((size_t)last + 1 > W.level_cap || (size_t)next_base + last + 1 > W.pool) {
        W.lvl[LVL_FLAG] = 1u;  // outgrew the pool: the host redoes the frame with a larger one
        return;
    }
    for (int j = 0; j < nchild; ++j) {
        const Child &c = j == 0 ? ch0 : ch1;
        const uint32_t rr = next_base + at + co[j];
        W.ox[rr] = out.h.pos.x; W.oy[rr] = out.h.pos.y; W.oz[rr] = out.h.pos.z;
        W.dx[rr] = c.dir.x; W.dy[rr] = c.dir.y; W.dz[rr] = c.dir.z;
        W.addr[rr] = mix32(out.h.addr, (uint32_t)j + 1);
        W.key[rr] = out.h.key;
        W.path[rr] = path;
        W.parent[rr] = 2 * i + (uint32_t)j;
        W.prim[rr] = -1;
    }
}

// The light samples of the lit nodes of level L (lights.js sampleIterator), their shadow casts
// (materials.js:250-252), colorFromLightSample (materials.js:261-269, 340-356) and the
// colorFromLights sums (materials.js:244-257), which turn the node's ambient into its surface.
// W.group lanes serve one node (sample s on lane s, a power of two >= ns); the node's first lane
// adds the samples in the reference's order from its neighbours' registers.  SERIAL (more than 64
// samples per node, group 1): one lane per node walks all samples itself.
// One light sample of a lit node without its shadow cast: the light sample (lights.js), its
// unshadowed colour (colorFromLightSample) and the shadow ray (origin P = the hit point, direction
// delta, accepted distances (1e-4, 1), materials.js:250-252).
__device__ __forceinline__ F3 mc_const3(const DScene &S, int m) {  // a constant colour chain's value
    const float4 c = *reinterpret_cast<const float4 *>(S.mc_const + 4 * m);
    return f3(c.x, c.y, c.z);
}
template <int PF, bool SPH = true>
__device__ __forceinline__ F3 sample_unshadowed(const DScene &S, const float4 &h0, const float4 &h1, const float4 *hp,
                                                size_t hs, uint32_t s, F3 &P, F3 &delta) {
    P = f3(h0.x, h0.y, h0.z);
    RngH rng{f2u(h0.w), (uint32_t)S.sample_call[s]};
    F3 L, lcol;
    if (S.n_lights == 1)  // (kernel argument: uniform) the light record through scalar loads
        light_sample<SPH>(S, as_const(S.lights)[0], P, rng, delta, L, lcol);
    else
        light_sample<SPH>(S, S.lights[S.sample_light[s]], P, rng, delta, L, lcol);
    const uint32_t tag = f2u(h1.w);
    const jsrt_rec_material &M = S.mat[(tag & HAND_MAT) >> 8];
    ShadeData sd;
    sd.N = f3(h1.x, h1.y, h1.z);
    sd.diff = (tag & HAND_DIFF) ? f3(hp[2 * hs].x, hp[2 * hs].y, hp[2 * hs].z) : mc_const3(S, M.diffuse);
    sd.spec = (tag & HAND_SPEC) ? f3(hp[4 * hs].x, hp[4 * hs].y, hp[4 * hs].z) : mc_const3(S, M.specular);
    sd.R = f3(0, 0, 0);
    sd.refr = f3(0, 0, 0);
    sd.kr = 1.0;
    if (tag & HAND_R) {
        const float4 h3 = hp[3 * hs];
        sd.R = f3(h3.x, h3.y, h3.z);
        if (tag & HAND_KR) {
            const float4 h5 = hp[5 * hs];
            sd.refr = f3(h5.x, h5.y, h5.z);
            sd.kr = __hiloint2double((int)f2u(h3.w), (int)f2u(h5.w));
        }
    }
    sd.smoothness = M.smoothness;
    return light_sample_color((int)M.kind, sd, L, lcol, !(tag & HAND_R));
}

__device__ __forceinline__ bool shadowed(const Hit &sh) { return sh.prim >= 0 && sh.t > 0 && sh.t < 1; }

template <int PF, bool SPH = true>
__device__ __forceinline__ F3 sample_unshadowed(const DScene &S, const float4 *hp, size_t hs, uint32_t s, F3 &P, F3 &delta) {
    return sample_unshadowed<PF, SPH>(S, hp[0], hp[hs], hp, hs, s, P, delta);
}

// FLAT: the flat shadow loop (device_common.h shadow_cast_flat; `mask` is over DScene::sroot records)
template <int PF, bool SPH = true, bool FLAT = false>
__device__ __forceinline__ F3 sample_color(const DScene &S, const float4 &h0, const float4 &h1, const float4 *hp,
                                           size_t hs, uint32_t s, uint64_t mask = ~0ull) {
    F3 P, delta;
    const F3 c = sample_unshadowed<PF, SPH>(S, h0, h1, hp, hs, s, P, delta);
    // A shadowed sample contributes +0.  An unshadowed one whose colour is +-0 in every component
    // (the light behind the surface, a black material, an edge-on area light) adds the same
    // nothing to colorFromLights' running sum (+0 + -0 = +0), so its shadow cast is skipped.
    if (c.x == 0.0f && c.y == 0.0f && c.z == 0.0f) return f3(0, 0, 0);
#ifdef JSRT_X_NOCAST  // (timing experiment only) no shadow cast: every sample unshadowed
    if (delta.x != 12345.0f) return c;
#endif
    if constexpr (FLAT) {
        if (shadow_cast_flat(S, P, delta, 0.0001, 1, mask)) return f3(0, 0, 0);  // shadowed: contributes +0
        return c;
    }
    const Hit sh = world_cast<PF, true>(S, P, delta, 0.0001, 1, false, mask);
    if (shadowed(sh)) return f3(0, 0, 0);  // shadowed: contributes +0
    return c;
}

// colorFromLights: per light, its samples in order (a shadowed sample adds +0, which never changes
// an f32 running sum that starts at +0), times 1/samples, added to the ambient `ret`.  Sample s of
// the node sits on lane (lane & ~(G - 1)) + s; every lane takes part in the shuffles.
__device__ __forceinline__ F3 light_sums(const DScene &S, uint32_t G, F3 ret, F3 c) {
    const int lane0 = (int)(__lane_id() & ~(G - 1));
    uint32_t k = 0;
    for (int li = 0; li < S.n_lights; ++li) {
        const DLight &Lt = S.lights[li];
        const int n = Lt.kind == JSRT_LIGHT_POINT ? 1 : Lt.samples;
        F3 light_color = f3(0, 0, 0);
        for (int j = 0; j < n; ++j, ++k) {
            const int src = lane0 + (int)k;
            light_color = add(light_color, f3(__shfl(c.x, src), __shfl(c.y, src), __shfl(c.z, src)));
        }
        if (n > 0) ret = add(ret, scale(light_color, Lt.inv_n));  // times(1 / samples)
    }
    return ret;
}

// STAGE (flat scenes, DScene::stab; not SERIAL): k_shadow's tables (materials, colour constants, light-sample
// indices) copied into LDS by every block behind its hand-off loads, so a sample's material -> colour chain is
// LDS round trips
// FLAT (with STAGE; DScene::n_sroot > 0): the shadow casts through the flat shadow loop (shadow_cast_flat)
template <int PF, bool CHAIN, bool SERIAL, bool SPH, bool STAGE = false, bool FLAT = false>
__global__ __launch_bounds__(256, PF == PF_ANALYTIC ? JSRT_SHADOW_OCC_FLAT : JSRT_SHADOW_OCC) SHADOW_ATTR void k_shadow(
    DScene S, WArgs W, int L) {
    const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
    const uint32_t count = R.count, base = R.base;
    const uint32_t G = (uint32_t)W.group, ns = (uint32_t)W.ns;
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    uint32_t q = e / G;  // G is a power of two
    const uint32_t s = e % G;
    bool in = q < count;
    const float4 *hp = W.hand + (in ? q : 0u);
    uint32_t mi = 0;  // the node's shadow-root mask (grid cell of its hit point)
    if (W.bucket) {  // hand-off slot q of the level's lit nodes (all filled)
        in = q < as_const(W.bkt + (size_t)L * BKT_LEVEL)[3 * BKT_K];
        const uint32_t h = in ? q : 0u;
        q = W.hnode[h];
        mi = f2u(hp[W.hstride].w) & 0xFFu;
    }
    // Shadow-root mask of the wave (scene_load.cpp shadow_grid): when every node of the wave has its hit
    // point in one grid cell -- the hand-off is bucketed by cell, so nearly every wave -- the world loop
    // visits only the roots a shadow segment from that cell can meet.
    uint64_t mask = ~0ull;
    if (FLAT) mask = S.n_sroot >= 64 ? ~0ull : ((1ull << S.n_sroot) - 1);  // every record
    if (W.bucket && W.bucket_grid && S.grid_masked) {
        const uint64_t on = __ballot(in);
        if (on) {
            const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)mi, __builtin_ctzll(on));
            if (!__ballot(in && mi != m0) && m0 <= (uint32_t)S.grid_cells)
                mask = FLAT ? as_const(S.grid_smask)[m0] : as_const(S.grid_mask)[m0];
        }
    }
    if (CHAIN && !W.bucket && in) q = chain_slot(W, L, q);  // hand-off in level order: the chain's slot
    const uint32_t i = base + (in ? q : 0u);
    const float4 nd = W.node[i];
    const bool lit = in && (f2u(nd.w) & INFO_LIT);
    F3 ret = f3(nd.x, nd.y, nd.z);  // ambient
    if (SERIAL) {  // one lane per node: every sample in order
        if (!lit) return;
        uint32_t k = 0;
        for (int li = 0; li < S.n_lights; ++li) {
            const DLight &Lt = S.lights[li];
            const int n = Lt.kind == JSRT_LIGHT_POINT ? 1 : Lt.samples;
            F3 light_color = f3(0, 0, 0);
            for (int j = 0; j < n; ++j, ++k)
                light_color = add(light_color, sample_color<PF, SPH>(S, hp[0], hp[W.hstride], hp, W.hstride, k, mask));
            if (n > 0) ret = add(ret, scale(light_color, Lt.inv_n));  // times(1 / samples)
        }
        W.node[i] = make_float4(ret.x, ret.y, ret.z, nd.w);
        return;
    }
    F3 c = f3(0, 0, 0);
    const float4 h0 = hp[0], h1 = hp[W.hstride];  // (loaded by every lane: before the staging barrier)
    if constexpr (STAGE) {
        extern __shared__ uint4 stab_lds[];
        const uint4 *src = reinterpret_cast<const uint4 *>(S.stab);
        for (int k = (int)threadIdx.x; k < S.stab_words_shadow; k += 256) stab_lds[k] = src[k];
        __syncthreads();
        DScene SL = S;
        stab_bind(SL, stab_lds, false);
        if (lit && s < ns) c = sample_color<PF, SPH, FLAT>(SL, h0, h1, hp, W.hstride, s, mask);
    } else {
        if (lit && s < ns) c = sample_color<PF, SPH>(S, h0, h1, hp, W.hstride, s, mask);
    }
    ret = light_sums(S, G, ret, c);
    if (lit && s == 0) W.node[i] = make_float4(ret.x, ret.y, ret.z, nd.w);
}

// ---------------------------------------------------------------------------------------------
// Persistent casts for SDF scenes (device_common.h persistent_cast): same results as k_extend /
// k_shadow, with lanes refilled from a work counter while other lanes keep marching.
struct ExtendSrc {  // the level's rays (k_extend's inputs and outputs)
    const WArgs &W;
    uint32_t base;
    int L;  // chain schedule: >= 0, ray j is the level's j-th chain (chain_slot); tree: -1, ray base + j
    __device__ __forceinline__ uint32_t ray(uint32_t j) const { return L >= 0 ? chain_slot(W, L, j) : base + j; }
    __device__ __forceinline__ bool load(uint32_t j, F3 &o, F3 &d) const {
        const uint32_t i = ray(j);
        if (W.prim[i] == NO_RAY) return false;
        o = f3(W.ox[i], W.oy[i], W.oz[i]);
        d = f3(W.dx[i], W.dy[i], W.dz[i]);
        return true;
    }
    __device__ __forceinline__ void store(uint32_t j, const Hit &h) const {
        const uint32_t i = ray(j);
        W.t[i] = h.t;
        W.prim[i] = h.prim;
        W.ctx[i] = h.ctx;
    }
};

template <int PF, bool CHAIN, bool FO>
__global__ __launch_bounds__(256, JSRT_MARCH_OCC) void k_extend_q(DScene S, WArgs W, int L, double minD) {
    const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
    const uint32_t count = R.count, base = CHAIN ? 0u : R.base;  // ray slots
    ExtendSrc src{W, base, CHAIN ? L : -1};
    persistent_cast<PF, false, FO>(S, W.qctr + L, count, minD, DINF, true, src);
}

struct ShadowSrc {  // the light samples' shadow rays written by k_shadow_prep
    const WArgs &W;
    __device__ __forceinline__ bool load(uint32_t e, F3 &o, F3 &d) const {
        const float4 c = W.scol[e];
        if (f2u(c.w) != 1u) return false;
        const float4 a = W.sray[e], b = W.sray[W.sstride + e];
        o = f3(a.x, a.y, a.z);
        d = f3(b.x, b.y, b.z);
        return true;
    }
    __device__ __forceinline__ void store(uint32_t e, const Hit &h) const {
        if (shadowed(h)) W.scol[e].w = u2f(2u);
    }
};

// k_shadow's lane layout (node q on lanes [q * G, q * G + G), sample s on lane s): the unshadowed
// colour and shadow ray of every light sample
template <int PF, bool CHAIN>
__global__ __launch_bounds__(256) void k_shadow_prep(DScene S, WArgs W, int L) {
    const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
    const uint32_t count = R.count, base = R.base;
    const uint32_t G = (uint32_t)W.group, ns = (uint32_t)W.ns;
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    const uint32_t q = e / G, s = e % G;
    if (q >= count || s >= ns) return;
    const float4 nd = W.node[base + (CHAIN ? chain_slot(W, L, q) : q)];
    if (!(f2u(nd.w) & INFO_LIT)) return;
    F3 P, delta;
    const F3 c = sample_unshadowed<PF>(S, W.hand + q, W.hstride, s, P, delta);
    const bool cast = !(c.x == 0.0f && c.y == 0.0f && c.z == 0.0f);  // see sample_color
    W.scol[e] = make_float4(c.x, c.y, c.z, u2f(cast ? 1u : 0u));
    if (cast) {
        W.sray[e] = make_float4(P.x, P.y, P.z, 0.0f);
        W.sray[W.sstride + e] = make_float4(delta.x, delta.y, delta.z, 0.0f);
    }
}

template <int PF, bool CHAIN, bool FO>
__global__ __launch_bounds__(256, JSRT_MARCH_OCC) void k_shadow_cast(DScene S, WArgs W, int L) {
    const uint32_t count = CHAIN ? chain_level(W, L).count : level_range(W, L).count;
    ShadowSrc src{W};
    persistent_cast<PF, true, FO>(S, W.qctr + 32 + L, count * (uint32_t)W.group, 0.0001, 1, false, src);
}

// colorFromLights' sums of k_shadow from the stored sample colours (shadowed: +0)
template <bool CHAIN>
__global__ __launch_bounds__(256) void k_shadow_sum(DScene S, WArgs W, int L) {
    const LevelRange R = CHAIN ? chain_level(W, L) : level_range(W, L);
    const uint32_t count = R.count, base = R.base;
    const uint32_t G = (uint32_t)W.group, ns = (uint32_t)W.ns;
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    const uint32_t q = e / G, s = e % G;
    const bool in = q < count;
    const uint32_t i = base + (in ? (CHAIN ? chain_slot(W, L, q) : q) : 0u);
    const float4 nd = W.node[i];
    const bool lit = in && (f2u(nd.w) & INFO_LIT);
    F3 c = f3(0, 0, 0);
    if (lit && s < ns) {
        const float4 v = W.scol[e];
        if (f2u(v.w) != 2u) c = f3(v.x, v.y, v.z);
    }
    const F3 ret = light_sums(S, G, f3(nd.x, nd.y, nd.z), c);
    if (lit && s == 0) W.node[i] = make_float4(ret.x, ret.y, ret.z, nd.w);
}

// World.cast of a batch of independent rays (jsrt_cast): the closest-hit cast k_extend runs,
// with the caller's (minD, maxD, intersectTransparent).
template <int PF>
__global__ __launch_bounds__(256) void k_cast_rays(DScene S, const float *rays, uint32_t n, double minD, double maxD,
                                                   int transp, double *out_t, int32_t *out_prim) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + 6 * (size_t)i;
    const F3 o = f3(r[0], r[1], r[2]), d = f3(r[3], r[4], r[5]);
    const Hit h = world_cast<PF, false>(S, o, d, minD, maxD, transp != 0);
    out_t[i] = h.t;
    out_prim[i] = h.prim;
}
template <int PF>
void cast_rays_pf(const DScene &S, const float *rays, uint32_t n, double minD, double maxD, int transp, double *t,
                  int32_t *prim, hipStream_t st) {
    const size_t lds = (PF & (PF_BVH | PF_AGG)) ? bvh_lds_bytes(S, 256) : 0;
    hipLaunchKernelGGL((k_cast_rays<PF>), dim3(grid_ub(n)), dim3(256), lds, st, S, rays, n, minD, maxD, transp, t, prim);
}

// World.color(ray, 1) up to Material.color for a batch of rays (jsrt_material_data, the material-data
// known answers): the closest hit of World.cast(ray, 0) (world.js:34) and the hit's surface_data.
// Absent fields are NaN; uv[2] is always NaN (the kernels read u, v only).
template <int PF>
__global__ __launch_bounds__(256) void k_material_data(DScene S, const float *rays, uint32_t n, double *out_t,
                                                       int32_t *out_prim, float *nrm, float *pos, float *uv,
                                                       float *bary, float *bc) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + 6 * (size_t)i;
    const F3 o = f3(r[0], r[1], r[2]), d = f3(r[3], r[4], r[5]);
    const Hit h = world_cast<PF, false>(S, o, d, 0.0, DINF, true);
    out_t[i] = h.t;
    out_prim[i] = h.prim;
    const float nan = __builtin_nanf("");
    float *N = nrm + 4 * (size_t)i, *P = pos + 4 * (size_t)i, *U = uv + 3 * (size_t)i, *B = bary + 3 * (size_t)i,
          *C = bc + 3 * (size_t)i;
    if (h.prim < 0) {
        for (int k = 0; k < 4; ++k) N[k] = P[k] = nan;
        for (int k = 0; k < 3; ++k) U[k] = B[k] = C[k] = nan;
        return;
    }
    Surface sf;
    surface_data<PF, true>(S, h, o, d, true, sf);
    const F3 p = ray_point(o, d, h.t);  // material_data.position = ray.getPoint(distance)
    N[0] = sf.N.x; N[1] = sf.N.y; N[2] = sf.N.z; N[3] = 0.0f;
    P[0] = p.x; P[1] = p.y; P[2] = p.z; P[3] = 1.0f;
    U[0] = sf.has_uv ? sf.u : nan; U[1] = sf.has_uv ? sf.v : nan; U[2] = nan;
    B[0] = sf.has_bary ? sf.bary.x : nan; B[1] = sf.has_bary ? sf.bary.y : nan; B[2] = sf.has_bary ? sf.bary.z : nan;
    C[0] = sf.has_bc ? sf.basecolor.x : nan; C[1] = sf.has_bc ? sf.basecolor.y : nan; C[2] = sf.has_bc ? sf.basecolor.z : nan;
}
template <int PF>
void material_data_pf(const DScene &S, const float *rays, uint32_t n, double *t, int32_t *prim, float *nrm, float *pos,
                      float *uv, float *bary, float *bc, hipStream_t st) {
    const size_t lds = (PF & (PF_BVH | PF_AGG)) ? bvh_lds_bytes(S, 256) : 0;
    hipLaunchKernelGGL((k_material_data<PF>), dim3(grid_ub(n)), dim3(256), lds, st, S, rays, n, t, prim, nrm, pos, uv,
                       bary, bc);
}

// Enqueues one batch without a host round trip.  Chain: every level has exactly npaths slots.
// Tree: level L's launches cover bound[L] rays (the real count is on the device and surplus
// blocks exit at once; a count above the bound sets LVL_UNDER and the frame is redone);
// levels are reduced bottom-up afterwards.
template <int PF, bool CHAIN>
void run_batch(const DScene &S, const RenderArgs &A, const WArgs &W, hipStream_t st, KernelTimes *kt,
               const std::vector<size_t> &bound, const BatchSync *sync) {
    auto accum_wait = [&] { if (sync && sync->wait) (void)hipStreamWaitEvent(st, sync->wait, 0); };
    auto accum_done = [&] { if (sync && sync->done) (void)hipEventRecord(sync->done, st); };
    const hipStream_t ss = (sync && sync->aux) ? sync->aux : st;  // k_shadow's stream
    const bool split = ss != st;
    auto timed = [&](int which, auto launch) {
        const bool ev = kt && kt->on(which);
        const hipStream_t s = which == KT_SHADOW ? ss : st;
        if (ev) kt->ev[which].begin(s);
        launch();
        if (ev) kt->ev[which].end(s);
    };
    // dynamic LDS of the casting kernels: the BVH traversal stack (bvh_cast), 256 lanes x entries
    const size_t lds = (PF & (PF_BVH | PF_AGG)) ? bvh_lds_bytes(S, 256) : 0;
    // persistent casts for SDF scenes with a flat top level (W.sstride != 0 when enabled)
    const bool Q = (PF & PF_SDF) && W.sstride != 0;
    if (Q) (void)hipMemsetAsync(W.qctr, 0, 64 * sizeof(uint32_t), st);
    if (W.bucket) (void)hipMemsetAsync(W.bkt, 0, (size_t)MAX_TREE_DEPTH * BKT_LEVEL * sizeof(uint32_t), st);
    timed(KT_GEN, [&] { hipLaunchKernelGGL(k_gen, dim3(grid(W.npaths)), dim3(256), 0, st, S, A, W); });
    std::vector<size_t> ubs;  // launch bound of each level's ray count
    const bool learned = !CHAIN || W.hybrid;  // launch bounds from the host (learned level counts)
    for (int L = 0; L < A.max_depth && (!learned || bound[L] > 0); ++L) {
        const size_t ub = learned ? bound[L] : (size_t)W.npaths;
        ubs.push_back(ub);
        const int child_depth = A.max_depth - L - 1;
        timed(KT_EXTEND, [&] {
            if (Q && S.sdf_all_forms)  // every SDF root a recognised form: the march without the VM
                hipLaunchKernelGGL((k_extend_q<PF, CHAIN, true>), dim3(persistent_grid((const void *)k_extend_q<PF, CHAIN, true>, ub)),
                                   dim3(256), 0, st, S, W, L, L == 0 ? 0.0 : 0.0001);
            else if (Q)
                hipLaunchKernelGGL((k_extend_q<PF, CHAIN, false>), dim3(persistent_grid((const void *)k_extend_q<PF, CHAIN, false>, ub)),
                                   dim3(256), 0, st, S, W, L, L == 0 ? 0.0 : 0.0001);
            else
                hipLaunchKernelGGL((k_extend<PF, CHAIN>), dim3(grid_ub(ub)), dim3(256), lds, st, S, W, L, L == 0 ? 0.0 : 0.0001);
        });
        if (W.bucket) hipLaunchKernelGGL(k_bucket_offsets, dim3(1), dim3(256), 0, st, W, L);
        if (split && L > 0 && W.ns > 0) (void)hipStreamWaitEvent(st, sync->shadow_done, 0);  // the hand-off is free
        timed(KT_SHADE, [&] {
            if (PF == PF_ANALYTIC && S.stab_words > 0)  // the LDS-staged shading tables
                hipLaunchKernelGGL((k_shade<PF, CHAIN, PF == PF_ANALYTIC>), dim3(grid_ub(ub)), dim3(256), (size_t)S.stab_words * 16,
                                   st, S, W, L, child_depth);
            else
                hipLaunchKernelGGL((k_shade<PF, CHAIN, false>), dim3(grid_ub(ub)), dim3(256), 0, st, S, W, L, child_depth);
            if (child_depth > 0) hipLaunchKernelGGL(k_fix_dirs, dim3(1), dim3(256), 0, st, W);
        });
        if (W.ns > 0 && split) {
            (void)hipEventRecord(sync->shade_done, st);
            (void)hipStreamWaitEvent(ss, sync->shade_done, 0);
        }
        if (W.ns > 0)
            timed(KT_SHADOW, [&] {
                const hipStream_t st = ss;  // (the launches below name `st`)
                const size_t ne = ub * (size_t)W.group;
                if (Q && W.ns <= 64) {
                    hipLaunchKernelGGL((k_shadow_prep<PF, CHAIN>), dim3(grid_ub(ne)), dim3(256), 0, st, S, W, L);
                    if (S.sdf_all_forms)
                        hipLaunchKernelGGL((k_shadow_cast<PF, CHAIN, true>),
                                           dim3(persistent_grid((const void *)k_shadow_cast<PF, CHAIN, true>, ne)), dim3(256), 0, st, S, W, L);
                    else
                        hipLaunchKernelGGL((k_shadow_cast<PF, CHAIN, false>),
                                           dim3(persistent_grid((const void *)k_shadow_cast<PF, CHAIN, false>, ne)), dim3(256), 0, st, S, W, L);
                    hipLaunchKernelGGL((k_shadow_sum<CHAIN>), dim3(grid_ub(ne)), dim3(256), 0, st, S, W, L);
                } else if (W.ns <= 1 || W.group > 1) {
                    const dim3 g(grid_ub(ub * (size_t)W.group));
                    const size_t sl = (size_t)S.stab_words_shadow * 16;  // the LDS-staged tables (flat scenes)
                    if (PF == PF_ANALYTIC && sl && S.sphere_lights && S.n_sroot > 0)
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, true, PF == PF_ANALYTIC, PF == PF_ANALYTIC>), g, dim3(256), sl, st, S, W, L);
                    else if (PF == PF_ANALYTIC && sl && S.n_sroot > 0)
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, false, PF == PF_ANALYTIC, PF == PF_ANALYTIC>), g, dim3(256), sl, st, S, W, L);
                    else if (PF == PF_ANALYTIC && sl && S.sphere_lights)
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, true, PF == PF_ANALYTIC>), g, dim3(256), sl, st, S, W, L);
                    else if (PF == PF_ANALYTIC && sl)
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, false, PF == PF_ANALYTIC>), g, dim3(256), sl, st, S, W, L);
                    else if (S.sphere_lights)
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, true>), g, dim3(256), lds, st, S, W, L);
                    else
                        hipLaunchKernelGGL((k_shadow<PF, CHAIN, false, false>), g, dim3(256), lds, st, S, W, L);
                } else if (S.sphere_lights) {
                    hipLaunchKernelGGL((k_shadow<PF, CHAIN, true, true>), dim3(grid_ub(ub)), dim3(256), lds, st, S, W, L);
                } else {
                    hipLaunchKernelGGL((k_shadow<PF, CHAIN, true, false>), dim3(grid_ub(ub)), dim3(256), lds, st, S, W, L);
                }
            });
        if (W.ns > 0 && split) (void)hipEventRecord(sync->shadow_done, ss);
    }
    if (split && W.ns > 0 && !ubs.empty()) (void)hipStreamWaitEvent(st, sync->shadow_done, 0);  // the lit colours
    if (CHAIN && W.hybrid) {  // side chains deepest start first, then the paths; k_accum adds them in sample order
        timed(KT_RESOLVE, [&] {
            for (int s = (int)ubs.size() - 1; s >= 1; --s)  // (the chains started at s are live at s: <= ubs[s])
                hipLaunchKernelGGL(k_resolve_side, dim3(grid_ub(ubs[s])), dim3(256), 0, st, A, W, s);
            hipLaunchKernelGGL(k_resolve_paths, dim3(grid(W.npaths)), dim3(256), 0, st, A, W);
        });
        accum_wait();
        timed(KT_ACCUM, [&] { hipLaunchKernelGGL(k_accum, dim3(grid(W.npix)), dim3(256), 0, st, A, W); });
        accum_done();
        return;
    }
    if (CHAIN) {
        accum_wait();
        timed(KT_RESOLVE, [&] { hipLaunchKernelGGL(k_resolve, dim3(grid(W.npix)), dim3(256), 0, st, A, W); });
        accum_done();
        return;
    }
    for (int L = (int)ubs.size() - 1; L >= 0; --L)
        timed(KT_REDUCE, [&] { hipLaunchKernelGGL(k_reduce, dim3(grid_ub(ubs[L])), dim3(256), 0, st, W, L); });
    accum_wait();
    timed(KT_ACCUM, [&] { hipLaunchKernelGGL(k_accum, dim3(grid(W.npix)), dim3(256), 0, st, A, W); });
    accum_done();
}

}  // namespace jsrt
