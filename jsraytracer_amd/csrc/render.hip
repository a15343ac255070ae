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
#include "render_levels.h"

#include <mutex>

namespace jsrt {

const char *const KT_NAMES[KT_N] = {"k_gen", "k_extend", "k_shade", "k_shadow", "k_reduce", "k_accum", "k_final",
                                    "k_resolve"};

// camera rays: one per path q of the batch, sample-major (neighbouring q are neighbouring pixels)
__global__ __launch_bounds__(256) void k_gen(DScene S, RenderArgs A, WArgs W) {
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if ((!W.chain || W.hybrid) && q < LVL_UNDER) W.lvl[q] = q == 0 ? W.npaths : 0u;  // level counts (not the frame flags)
    if (q >= W.npaths) return;
    int c = 0, py = 0, px = 0;
    const uint32_t nsb = W.npaths / W.npix;
    const uint32_t pl = W.pixel_major ? q / nsb : q % W.npix, sl = W.pixel_major ? q % nsb : q / W.npix;
    const uint32_t smp = W.s0 + sl;
    const bool valid = pixel_of(A, W.p0 + pl, c, py, px);
    if (!W.chain) {
        if (A.max_depth <= 0) {  // World.color(ray, 0) = black; no level is traced
            W.root[3 * q] = W.root[3 * q + 1] = W.root[3 * q + 2] = 0.0f;
            return;
        }
        W.path[q] = q;
        W.parent[q] = valid ? NO_PARENT : DEAD_RAY;
    }
    if (!valid || A.max_depth <= 0) {  // edge patch outside the image: no ray
        W.prim[q] = NO_RAY;
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
    W.prim[q] = -1;
}

// tree schedule: surface + children, bottom-up into the parent's child slot (materials.js:277-330)
__global__ __launch_bounds__(256) void k_reduce(WArgs W, int L) {
    const LevelRange R = level_range(W, L);
    const uint32_t tt = blockIdx.x * 256 + threadIdx.x;
    if (tt >= R.count) return;
    const uint32_t i = R.base + tt;
    // the node record, its parent and its first child's colour and record are loaded together (most
    // nodes have exactly one child): one memory round trip instead of two dependent ones
    const float4 nd = W.node[i];
    const uint32_t p = W.parent[i];
    const float4 v0 = W.slot[i];
    const float4 c0 = W.child[i];
    const uint32_t info = f2u(nd.w);
    if (!(info & INFO_HIT) || p == DEAD_RAY) return;
    F3 c = f3(nd.x, nd.y, nd.z);
    const int n = (int)((info >> INFO_NCHILD_SHIFT) & 3);
    if (n > 0) c = add_child(W, i, 0u, c, f3(v0.x, v0.y, v0.z), info, &c0);
    if (n > 1) {
        const float4 v1 = W.slot[W.nstride + i];
        c = add_child(W, i, 1u, c, f3(v1.x, v1.y, v1.z), info);
    }
    if (p == NO_PARENT) {  // write_result
        float *dst = W.root + 3 * (size_t)W.path[i];
        dst[0] = c.x;
        dst[1] = c.y;
        dst[2] = c.z;
    } else {
        W.slot[(size_t)(p & 1u) * W.nstride + (p >> 1)] = make_float4(c.x, c.y, c.z, 0.0f);
    }
}

__global__ __launch_bounds__(256) void k_bucket_offsets(WArgs W, int L) {
    __shared__ uint32_t part[256];
    uint32_t *B = W.bkt + (size_t)L * BKT_LEVEL;
    constexpr int PER = BKT_K / 256;
    const int t = (int)threadIdx.x;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) { c[j] = B[t * PER + j]; sum += c[j]; }
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {  // inclusive scan of the per-thread sums
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t off = part[t] - sum;
#pragma unroll
    for (int j = 0; j < PER; ++j) { B[2 * BKT_K + t * PER + j] = off; off += c[j]; }
    if (t == 255) B[3 * BKT_K] = part[255];
}

// tree schedule: per pixel, the batch's samples in order
__global__ __launch_bounds__(256) void k_accum(RenderArgs A, WArgs W) {
    const uint32_t pl = blockIdx.x * 256 + threadIdx.x;
    if (pl >= W.npix || W.lvl[LVL_FLAG]) return;  // a poisoned frame is redone by the host
    int c, py, px;
    if (!pixel_of(A, W.p0 + pl, c, py, px)) return;
    const size_t oi = (size_t)c * A.H + py;
    F3 acc = f3(A.accum[4 * oi], A.accum[4 * oi + 1], A.accum[4 * oi + 2]);
    const uint32_t nsb = W.npaths / W.npix;
    for (uint32_t sl = 0; sl < nsb; ++sl) {
        const uint32_t q = W.pixel_major ? pl * nsb + sl : sl * W.npix + pl;
        acc = accumulate(A, acc, f3(W.root[3 * q], W.root[3 * q + 1], W.root[3 * q + 2]));
    }
    A.accum[4 * oi] = acc.x;
    A.accum[4 * oi + 1] = acc.y;
    A.accum[4 * oi + 2] = acc.z;
}

// chain schedule: per pixel, its samples in order; each path's colour is resolved bottom-up over
// its levels (surface + child contribution; a last-level child is black without a cast)
__global__ __launch_bounds__(256) void k_resolve(RenderArgs A, WArgs W) {
    const uint32_t pl = blockIdx.x * 256 + threadIdx.x;
    if (pl >= W.npix) return;
    int c, py, px;
    if (!pixel_of(A, W.p0 + pl, c, py, px)) return;
    const size_t oi = (size_t)c * A.H + py;
    F3 acc = f3(A.accum[4 * oi], A.accum[4 * oi + 1], A.accum[4 * oi + 2]);
    const uint32_t nsb = W.npaths / W.npix;
    for (uint32_t sl = 0; sl < nsb; ++sl) {
        const uint32_t q = W.pixel_major ? pl * nsb + sl : sl * W.npix + pl;
        F3 v = f3(0, 0, 0);  // World.color(ray, 0) = black
        for (int L = A.max_depth - 1; L >= 0; --L) {
            const uint32_t i = (uint32_t)L * W.cap + q;
            const float4 nd = W.node[i];
            const uint32_t info = f2u(nd.w);
            if (info & INFO_MISS) {
                v = f3(nd.x, nd.y, nd.z);
            } else if (info & INFO_HIT) {
                F3 col = f3(nd.x, nd.y, nd.z);
                if ((info >> INFO_NCHILD_SHIFT) & 3) col = add_child(W, i, 0, col, L == A.max_depth - 1 ? f3(0, 0, 0) : v, info);
                v = col;
            }
        }
        acc = accumulate(A, acc, v);
    }
    A.accum[4 * oi] = acc.x;
    A.accum[4 * oi + 1] = acc.y;
    A.accum[4 * oi + 2] = acc.z;
}

// hybrid chain: the colour of chain c, which starts at level s, bottom-up over its levels (surface + the
// first child's contribution -- the chain's own next level -- + the second child's, a side chain's colour
// in slot[i]; children of the last level are black without a cast), materials.js:277-330
__device__ __forceinline__ F3 resolve_chain(const RenderArgs &A, const WArgs &W, uint32_t c, int s) {
    F3 v = f3(0, 0, 0);
    const int end = W.endl[c];
    // the node records of the chain's levels, loaded before the bottom-up pass (their addresses do not
    // depend on it): up to 8 levels' loads in flight at once instead of one dependent round trip per level
    constexpr int PRE = 8;
    float4 pre[PRE];
#pragma unroll
    for (int k = 0; k < PRE; ++k)
        if (s + k <= end) pre[k] = W.node[(uint32_t)(s + k) * W.cap + c];
    for (int L = end; L >= s; --L) {
        const uint32_t i = (uint32_t)L * W.cap + c;
        float4 nd = L - s < PRE ? pre[0] : W.node[i];
#pragma unroll
        for (int k = 1; k < PRE; ++k)
            if (L - s == k) nd = pre[k];
        const uint32_t info = f2u(nd.w);
        if (info & INFO_MISS) {
            v = f3(nd.x, nd.y, nd.z);
        } else if (info & INFO_HIT) {
            const bool last = L == A.max_depth - 1;
            const int n = (int)((info >> INFO_NCHILD_SHIFT) & 3);
            F3 col = f3(nd.x, nd.y, nd.z);
            if (n > 0) col = add_child(W, i, 0, col, last ? f3(0, 0, 0) : v, info);
            if (n > 1) {
                const float4 v1 = last ? make_float4(0, 0, 0, 0) : W.slot[i];
                col = add_child(W, i, 1, col, f3(v1.x, v1.y, v1.z), info);
            }
            v = col;
        }
    }
    return v;
}

// hybrid chain: the side chains that start at level s (ids npaths + [side(< s), side(<= s))), into their
// parents' second-child slots.  Launched for s = depth - 1 .. 1, so a chain's own side chains are resolved
// first.
__global__ __launch_bounds__(256) void k_resolve_side(RenderArgs A, WArgs W, int s) {
    if (W.lvl[LVL_FLAG]) return;
    const uint32_t lo = side_base(W, s);
    const uint32_t c = lo + blockIdx.x * 256 + threadIdx.x;
    if (c >= lo + W.lvl[2 * s + 1]) return;
    const F3 v = resolve_chain(A, W, c, s);
    W.slot[W.parent[c]] = make_float4(v.x, v.y, v.z, 0.0f);
}

// hybrid chain: every path's colour -> root (k_accum adds them per pixel in sample order)
__global__ __launch_bounds__(256) void k_fix_dirs(WArgs W) {
    const uint32_t n = *W.fixctr, m = n < W.fixcap ? n : W.fixcap;
    // a child slot past the ray arrays belongs to a frame k_shade flagged for a redo (out of chain slots or
    // pool): not written
    const size_t bound = W.chain ? (size_t)W.cap : (size_t)W.pool;
    for (uint32_t k = threadIdx.x; k < m; k += 256) {
        const uint4 a = W.fixrec[3 * (size_t)k], b = W.fixrec[3 * (size_t)k + 1], c = W.fixrec[3 * (size_t)k + 2];
        const F3 N = f3(__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z));
        for (int j = 0; j < 2; ++j) {
            const uint32_t f = j == 0 ? b.x : b.y;
            if (j >= (int)b.z || f == 0u) continue;
            Rng rg{a.z, a.w, (f & 0x7FFFFFFFu) - 1u};  // the pick's draws (path_scatter: theta, then acos's argument)
            const F3 sp3 = sphere_pick_v8(rg);
            const F3 dir = normalized(add((f >> 31) ? neg(N) : N, sp3));  // scatterDiffuse about N or -N
            const uint32_t dst = j == 0 ? a.x : a.y;
            if (dst >= bound) continue;
            W.dx[dst] = dir.x;
            W.dy[dst] = dir.y;
            W.dz[dst] = dir.z;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *W.fixctr = 0u;  // the next level's records
}

__global__ __launch_bounds__(256) void k_resolve_paths(RenderArgs A, WArgs W) {
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (q >= W.npaths || W.lvl[LVL_FLAG]) return;
    const F3 v = resolve_chain(A, W, q, 0);
    W.root[3 * q] = v.x;
    W.root[3 * q + 1] = v.y;
    W.root[3 * q + 2] = v.z;
}

__global__ __launch_bounds__(256) void k_final(RenderArgs A, int32_t passes) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= (uint32_t)A.ncols * A.H) return;
    const F3 acc = f3(A.accum[4 * p], A.accum[4 * p + 1], A.accum[4 * p + 2]);
    const F3 out = (A.kind == JSRT_RENDERER_INCREMENTAL) ? scale(acc, 1.0 / passes) : acc;  // times(1/(iter+1))
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
double EventPairs::total_ms(uint32_t *lost) const {
    double ms = 0;
    for (size_t k = 0; k < used; ++k) {
        float x = 0;
        if (hipEventElapsedTime(&x, b[k], e[k]) == hipSuccess) ms += x;
        else if (lost) ++*lost;
    }
    return ms;
}
EventPairs::~EventPairs() {
    for (auto x : b) (void)hipEventDestroy(x);
    for (auto x : e) (void)hipEventDestroy(x);
}

hipError_t Wavefront::reserve(size_t rays, size_t nodes, size_t hands, size_t paths, int mode, size_t shadow) {
    const bool tree = mode == SCHED_TREE, hybrid = mode == SCHED_HYBRID;
    size_t bytes = 0;
    bytes += 8 * need(rays, 4) + need(rays, 8) + 2 * need(rays, 4);  // o d addr key + t + prim ctx
    if (tree) bytes += 2 * need(rays, 4);                            // path parent
    if (hybrid) bytes += 3 * need(rays, 4) + need(rays, 1);          // parent, live lists, last levels
    bytes += need(nodes, 16) + need(4 * nodes, 16);                  // node + child
    if (tree) bytes += need(2 * nodes, 16);                          // slot
    if (hybrid) bytes += need(nodes, 16);                            // slot (second children)
    if (tree || hybrid) bytes += need(3 * paths, 4);                 // root
    bytes += need(HAND_PLANES * hands, 16) + need(hands, 4) + need(64, 4);  // hand-off + nodes + level counts
    bytes += need(64, 4) + need(2 * shadow, 16) + need(shadow, 16);  // work counters + shadow rays
    // unstable spherePicks per level: ~1e-5 of the nodes (k_fix_dirs); every node under JSRT_FORCE_EXACT_PICK,
    // or after a frame that ran out of records (fix_all: the frame is redone with one record per ray slot)
    const char *fx = getenv("JSRT_FORCE_EXACT_PICK");
    const bool force_fix = fx && fx[0] == '1';
    // (JSRT_FIX_CAP=n, a test knob: n records until a frame runs out, to exercise the redo on either pool)
    const char *fc = getenv("JSRT_FIX_CAP");
    const size_t fixcap = fix_all ? rays + 4096 : fc ? (size_t)std::max(0, atoi(fc)) : force_fix ? rays + 4096 : rays / 8 + 4096;
    bytes += need(3 * fixcap, 16) + need(64, 4);
    if (tree || hybrid)  // buckets
        bytes += need(MAX_TREE_DEPTH * BKT_LEVEL, 4) + need((hands / 256 + 1) * BKT_N, 4) + need(rays, 4);
    if (mem && bytes <= cap_bytes) {  // carve the cached allocation again
    } else {
        if (mem) (void)hipFree(mem);
        mem = nullptr;
        cap_bytes = 0;
        hipError_t e = hipMalloc(&mem, bytes);
        if (e != hipSuccess) return e;
        cap_bytes = bytes;
    }
    uint8_t *p = static_cast<uint8_t *>(mem);
    WArgs &w = args;
    w = WArgs{};
    w.ox = carve<float>(p, rays); w.oy = carve<float>(p, rays); w.oz = carve<float>(p, rays);
    w.dx = carve<float>(p, rays); w.dy = carve<float>(p, rays); w.dz = carve<float>(p, rays);
    w.addr = carve<uint32_t>(p, rays); w.key = carve<uint32_t>(p, rays);
    w.t = carve<double>(p, rays); w.prim = carve<int32_t>(p, rays); w.ctx = carve<int32_t>(p, rays);
    if (tree) { w.path = carve<uint32_t>(p, rays); w.parent = carve<uint32_t>(p, rays); }
    if (hybrid) {
        w.parent = carve<uint32_t>(p, rays);
        w.list0 = carve<uint32_t>(p, rays);
        w.list1 = carve<uint32_t>(p, rays);
        w.endl = carve<uint8_t>(p, rays);
    }
    w.node = carve<float4>(p, nodes);
    w.child = carve<float4>(p, 4 * nodes);
    if (tree) w.slot = carve<float4>(p, 2 * nodes);
    if (hybrid) w.slot = carve<float4>(p, nodes);
    if (tree || hybrid) w.root = carve<float>(p, 3 * paths);
    w.hand = carve<float4>(p, HAND_PLANES * hands);
    w.hnode = carve<uint32_t>(p, hands);
    w.lvl = carve<uint32_t>(p, 64);
    w.qctr = carve<uint32_t>(p, 64);
    w.fixrec = carve<uint4>(p, 3 * fixcap);
    w.fixctr = carve<uint32_t>(p, 64);
    w.fixcap = (uint32_t)fixcap;
    w.force_fix = force_fix ? 1 : 0;
    if (shadow) { w.sray = carve<float4>(p, 2 * shadow); w.scol = carve<float4>(p, shadow); }
    if (tree || hybrid) {
        w.bkt = carve<uint32_t>(p, MAX_TREE_DEPTH * BKT_LEVEL);
        w.bbase = carve<uint32_t>(p, (hands / 256 + 1) * BKT_N);
        w.brank = carve<uint32_t>(p, rays);
    }
    w.nstride = nodes;
    w.hstride = hands;
    w.sstride = shadow;
    return hipSuccess;
}

void Wavefront::release() {
    if (mem) (void)hipFree(mem);
    mem = nullptr;
    cap_bytes = 0;
    if (twin) twin->release();
}

Wavefront::~Wavefront() {
    release();
    delete twin;
    if (side) (void)hipStreamDestroy(side);
    if (aux) (void)hipStreamDestroy(aux);
    if (ev_shade) (void)hipEventDestroy(ev_shade);
    if (ev_shadow) (void)hipEventDestroy(ev_shadow);
}

// The schedule of a scene's frames: chain when no node can have two children; otherwise the hybrid chain
// (side chains for second children) for flat scenes, the tree for BVH / SDF scenes (JSRT_HYBRID=0/1 forces
// one).  A/B on MI355X (profiles/r04_s6_ab.txt): cornell hybrid 493.8 vs tree 466.3 Ms/s; bunny 518.4 vs
// 555.7, dragon 785.4 vs 792.5, SDF_Menger 112.8 vs 116.1 -- the tree's octant-sorted appends keep BVH
// casts coherent, and its compaction suits sky-heavy scenes.
int schedule_of(const DScene &S) {
    if (S.max_children <= 1) return SCHED_CHAIN;
    const char *hy = getenv("JSRT_HYBRID");
    if (hy) return hy[0] == '0' ? SCHED_TREE : SCHED_HYBRID;
    return S.profile == PF_ANALYTIC ? SCHED_HYBRID : SCHED_TREE;
}
constexpr size_t HYBRID_POOL_FACTOR = 2;  // initial hybrid side-chain slots: paths x factor / 4

size_t wavefront_bytes_per_path(const DScene &S, int ns, int max_depth) {
    const size_t ray = 8 * 4 + 8 + 2 * 4, node = 16 + 4 * 16, hand = HAND_PLANES * 16 + 4;
    const bool persist = (S.profile & PF_SDF) && S.all_roots_prims;
    size_t group = 1;
    while ((int)group < ns && ns <= 64) group *= 2;
    const int sched = schedule_of(S);
    const size_t depth = (size_t)std::max(1, max_depth);
    if (sched == SCHED_CHAIN)  // chain: one ray and depth nodes per path
        return ray + depth * node + hand + (persist ? group * 48 : 0);
    if (sched == SCHED_HYBRID)  // per chain slot: ray + parent + rank, depth x (node + second-child slot), hand-off
        return (4 + HYBRID_POOL_FACTOR) * (ray + 17 + depth * (node + 16) + hand + (persist ? group * 48 : 0) +
                                           BKT_N * 4 / 256) / 4 + 12;
    const size_t pool = 8, level_cap = pool / 2;  // render_frame: pool = 8 x paths, level_cap = pool / 2
    // + the bucketed hand-off's ranks (4 B per pool slot) and block bases (BKT_N words per 256 hand-off slots)
    return pool * (ray + 8 + node + 2 * 16 + 4) + level_cap * (hand + (persist ? group * 48 : 0) + BKT_N * 4 / 256) + 12;
}


// Grid of a persistent kernel: as many 256-thread blocks as the device keeps resident (occupancy x
// CUs), never more than the work needs.  Cached per kernel and device behind a mutex: renders run
// concurrently on several host threads (Node async work, worker threads, one scene per thread).
unsigned persistent_grid(const void *kernel, size_t work) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<const void *, int>, unsigned>> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    unsigned resident = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (auto &c : cache)
            if (c.first.first == kernel && c.first.second == dev) resident = c.second;
    }
    if (!resident) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
        resident = (unsigned)(per_cu * cus);
        std::lock_guard<std::mutex> lk(mu);
        cache.push_back({{kernel, dev}, resident});
    }
    return std::max(1u, std::min(resident, grid_ub(work)));
}

// instantiated in render_pf.hip, one translation unit per profile
extern template void run_batch<PF_ANALYTIC, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_ANALYTIC, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_MESH, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_MESH, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_SDF, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_SDF, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_ALL, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);
extern template void run_batch<PF_ALL, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t,
                                         KernelTimes *, const std::vector<size_t> &, const BatchSync *);

#define JSRT_CAST_EXTERN(PFV) \
    extern template void cast_rays_pf<PFV>(const DScene &, const float *, uint32_t, double, double, int, double *, \
                                           int32_t *, hipStream_t);
JSRT_CAST_EXTERN(PF_ANALYTIC)
JSRT_CAST_EXTERN(PF_MESH)
JSRT_CAST_EXTERN(PF_SDF)
JSRT_CAST_EXTERN(PF_ALL)
#undef JSRT_CAST_EXTERN

#define JSRT_MD_EXTERN(PFV)                                                                                          \
    extern template void material_data_pf<PFV>(const DScene &, const float *, uint32_t, double *, int32_t *, float *, \
                                               float *, float *, float *, float *, hipStream_t);
JSRT_MD_EXTERN(PF_ANALYTIC)
JSRT_MD_EXTERN(PF_MESH)
JSRT_MD_EXTERN(PF_SDF)
JSRT_MD_EXTERN(PF_ALL)
#undef JSRT_MD_EXTERN

hipError_t material_data_rays(const DScene &S, const float *d_rays, uint32_t n, double *d_t, int32_t *d_prim,
                              float *d_nrm, float *d_pos, float *d_uv, float *d_bary, float *d_bc, hipStream_t st) {
    if (n == 0) return hipSuccess;
    switch (S.profile) {
    case PF_ANALYTIC: material_data_pf<PF_ANALYTIC>(S, d_rays, n, d_t, d_prim, d_nrm, d_pos, d_uv, d_bary, d_bc, st); break;
    case PF_MESH: material_data_pf<PF_MESH>(S, d_rays, n, d_t, d_prim, d_nrm, d_pos, d_uv, d_bary, d_bc, st); break;
    case PF_SDF: material_data_pf<PF_SDF>(S, d_rays, n, d_t, d_prim, d_nrm, d_pos, d_uv, d_bary, d_bc, st); break;
    default: material_data_pf<PF_ALL>(S, d_rays, n, d_t, d_prim, d_nrm, d_pos, d_uv, d_bary, d_bc, st); break;
    }
    return hipGetLastError();
}

// SDF.distance of SDF geometry g's root (sdf.js:53-74) at points (f32 x 4, w = 1): the same program VM
// the render's march runs (jsrt_sdf_distance)
__global__ __launch_bounds__(256) void k_sdf_distance(DScene S, int g, const float *pts, uint32_t n, double *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *p = pts + 4 * (size_t)i;
    out[i] = sdf_node_dist(S, S.sdfg[g].root, f3(p[0], p[1], p[2]));
}

hipError_t sdf_distance_points(const DScene &S, int g, const float *d_pts, uint32_t n, double *d_out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sdf_distance, dim3(grid_ub(n)), dim3(256), 0, st, S, g, d_pts, n, d_out);
    return hipGetLastError();
}

hipError_t cast_rays(const DScene &S, const float *d_rays, uint32_t n, double min_dist, double max_dist, bool transparent,
                     double *d_t, int32_t *d_prim, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const int tr = transparent ? 1 : 0;
    switch (S.profile) {
    case PF_ANALYTIC: cast_rays_pf<PF_ANALYTIC>(S, d_rays, n, min_dist, max_dist, tr, d_t, d_prim, st); break;
    case PF_MESH: cast_rays_pf<PF_MESH>(S, d_rays, n, min_dist, max_dist, tr, d_t, d_prim, st); break;
    case PF_SDF: cast_rays_pf<PF_SDF>(S, d_rays, n, min_dist, max_dist, tr, d_t, d_prim, st); break;
    default: cast_rays_pf<PF_ALL>(S, d_rays, n, min_dist, max_dist, tr, d_t, d_prim, st); break;
    }
    return hipGetLastError();
}

namespace {
template <bool CHAIN>
void run_batch_pf(const DScene &S, const RenderArgs &A, const WArgs &W, hipStream_t st, KernelTimes *kt,
                  const std::vector<size_t> &bound, const BatchSync *sync) {
    switch (S.profile) {
    case PF_ANALYTIC: run_batch<PF_ANALYTIC, CHAIN>(S, A, W, st, kt, bound, sync); break;
    case PF_MESH: run_batch<PF_MESH, CHAIN>(S, A, W, st, kt, bound, sync); break;
    case PF_SDF: run_batch<PF_SDF, CHAIN>(S, A, W, st, kt, bound, sync); break;
    default: run_batch<PF_ALL, CHAIN>(S, A, W, st, kt, bound, sync); break;
    }
}
}  // namespace

#ifndef TILE_PATCHES_DEFAULT
#define TILE_PATCHES_DEFAULT 8
#endif
#ifndef SPLIT_PIXELS_DEFAULT
#define SPLIT_PIXELS_DEFAULT true  // bunny 656.6 -> 687.2 M/s (profiles/r06_s9_bunny.txt)
#endif
hipError_t render_frame(const DScene &S, const RenderArgs &A, int ns, Wavefront &wf, hipStream_t st, KernelTimes *kt,
                        size_t max_paths, const std::function<bool(int, double, bool)> &progress,
                        const std::function<bool()> &due) {
    if (!A.accum) return hipErrorInvalidValue;
    const uint32_t npix_total = (uint32_t)A.patches * 64u;
    if (npix_total == 0) {  // a rank that owns no column (a multi-GPU frame narrower than its column blocks):
        // nothing to trace, but an Incremental frame's passes are still reported, so that the rank's callbacks
        // keep step with its peers' (tiles.render_progressive runs one collective per reported pass)
        if (progress && A.kind == JSRT_RENDERER_INCREMENTAL) {
            const uint32_t step = A.samples_per_batch > 0 ? (uint32_t)A.samples_per_batch : (uint32_t)A.spp;
            for (uint32_t s_end = step; s_end < (uint32_t)A.spp; s_end += step)
                if ((!due || due()) && !progress((int)s_end - 1, (double)s_end / A.spp, true)) break;
        }
        return hipSuccess;
    }
    if (ns > 4) max_paths = max_paths * 4 / (size_t)ns;  // the per-sample hand-off scales with ns
    if (max_paths < 64) max_paths = 64;
    uint32_t npix = npix_total, nsb = 1;  // batch: [p0, p0 + npix) pixels x [s0, s0 + nsb) samples
    if ((size_t)npix > max_paths) npix = (uint32_t)(max_paths & ~(size_t)63);
    else nsb = (uint32_t)std::max<size_t>(1, std::min<size_t>(max_paths / npix, (size_t)A.spp));
    if (A.samples_per_batch > 0) nsb = std::min<uint32_t>(nsb, (uint32_t)A.samples_per_batch);
    // Pixel-major batches (round 6; the BVH and SDF profiles, WArgs::pixel_major): a pixel's samples are side by
    // side in the batch, and a batch holds every sample of its pixels (up to JSRT_BATCH_SPP = 256) rather than a
    // few samples of every pixel.  The rays in flight (~0.5 M) then come from a small patch of the image, so their
    // casts walk a small part of the BVH and keep it in the caches.  The keyed RNG and the per-pixel
    // accumulation in sample order leave the image unchanged.  Measured (profiles/r06_s6_ab_pixel_major_*.txt,
    // r06_s7_dragon.txt, r06_s8_dragon.txt): bunny 556 -> 657 M/s, SDF_Menger 148 -> 160, the dragon 798 -> 889 in
    // pixel-major order alone, then 1,116 / 1,228 / 1,306 / 1,416 / 1,475 / 1,533 M/s at 8 / 16 / 32 / 64 / 128 /
    // 256 samples per batch; the flat hybrid chain loses (cornell k_accum's strided reads), so it keeps the
    // sample-major order.  JSRT_PIXEL_MAJOR=0/1: A/B.
    const char *pm = getenv("JSRT_PIXEL_MAJOR");
    const bool pixel_major = pm ? pm[0] == '1' : S.profile != PF_ANALYTIC;
    if (pixel_major) {
        const char *bs = getenv("JSRT_BATCH_SPP");
        uint32_t want = (uint32_t)(bs ? std::max(1, atoi(bs)) : 256);
        want = std::min<uint32_t>(want, (uint32_t)A.spp);
        if (A.samples_per_batch > 0) want = std::min<uint32_t>(want, (uint32_t)A.samples_per_batch);
        if (nsb < want) {  // fewer pixels, more of their samples
            npix = (uint32_t)std::min<size_t>(npix_total, std::max<size_t>(64, (max_paths / want) & ~(size_t)63));
            nsb = (uint32_t)std::max<size_t>(1, std::min<size_t>(max_paths / npix, (size_t)want));
        }
    }
    // ... and their pixels in compact tiles of JSRT_TILE_PATCHES x JSRT_TILE_PATCHES 8 x 8 patches (pixel_of)
    RenderArgs At = A;
    {
        const char *tp = getenv("JSRT_TILE_PATCHES");
        At.tile_p = pixel_major ? (tp ? std::max(0, atoi(tp)) : TILE_PATCHES_DEFAULT) : 0;
    }
    // persistent casts: SDF scenes whose top level is primitives only (JSRT_PERSIST=0 disables)
    const char *pe = getenv("JSRT_PERSIST");
    const bool persist = (S.profile & PF_SDF) && S.all_roots_prims && !(pe && pe[0] == '0');
    // A frame that fits one batch of 4 M paths or more (a rank's columns of a multi-GPU render) is cut into
    // two batches of half the samples, so that they run on the two batch streams (below).  Round 3 split only
    // from 32 M paths (cornell 1024^2 x 32 +3.6 %; halves of 16 M lost 5 %, profiles/r03_s18_ab.txt s28); with
    // the hybrid chain the halves win down to 4 M: cornell's 4-rank share (16.7 M paths) 32.0 -> 29.5 ms, its
    // 8-rank share (8.4 M) 17.0 -> 16.3 ms (tools/project_scaling.py, profiles/r05_s6_projection.txt).
    // JSRT_SPLIT_FRAME=0 keeps one batch; JSRT_SPLIT_MIN=k (A/B) splits from 2^k paths.
    const char *sf = getenv("JSRT_SPLIT_FRAME"), *sm = getenv("JSRT_SPLIT_MIN");  // (A/B: log2 of the paths)
    const int split_min = sm ? std::max(1, std::min(40, atoi(sm))) : 22;
    // (Pixel-major batches split their pixels instead -- two halves of the image, every sample each -- so that the
    // rays in flight keep coming from few pixels; JSRT_SPLIT_PIXELS=0/1: A/B.)
    const char *spx = getenv("JSRT_SPLIT_PIXELS");
    const bool split_pixels = pixel_major && (spx ? spx[0] == '1' : SPLIT_PIXELS_DEFAULT);
    if (!persist && !(sf && sf[0] == '0') && npix == npix_total && nsb == (uint32_t)A.spp && A.spp >= 2 &&
        (uint64_t)npix * (uint64_t)A.spp >= ((uint64_t)1 << split_min)) {
        if (split_pixels && npix_total >= 128) npix = ((npix_total / 2) + 63) & ~63u;  // whole patches: 64-pixel units
        else nsb = (uint32_t)((A.spp + 1) / 2);  // odd spp: halves of (spp + 1) / 2 and (spp - 1) / 2 samples
    }
    // Chain schedule when no node can have two children: depth x paths node records, nothing can
    // overflow, batches are enqueued back to back.  Tree schedule otherwise: a ray pool for all
    // levels of a batch (one level may hold half of it), compacted level by level.  Its launches
    // are sized by level counts learned from the scene's first batch (one read-back per scene and
    // batch shape) with a margin; a batch that outgrows its pool (LVL_FLAG) or a launch bound
    // (LVL_UNDER) poisons the frame, which is redone with a larger pool / conservative bounds.
    // The frame flags are read once, after the last batch.
    // Hybrid chain (branching materials, the default): the chain layout -- ray slot = path, node [L * cap +
    // slot], no parent / path planes, one bottom-up resolve -- plus a side chain per second child (a slot
    // appended after the paths, cap = paths + paths x pool_factor / 4).  Its level counts (the side chains
    // started so far) live on the device; launch bounds, overflow and redo work as for the tree.
    const int sched = schedule_of(S);
    const bool hybrid = sched == SCHED_HYBRID, chain = sched != SCHED_TREE, learned = sched != SCHED_CHAIN;
    const int depth = std::max(1, A.max_depth);
    const size_t paths = (size_t)npix * nsb;
    // test knobs: a smaller first pool / tighter learned bounds exercise the frame redo paths
    const char *pf_env = getenv("JSRT_POOL_FACTOR"), *bm_env = getenv("JSRT_BOUND_MARGIN");
    const double margin = bm_env ? atof(bm_env) : 1.25;
    const size_t slack = bm_env ? 0 : 4096;
    if (learned && (wf.pool_paths != paths || wf.pool_mode != sched)) {  // learned pool / bounds: per batch shape
        // (a batch of at most 1 M paths starts with 3 side-chain slots per path: a band of columns through a
        // glass sphere outgrows the default 0.5 -- a redo the memory of small batches need not risk)
        wf.pool_factor = pf_env ? std::max(1, atoi(pf_env))
                                : (hybrid ? (paths <= ((size_t)1 << 20) ? 8 : HYBRID_POOL_FACTOR) : 8);
        wf.frac.clear();
        wf.pool_paths = paths;
        wf.pool_mode = sched;
    }
    hipError_t e = hipSuccess;
    uint32_t *h_lvl = nullptr;  // read-back of the level counts (tree / hybrid schedule) and the frame flags
    if ((e = hipHostMalloc((void **)&h_lvl, 128 * sizeof(uint32_t), 0)) != hipSuccess) return e;
    // Two batch pools on two streams: consecutive batches alternate between them, so one batch's levels
    // (latency-bound casts, VALU-bound shadow samples, their launch tails) overlap the other's.  Only the
    // accumulation into A.accum is ordered across them -- each batch's k_accum / k_resolve waits for the
    // previous batch's (renderers.js:93-97: samples in order) -- so the image is unchanged bit for bit.
    // (A/B on MI355X, profiles/r03_s18_ab.txt: cornell +12.5 %, the dragon +2.6 %, bunny +0.6 %; two
    // persistent SDF marches side by side lose 1 %, so SDF scenes with persistent casts run on one
    // stream.)  The twin pool is allocated only if it fits; otherwise the frame runs on one pool.
    const uint64_t nbatches = (uint64_t)((A.spp + nsb - 1) / nsb) * ((npix_total + npix - 1) / npix);
    // A render that asks for its launches' own times (JSRT_EVENTS_ONE_STREAM) runs on one stream: a
    // launch's event interval is only its own time when no other batch's kernels share the CUs.
    const bool timed_launches = kt && kt->one_stream;
    const char *de = getenv("JSRT_DUAL");
    // two streams need two batches of comparable size: a frame of one full batch and a small remainder
    // (bunny: 32 M + 1.2 M paths) has nothing to overlap; a split frame of odd spp (nsb and nsb - 1 samples)
    // does
    const bool two_full = (uint64_t)npix_total * (uint64_t)A.spp >= 2 * (uint64_t)npix * nsb - (uint64_t)npix;
    bool dual = !timed_launches && nbatches > 1 && (de ? de[0] == '1' : (!persist && two_full));
    hipEvent_t ev_start = nullptr, ev_end = nullptr, ev_acc[2] = {nullptr, nullptr};
    auto release_events = [&] {
        for (hipEvent_t x : {ev_start, ev_end, ev_acc[0], ev_acc[1]})
            if (x) (void)hipEventDestroy(x);
    };
    if (dual) {
        if (!wf.twin) wf.twin = new Wavefront();
        if (!wf.side) e = hipStreamCreateWithFlags(&wf.side, hipStreamNonBlocking);
        for (hipEvent_t *x : {&ev_start, &ev_end, &ev_acc[0], &ev_acc[1]})
            if (e == hipSuccess) e = hipEventCreateWithFlags(x, hipEventDisableTiming);
        if (e != hipSuccess) {
            if (h_lvl) (void)hipHostFree(h_lvl);
            release_events();
            return e;
        }
    }
    hipStream_t st2 = dual ? wf.side : st;
    // A frame with persistent SDF casts (one stream) runs k_shadow on a stream of its own (BatchSync::aux):
    // level L's shadow samples overlap level L + 1's march.  SDF_Menger +6.5 %; elsewhere it loses
    // (bunny on one stream -5 %; beside two batch streams cornell +-0, dragon -1.3 %; profiles/
    // r03_s18_ab.txt s22, s26).  JSRT_SPLIT=0/1 forces it.
    const char *se = getenv("JSRT_SPLIT");
    const bool split = !timed_launches && ns > 0 && (se ? se[0] == '1' : (persist && !dual));
    auto aux_of = [&](Wavefront &w) -> hipError_t {
        hipError_t r = hipSuccess;
        if (!w.aux) r = hipStreamCreateWithFlags(&w.aux, hipStreamNonBlocking);
        if (r == hipSuccess && !w.ev_shade) r = hipEventCreateWithFlags(&w.ev_shade, hipEventDisableTiming);
        if (r == hipSuccess && !w.ev_shadow) r = hipEventCreateWithFlags(&w.ev_shadow, hipEventDisableTiming);
        return r;
    };
    if (split && (e = aux_of(wf)) == hipSuccess && dual) e = aux_of(*wf.twin);
    if (e != hipSuccess) {
        if (h_lvl) (void)hipHostFree(h_lvl);
        release_events();
        return e;
    }
    bool conservative = false, aborted = false;
    double reported = 0;  // completion already reported: a redone frame reports only beyond it
    for (int attempt = 0; e == hipSuccess; ++attempt) {
        if (kt) kt->attempts = (uint32_t)attempt + 1;
        // chain slots (hybrid: paths + side chains, 256-aligned)
        const size_t cap = hybrid ? ((paths + paths * wf.pool_factor / 4 + 255) & ~(size_t)255) : paths;
        if (hybrid && cap * (size_t)depth >= ((size_t)1 << 32)) { e = hipErrorOutOfMemory; break; }  // u32 node index
        const size_t pool = chain ? cap : paths * wf.pool_factor, level_cap = chain ? cap : pool / 2;
        int group = 1;
        // k_shadow: a node's light samples on `group` lanes (one each), or all on one lane (group 1: more than
        // 64 samples, or JSRT_SHADOW_SERIAL=1, an A/B knob)
        const char *ss = getenv("JSRT_SHADOW_SERIAL");
        if (ns > 1 && ns <= 64 && !(ss && ss[0] == '1' && !persist))
            while (group < ns) group *= 2;
        // hand-off slots: one per node of a level; level 0 holds all `paths` camera rays, the
        // deeper levels at most level_cap (k_shade poisons the batch before writing past it)
        const size_t hands = chain ? cap : std::max(level_cap, paths);
        const size_t shadow = persist ? hands * (size_t)group : 0;
        auto reserve = [&](Wavefront &w) {
            return chain ? w.reserve(cap, cap * (size_t)depth, cap, paths, sched, shadow)
                         : w.reserve(pool, pool, hands, paths, SCHED_TREE, shadow);
        };
        e = reserve(wf);
        if (e == hipSuccess && dual) {
            const hipError_t e2 = reserve(*wf.twin);
            if (e2 == hipErrorOutOfMemory) {  // no room for a second pool: one pool, one stream
                (void)hipGetLastError();
                wf.twin->release();
                dual = false;
                st2 = st;
            } else {
                e = e2;
            }
        }
        if (e != hipSuccess) break;
        WArgs W = wf.args;
        W.ns = ns;
        W.group = group;
        W.chain = chain ? 1 : 0;
        W.hybrid = hybrid ? 1 : 0;
        W.cap = (uint32_t)cap;
        // shadow hand-off bucketed by hit primitive (<= BKT_N buckets of consecutive primitives)
        const char *be = getenv("JSRT_BUCKET");
        int shift = 0;
        while (S.n_prims > 0 && ((S.n_prims - 1) >> shift) >= BKT_N) ++shift;
        W.bucket = (learned && !persist && S.n_prims > 0 && ns > 0 && ns <= 64 && !(be && be[0] == '0')) ? shift + 1 : 0;
        W.pool = pool;
        W.level_cap = level_cap;
        // children grouped by direction octant where the next cast walks a BVH (A/B on MI355X,
        // profiles/r03_s3_ab.txt: bunny +5.5 %; cornell -0.8 %, its keyed append costing k_shade 3 ms)
        const char *cs = getenv("JSRT_CHILD_SORT");
        W.child_sort = !chain && (cs ? (cs[0] == '1') : ((S.profile & PF_BVH) != 0));  // (tree appends only)
        // hand-off buckets keyed by the hit point's grid cell, with per-cell shadow-root masks, for flat
        // scenes (cornell +1.5 %, r03_s15); by hit primitive (runs of consecutive triangles) for meshes,
        // where the BVH and not the root loop carries the shadow casts (bunny +-0.2 %, r03_s6)
        const char *bg = getenv("JSRT_BUCKET_GRID");
        const bool grid = bg ? bg[0] == '1' : S.profile == PF_ANALYTIC;
        W.bucket_grid = (W.bucket && S.grid_cells > 0 && grid) ? 1 : 0;
        W.pixel_major = pixel_major ? 1 : 0;  // the order of a batch's paths (above)
        WArgs W2 = W;  // the twin pool: the same settings over its own buffers
        if (dual) {
            const WArgs &t = wf.twin->args;
            W2.ox = t.ox; W2.oy = t.oy; W2.oz = t.oz; W2.dx = t.dx; W2.dy = t.dy; W2.dz = t.dz;
            W2.addr = t.addr; W2.key = t.key; W2.path = t.path; W2.parent = t.parent; W2.t = t.t;
            W2.prim = t.prim; W2.ctx = t.ctx; W2.node = t.node; W2.child = t.child; W2.slot = t.slot;
            W2.hand = t.hand; W2.hnode = t.hnode; W2.root = t.root; W2.lvl = t.lvl; W2.qctr = t.qctr; W2.sray = t.sray;
            W2.scol = t.scol; W2.bkt = t.bkt; W2.bbase = t.bbase; W2.brank = t.brank;
            W2.list0 = t.list0; W2.list1 = t.list1; W2.endl = t.endl;
            W2.fixrec = t.fixrec; W2.fixctr = t.fixctr; W2.fixcap = t.fixcap;
        }
        if ((e = hipMemsetAsync(A.accum, 0, (size_t)A.ncols * A.H * 4 * sizeof(float), st)) != hipSuccess) break;
        if ((e = hipMemsetAsync(W.lvl + LVL_UNDER, 0, 2 * sizeof(uint32_t), st)) != hipSuccess) break;  // frame flags
        if ((e = hipMemsetAsync(W.fixctr, 0, sizeof(uint32_t), st)) != hipSuccess) break;
        if (dual && (e = hipMemsetAsync(W2.fixctr, 0, sizeof(uint32_t), st)) != hipSuccess) break;
        if (dual) {  // the side stream starts after everything enqueued on st so far
            if ((e = hipEventRecord(ev_start, st)) != hipSuccess || (e = hipStreamWaitEvent(st2, ev_start, 0)) != hipSuccess) break;
            if ((e = hipMemsetAsync(W2.lvl + LVL_UNDER, 0, 2 * sizeof(uint32_t), st2)) != hipSuccess) break;
        }
        // the frame flags (and, for progress, level counts) of both pools, read back after both streams idle
        auto read_flags = [&]() -> hipError_t {
            hipError_t r;
            if (dual && ((r = hipEventRecord(ev_end, st2)) != hipSuccess || (r = hipStreamWaitEvent(st, ev_end, 0)) != hipSuccess))
                return r;
            if ((r = hipMemcpyAsync(h_lvl, W.lvl, 64 * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) != hipSuccess) return r;
            if (dual && (r = hipMemcpyAsync(h_lvl + 64, W2.lvl, 64 * sizeof(uint32_t), hipMemcpyDeviceToHost, st)) != hipSuccess)
                return r;
            return hipStreamSynchronize(st);
        };
        auto flagged = [&](int k) { return h_lvl[k] != 0 || (dual && h_lvl[64 + k] != 0); };
        uint64_t bi = 0;  // batch index: even batches on (W, st), odd ones on (W2, st2)
        auto bounds = [&](uint32_t np) {  // per-level launch bound of a batch of np paths
            std::vector<size_t> b(depth, 0);
            if (hybrid) {  // level L: its live chains (<= cap)
                for (int L = 0; L < A.max_depth; ++L) {
                    b[L] = L == 0 ? np : cap;
                    if (L > 0 && !conservative && L < (int)wf.frac.size())  // (at least one block: a launch that
                        // can set LVL_UNDER for every level chains may continue into, even at a learned count of 0)
                        b[L] = std::min(cap, std::max<size_t>(256, (size_t)((double)np * wf.frac[L] * margin) + slack));
                }
                return b;
            }
            size_t ub = np;
            for (int L = 0; L < A.max_depth && ub > 0; ++L) {
                b[L] = ub;
                if (!conservative && L < (int)wf.frac.size())
                    b[L] = std::min(ub, std::max<size_t>(256, (size_t)((double)np * wf.frac[L] * margin) + slack));
                ub = L + 1 < A.max_depth ? std::min(ub * (size_t)S.max_children, level_cap) : 0;
            }
            return b;
        };
        const uint64_t total = (uint64_t)npix_total * A.spp;
        uint64_t done = 0;
        // stop: the callback aborted the frame.  redo_now: a progress check found a batch poisoned -- the frame is
        // redone at once instead of after its last batch, so that every pass is reported exactly once and from a
        // clean frame (a multi-rank caller keeps its collectives in step on the passes, tiles.render_progressive)
        bool stop = false, redo_now = false;
        for (uint32_t s0 = 0; s0 < (uint32_t)A.spp && e == hipSuccess && !stop && !redo_now; s0 += nsb) {
            const uint32_t nb = std::min<uint32_t>(nsb, (uint32_t)A.spp - s0);
            for (uint32_t p0 = 0; p0 < npix_total; p0 += npix, ++bi) {
                const bool odd = dual && (bi & 1);
                WArgs &Wb = odd ? W2 : W;
                const hipStream_t sb = odd ? st2 : st;
                Wb.p0 = p0;
                Wb.npix = std::min(npix, npix_total - p0);
                Wb.s0 = s0;
                Wb.npaths = Wb.npix * nb;
                Wb.cap = hybrid ? (uint32_t)cap : Wb.npaths;
                const std::vector<size_t> bound = learned ? bounds(Wb.npaths) : std::vector<size_t>();
                BatchSync sync;
                if (dual) {
                    sync.wait = bi > 0 ? ev_acc[(bi - 1) & 1] : nullptr;
                    sync.done = ev_acc[bi & 1];
                }
                if (split) {
                    Wavefront &pw = odd ? *wf.twin : wf;
                    sync.aux = pw.aux;
                    sync.shade_done = pw.ev_shade;
                    sync.shadow_done = pw.ev_shadow;
                }
                if (chain) run_batch_pf<true>(S, At, Wb, sb, kt, bound, &sync);
                else run_batch_pf<false>(S, At, Wb, sb, kt, bound, &sync);
                if ((e = hipGetLastError()) != hipSuccess) break;
                done += (uint64_t)Wb.npix * nb;
                if (kt) ++kt->batches;
                if (progress && A.kind != JSRT_RENDERER_INCREMENTAL && (!due || due())) {
                    // Simple / RandomMultisampling report {pass: 0, completion: pixels done / total} from
                    // inside their pixel loop (renderers.js:28-37): here after a batch, when a callback is
                    // due (the host's timelimit clock is checked first: no sync otherwise)
                    if ((e = read_flags()) != hipSuccess) break;
                    const bool clean = !flagged(LVL_FLAG) && !flagged(LVL_UNDER);
                    if (!clean) {
                        redo_now = true;
                        break;
                    }
                    const double c = (double)done / (double)total;
                    if (c > reported) {
                        reported = c;
                        if ((stop = !progress(0, c, clean))) break;
                    }
                }
                if (learned && ((wf.frac.empty() && !conservative) || conservative)) {
                    // learn the level counts: from the scene's first batch, or -- when that batch was
                    // not representative and a frame had to be redone -- as the maximum over every
                    // batch of the conservative redo, so later frames of this shape are not redone
                    if ((e = hipMemcpyAsync(h_lvl, Wb.lvl, 64 * sizeof(uint32_t), hipMemcpyDeviceToHost, sb)) != hipSuccess) break;
                    if ((e = hipStreamSynchronize(sb)) != hipSuccess) break;
                    if (!h_lvl[LVL_FLAG] && !h_lvl[LVL_UNDER]) {
                        if (wf.frac.size() < (size_t)A.max_depth) wf.frac.assign(A.max_depth, 0.0);
                        for (int L = 0; L < A.max_depth; ++L)
                            wf.frac[L] = std::max(wf.frac[L], (double)(hybrid ? h_lvl[2 * L] + h_lvl[2 * L + 1] : h_lvl[L]) / (double)Wb.npaths);
                    }
                }
            }
            if (e == hipSuccess && progress && A.kind == JSRT_RENDERER_INCREMENTAL && (!due || due())) {  // wait for the pass
                if ((e = read_flags()) != hipSuccess) break;
                const bool clean = !flagged(LVL_FLAG) && !flagged(LVL_UNDER);
                if (!clean) {
                    redo_now = true;
                    break;
                }
                const double c = (double)done / (double)total;
                if (c > reported) {
                    reported = c;
                    stop = !progress((int)(s0 + nb - 1), c, clean);
                }
            }
        }
        if (e != hipSuccess) break;
        if (stop) {  // an aborted frame is not redone (read_flags joins the side stream into st and waits for it)
            e = read_flags();
            aborted = true;
            break;
        }
        // The frame flags of both pools, every schedule.  read_flags also joins the side stream into st, so the
        // caller's stream orders after every batch of the frame (k_final below, and the caller's own work after
        // jsrt_render_device returns).  A frame that ended with a batch poisoned is redone, never returned: in
        // the round-4 draft of the hybrid chain this loop broke out for every chain-layout schedule before
        // reading the flags, so a hybrid frame whose side chains outgrew their slots came back with its
        // poisoned batches' pixels missing (tests/test_gpu_redo_streams.py).
        if ((e = read_flags()) != hipSuccess) break;
        if (!flagged(LVL_FLAG) && !flagged(LVL_UNDER)) break;
        if (!learned) {  // chain: only k_shade's k_fix_dirs records can run out (fix_record)
            // both pools take a record per ray slot (the overflow may have been in either); the setting stays for
            // later frames, like a doubled pool_factor.  A second overflow cannot happen: a level writes at most
            // one record per ray slot
            if (wf.fix_all && (!wf.twin || wf.twin->fix_all)) { e = hipErrorOutOfMemory; break; }
            wf.fix_all = true;
            if (wf.twin) wf.twin->fix_all = true;
        } else if (flagged(LVL_FLAG)) {  // a batch outgrew the pool: twice the pool, relearn the counts
            if (paths * wf.pool_factor > ((size_t)1 << 31) * (hybrid ? 4 : 1)) { e = hipErrorOutOfMemory; break; }
            wf.pool_factor *= 2;
            wf.frac.clear();
        } else {  // a level outgrew its learned bound: redo with the conservative bounds (and relearn)
            conservative = true;
            wf.frac.clear();
        }
        if (kt) kt->reset();
    }
    if (e != hipSuccess && dual) {  // nothing of this frame may still run on the side stream
        (void)hipStreamSynchronize(st2);
        (void)hipStreamSynchronize(st);
    }
    if (h_lvl) (void)hipHostFree(h_lvl);
    release_events();
    if (e != hipSuccess) return e;
    // an aborted frame leaves the caller's tile as the last preview left it (no k_final over a partial
    // accumulator), with the device idle (read_flags waited): jsrt.h's -4 contract
    if (aborted) return hipSuccess;
    if (!A.rgba) return hipSuccess;  // the caller takes the accumulator itself (jsrt_render_device_accum)
    const bool ev = kt && kt->on(KT_FINAL);
    if (ev) kt->ev[KT_FINAL].begin(st);
    hipLaunchKernelGGL(k_final, dim3(grid((size_t)A.ncols * A.H)), dim3(256), 0, st, A, (int32_t)A.spp);
    if (ev) kt->ev[KT_FINAL].end(st);
    return hipGetLastError();
}

hipError_t finish_accum(const float *accum, size_t n, int kind, int passes, uint32_t *rgba, float *colors, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (!accum || !rgba || passes < 1 || n > (size_t)INT32_MAX) return hipErrorInvalidValue;
    RenderArgs A{};
    A.kind = kind;
    A.ncols = (int32_t)n;
    A.H = 1;
    A.accum = const_cast<float *>(accum);
    A.rgba = rgba;
    A.colors = colors;
    hipLaunchKernelGGL(k_final, dim3(grid(n)), dim3(256), 0, st, A, (int32_t)passes);
    return hipGetLastError();
}

hipError_t render_preview(const RenderArgs &A, int passes, hipStream_t st) {
    if (!A.accum || !A.rgba || passes < 1) return hipErrorInvalidValue;
    if ((size_t)A.ncols * A.H == 0) return hipSuccess;
    hipLaunchKernelGGL(k_final, dim3(grid((size_t)A.ncols * A.H)), dim3(256), 0, st, A, (int32_t)passes);
    return hipGetLastError();
}


}  // namespace jsrt
