// render_kernel.h — launch interface of the wavefront renderer (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "device_scene.h"

namespace jsrt {

constexpr int MAX_TREE_DEPTH = 16;  // maxRecursionDepth supported (levels of the breadth-first schedule)
constexpr int LVL_FLAG = 63;        // WArgs::lvl word set when a batch outgrew its pool (frame redone)
constexpr int LVL_UNDER = 62;       // WArgs::lvl word set when a level outgrew its launch bound
static_assert(2 * MAX_TREE_DEPTH + 2 <= LVL_UNDER, "hybrid chain count pairs lvl[2L, 2L + 1] below the flags");
constexpr int BKT_N = 64;           // buckets of the shadow hand-off (hit primitive >> shift)
constexpr int BKT_S = 16;           // slices per bucket (block index % BKT_S): spreads the counters' atomics
constexpr int BKT_K = BKT_N * BKT_S;  // counters per level, key = bucket * BKT_S + slice
constexpr int BKT_LEVEL = 3 * BKT_K + 64;  // words per level: counts, (spare), offsets (+ total)

struct RenderArgs {
    int32_t W, H, kind, max_depth;
    int32_t s_begin, s_end, spp;  // (unused by the wavefront path: whole frames)
    uint32_t seed;
    int32_t x_offset, x_delt, col_block, ncols;
    float *accum;      // ncols*H*4 f32 accumulator
    uint32_t *rgba;    // ncols*H packed RGBA8 (PixelBuffer bytes), written by k_final
    float *colors;     // ncols*H*4 final colour (nullable)
    int32_t final_pass;
    int32_t patches_x; // ceil(ncols / 8)
    int32_t patches;   // patches_x * ceil(H / 8)
    int32_t samples_per_batch;  // progress granularity: cap on samples per batch (<= 0: none)
    int32_t tile_p;    // > 0: pixel order of the batches in tiles of tile_p x tile_p patches (render_levels.h pixel_of)
};

// node info bits (k_shade -> k_shadow / k_reduce / k_resolve)
constexpr uint32_t INFO_HIT = 1u, INFO_LIT = 2u, INFO_MISS = 16u;
// child j's weight is exactly (1, 1, 1) and its k exactly 1: its record's second plane is not stored and
// ((v * col) * w) * k is v * col bit for bit (x * 1 is exact in f32 and in f64)
constexpr uint32_t INFO_UNIT0 = 32u, INFO_UNIT1 = 64u;
constexpr int INFO_NCHILD_SHIFT = 2;

// Device buffers of one batch.  Two schedules share them (render.hip):
//   chain (no node has more than one child): ray q of the batch is path q at every level; node
//         records are level-major [L * cap + q]; the child ray replaces its parent's ray.
//         hybrid chain (branching materials, W.hybrid): the same, and a node's second child starts a
//         side chain in a slot appended after the paths (the chains started at level s have the ids
//         npaths + [side(< s), side(<= s))).  Level L > 0 visits only its live chains: those that continue
//         from L - 1, listed by k_shade(L - 1) (list[L & 1]), then the side chains started at L.  Counts:
//         the 64-bit word lvl[2L, 2L + 1] = {chains continuing into L, side chains started at L}, appended
//         with one 64-bit atomic per block.  A chain's last level is endl[slot].  A side chain's colour is
//         resolved bottom-up before its parent's and left in slot[parent node] (k_resolve_side).
//   tree  (branching materials): rays and nodes share pool slots; level L occupies
//         [base_L, base_L + count_L) with counts on the device; children are appended.
struct WArgs {
    // rays
    float *ox, *oy, *oz, *dx, *dy, *dz;
    uint32_t *addr;    // ray-tree address of the World.color frame this ray opens
    uint32_t *key;     // mix(mix(seed, pixel), sample): RNG key of the path
    uint32_t *path;    // tree: path index in the batch
    uint32_t *parent;  // tree: child slot 2 * parent + j, NO_PARENT (camera ray) or DEAD_RAY; hybrid chain:
                       // [side chain] its branching parent's node index
    double *t;         // closest hit
    int32_t *prim, *ctx;  // prim: hit primitive, -1 miss / to trace, NO_RAY no ray
    // nodes
    float4 *node;      // [i]: {surface colour (the ambient until k_shadow adds the lights), info}
    // record planes (plane stride nstride / hstride): every access is one coalesced 16-B load per lane
    float4 *child;     // [(2 * j + part) * nstride + i]: part 0 {col.xyz, w.x}, part 1 {w.y, w.z, k (f64)}
    float4 *slot;      // tree: [j * nstride + i] the child's colour; hybrid chain: [i] the second child's
    float4 *hand;      // [k * hstride + h], k < 6: shadow hand-off of a lit node (h: path / level index, render_levels.h store_hand)
    uint32_t *hnode;   // [h]: the node (level index / chain slot) of bucketed hand-off slot h
    float *root;       // tree: [3 * path] root colours
    uint32_t *lvl;     // tree: [L] ray count of level L; [LVL_FLAG] overflow flag
    uint32_t *list0, *list1;  // hybrid chain: the live chain slots of odd (list1) / even (list0) levels > 0
    uint8_t *endl;     // hybrid chain: [slot] the chain's last level
    // persistent casts (SDF scenes, render.hip k_extend_q / k_shadow_*): work counters per level
    // ([L] extend, [32 + L] shadow) and the shadow rays of the light samples ([e] = k_shadow lane e)
    uint32_t *qctr;
    // child directions of unstable spherePicks (k_shade's INFO_FIX), recomputed by k_fix_dirs before the next
    // level's casts: fixctr[0] records of 3 x uint4 {dst0, dst1, key, addr} {fix0, fix1, nchild, -} {N, -}
    uint4 *fixrec;
    uint32_t *fixctr;
    uint32_t fixcap;
    int32_t force_fix;  // JSRT_FORCE_EXACT_PICK=1 (tests): every diffuse pick through k_fix_dirs
    float4 *sray;      // [e] {P.xyz, -}, [sstride + e] {delta.xyz, -}
    float4 *scol;      // [e] {unshadowed colour.xyz, state: 0 no cast / lit, 1 cast pending, 2 shadowed}
    // hit-primitive buckets of the lit nodes per level (W.bucket), BKT_LEVEL words from L * BKT_LEVEL:
    // [k] lit nodes of key k (k_extend), [2 BKT_K + k] its first hand-off slot (k_bucket_offsets),
    // [3 BKT_K] the level's lit nodes
    uint32_t *bkt;
    uint32_t *bbase;   // [block * BKT_N + bucket]: the block's first slot in its key's range (k_extend)
    uint32_t *brank;   // [ray]: a lit hit's rank among its block's hits in its bucket (k_extend)
    // batch
    uint32_t p0, npix, s0, npaths;
    int32_t ns;        // light samples per lit node
    int32_t group;     // lanes per node in k_shadow: a power of two >= ns (<= 64), or 1 (serial)
    int32_t chain;     // schedule
    int32_t hybrid;    // chain schedule with side chains (level counts on the device)
    uint32_t cap;      // chain schedule: slots per level (node [L * cap + slot]); npaths without side chains
    int32_t bucket;    // tree schedule: 0, or 1 + shift: k_shadow reads lit nodes bucketed by hit primitive >> shift (bkt)
    int32_t child_sort; // tree schedule: k_shade appends a block's children grouped by direction octant
    int32_t bucket_grid; // bucketed hand-off keyed by the hit point's grid cell (DScene::grid_*), not the primitive
    int32_t pixel_major; // path q of the batch: pixel q / nsb, sample q % nsb (a pixel's samples side by side);
                         // else sample q / npix, pixel q % npix (render.hip k_gen / k_accum / k_resolve)
    size_t pool, level_cap;
    size_t nstride, hstride;  // plane strides of child / slot and of hand
    size_t sstride;           // entries of sray / scol (0: persistent casts not used)
};

// Accumulation order across the two batch streams (render_frame): the batch's k_accum / k_resolve waits
// for `wait` (the previous batch's accumulation, on the other stream) and records `done` after itself.
// aux (optional): the stream k_shadow runs on, so that level L's shadow samples overlap level L + 1's
// closest-hit casts (they share no buffer); shade_done / shadow_done order k_shadow(L) after k_shade(L)
// and k_shade(L + 1) -- which rewrites the hand-off -- after k_shadow(L).
struct BatchSync {
    hipEvent_t wait = nullptr, done = nullptr;
    hipStream_t aux = nullptr;
    hipEvent_t shade_done = nullptr, shadow_done = nullptr;
};

struct Wavefront {  // owns the batch buffers (cached per scene)
    void *mem = nullptr;
    // The second batch pool and the stream it runs on: consecutive batches alternate between two pools
    // and two streams so one batch's levels overlap the other's (render_frame); created on first use.
    Wavefront *twin = nullptr;
    hipStream_t side = nullptr;
    // this pool's k_shadow stream and its two ordering events (BatchSync::aux), created on first use
    hipStream_t aux = nullptr;
    hipEvent_t ev_shade = nullptr, ev_shadow = nullptr;
    // tree / hybrid chain schedule, learned per scene, batch shape and schedule: pool size (tree: x paths;
    // hybrid: paths + paths x pool_factor / 4 chain slots) and level counts
    size_t pool_paths = 0, pool_factor = 8;
    int pool_mode = -1;
    bool fix_all = false;  // k_fix_dirs records for every ray slot (a frame ran out of the default 1/8)
    std::vector<double> frac;  // level L ray count / paths of the first batch
    size_t cap_bytes = 0;
    WArgs args{};
    // rays: ray slots; nodes: node records; hands: hand-off records; paths: root colours
    // shadow: light-sample entries of the persistent shadow casts (0 if unused)
    // mode: 0 chain, 1 tree, 2 hybrid chain
    hipError_t reserve(size_t rays, size_t nodes, size_t hands, size_t paths, int mode, size_t shadow = 0);
    void release();  // frees the buffers (the learned pool / bounds stay)
    ~Wavefront();
};

enum { KT_GEN, KT_EXTEND, KT_SHADE, KT_SHADOW, KT_REDUCE, KT_ACCUM, KT_FINAL, KT_RESOLVE, KT_N };
constexpr int SCHED_CHAIN = 0, SCHED_TREE = 1, SCHED_HYBRID = 2;
extern const char *const KT_NAMES[KT_N];

struct EventPairs {  // reusable HIP events bracketing every launch of one kernel kind
    std::vector<hipEvent_t> b, e;
    size_t used = 0;
    void begin(hipStream_t s);
    void end(hipStream_t s);
    double total_ms(uint32_t *lost = nullptr) const;  // after the stream is synchronized; lost: pairs without a time
    ~EventPairs();
};

struct KernelTimes {
    EventPairs ev[KT_N];
    uint32_t mask = ~0u;  // stages whose launches are bracketed by events
    bool one_stream = false;  // jsrt.h JSRT_EVENTS_ONE_STREAM: no overlapping batch streams
    uint32_t batches = 0; // (pixels x samples) batches completed
    uint32_t attempts = 0; // frame attempts (a poisoned frame is redone)
    bool on(int k) const { return (mask >> k) & 1u; }
    void reset() {
        batches = 0;
        for (auto &p : ev) p.used = 0;
    }
};

// Renders all spp samples of the owned pixels: A.accum must hold ncols*H*4 floats.
// `ns` = light samples per lit node (sum over lights; point lights count 1).
// progress(pass, completion, clean) -> false aborts.  It is called after samples [0, pass] of every
// pixel are in A.accum and the stream is idle; clean = no batch so far outgrew its pool / bounds
// (so the accumulator holds exactly the reference's sums and render_preview may publish it).
// due (nullable): whether a callback is due now (the host's timelimit clock); the frame syncs and calls
// progress only then.
hipError_t render_frame(const DScene &S, const RenderArgs &A, int ns, Wavefront &wf, hipStream_t st, KernelTimes *kt,
                        size_t max_paths, const std::function<bool(int, double, bool)> &progress,
                        const std::function<bool()> &due = nullptr);

// Device bytes of the batch state per path of a batch (Wavefront::reserve for the schedule and pool
// render_frame picks for this scene): caps the default batch size.
size_t wavefront_bytes_per_path(const DScene &S, int ns, int max_depth);

// Running mean of the first `passes` samples -> A.rgba / A.colors (k_final with times(1/passes),
// renderers.js:93-98): the image IncrementalMultisamplingRenderer holds after pass passes-1.
hipError_t render_preview(const RenderArgs &A, int passes, hipStream_t st);
// k_final over n accumulators (f32 x 4 each, any pixel order): renderer `kind`'s final colour (Incremental:
// times(1 / passes)) and PixelBuffer.setColor's RGBA8 (jsrt_finish_accum).
hipError_t finish_accum(const float *accum, size_t n, int kind, int passes, uint32_t *rgba, float *colors, hipStream_t st);

// World.cast (world.js:28-30) of n rays (device buffers: n x 6 f32 rays, origin w = 1, direction
// w = 0): closest-hit distance and DPrim index (-1: none).  The jsrt_cast entry (known-answer tests).
hipError_t cast_rays(const DScene &S, const float *d_rays, uint32_t n, double min_dist, double max_dist, bool transparent,
                     double *d_t, int32_t *d_prim, hipStream_t st);

// World.color(ray, 1) up to Material.color for n rays (jsrt_material_data): closest hit of World.cast(ray,
// 0) and the hit's material_data -- world normal (n x 4), world position (n x 4), UV (n x 3), triangle
// barycentric coordinates (n x 3), SDF basecolor (n x 3), NaN where absent.
hipError_t material_data_rays(const DScene &S, const float *d_rays, uint32_t n, double *d_t, int32_t *d_prim,
                              float *d_nrm, float *d_pos, float *d_uv, float *d_bary, float *d_bc, hipStream_t st);
// SDF.distance of SDF geometry g's root at n local points (f32 x 4) (jsrt_sdf_distance).
hipError_t sdf_distance_points(const DScene &S, int g, const float *d_pts, uint32_t n, double *d_out, hipStream_t st);

// Owned column c -> image column px (see jsrt.h jsrt_render_device).
__host__ __device__ inline int32_t owned_to_px(int32_t c, int32_t x_offset, int32_t x_delt, int32_t col_block) {
    if (col_block <= 1) return x_offset + c * x_delt;
    return ((c / col_block) * x_delt + x_offset) * col_block + (c % col_block);
}

}  // namespace jsrt
