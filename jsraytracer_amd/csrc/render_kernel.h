// render_kernel.h — launch interface of the wavefront renderer (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "device_scene.h"

namespace jsrt {

constexpr int MAX_TREE_DEPTH = 16;  // maxRecursionDepth supported (levels of the breadth-first schedule)

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
    int32_t pad;
};

// node info bits (k_shade -> k_shadow / k_reduce)
constexpr uint32_t INFO_HIT = 1u, INFO_LIT = 2u;
constexpr int INFO_NCHILD_SHIFT = 2;

// Device buffers of one batch (structure of arrays over a ray pool shared by all levels).
struct WArgs {
    // rays (index = pool slot); level L occupies [base_L, base_L + count_L)
    float *ox, *oy, *oz, *dx, *dy, *dz;
    uint32_t *addr;    // ray-tree address of the World.color frame this ray opens
    uint32_t *key;     // mix(mix(seed, pixel), sample): RNG key of the path
    uint32_t *path;    // path index in the batch
    uint32_t *parent;  // 2 * parent slot + child index, or NO_PARENT for camera rays
    double *t;         // closest hit
    int32_t *prim, *ctx;
    // nodes (same index as the ray that reached them)
    uint32_t *info;
    float *sx, *sy, *sz;  // ambient, then resolved surface colour
    float *ccol, *cw, *slot;  // [3 * (2 * i + j)]: child weights and child results
    double *ck;               // [2 * i + j]
    // shade -> shadow hand-off of one level (index = ray index within the level): the node's
    // material_data after getBaseFactors, as colorFromLightSample reads it
    float *sox, *soy, *soz;          // position (shadow-ray origin)
    float *fnx, *fny, *fnz;          // N (flipped to the viewer's side)
    float *frx, *fry, *frz;          // R
    float *ftx, *fty, *ftz;          // refraction direction (0 when none)
    float *fdx, *fdy, *fdz;          // diffuse colour (basecolor applied)
    float *fsx, *fsy, *fsz;          // specular colour
    double *fkr;                     // Fresnel reflection factor (1 for Phong)
    int32_t *fmat;                   // material index
    float *scx, *scy, *scz;          // [level_idx * ns + sample]: unshadowed sample colour or 0
    float *root;       // [3 * path]
    uint32_t *counter; // append counter of the next level
    // batch
    uint32_t p0, npix, s0, npaths;
    int32_t ns;        // light samples per lit node
    uint32_t pad;
    size_t pool, level_cap;
};

struct Wavefront {  // owns the batch buffers (cached per scene)
    void *mem = nullptr;
    size_t cap_bytes = 0, cap_pool = 0, cap_level = 0;
    int cap_ns = 0;
    WArgs args{};
    hipError_t reserve(size_t pool, size_t level_cap, int ns);
    ~Wavefront();
};

enum { KT_GEN, KT_EXTEND, KT_SHADE, KT_SHADOW, KT_REDUCE, KT_ACCUM, KT_FINAL, KT_LIGHTSUM, KT_N };
extern const char *const KT_NAMES[KT_N];

struct EventPairs {  // reusable HIP events bracketing every launch of one kernel kind
    std::vector<hipEvent_t> b, e;
    size_t used = 0;
    void begin(hipStream_t s);
    void end(hipStream_t s);
    double total_ms() const;  // after the stream is synchronized
    ~EventPairs();
};

struct KernelTimes {
    EventPairs ev[KT_N];
    void reset() {
        for (auto &p : ev) p.used = 0;
    }
};

// Renders all spp samples of the owned pixels: A.accum must hold ncols*H*4 floats.
// `ns` = light samples per lit node (sum over lights; point lights count 1).
// progress(pass, completion) -> false aborts.
hipError_t render_frame(const DScene &S, const RenderArgs &A, int ns, Wavefront &wf, hipStream_t st, KernelTimes *kt,
                        size_t max_paths, const std::function<bool(int, double)> &progress);

// Owned column c -> image column px (see jsrt.h jsrt_render_device).
__host__ __device__ inline int32_t owned_to_px(int32_t c, int32_t x_offset, int32_t x_delt, int32_t col_block) {
    if (col_block <= 1) return x_offset + c * x_delt;
    return ((c / col_block) * x_delt + x_offset) * col_block + (c % col_block);
}

}  // namespace jsrt
