// render_kernel.h — launch interface of the render kernel (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_scene.h"

namespace jsrt {

constexpr int MAX_TREE_DEPTH = 16;  // maxRecursionDepth supported by the per-lane frame stack

struct RenderArgs {
    int32_t W, H, kind, max_depth;
    int32_t s_begin, s_end, spp;  // samples [s_begin, s_end) of spp this launch
    uint32_t seed;
    int32_t x_offset, x_delt, col_block, ncols;
    float *accum;      // ncols*H*4 f32 accumulator (in/out across launches), may be null if one launch
    uint32_t *rgba;    // ncols*H packed RGBA8 (PixelBuffer bytes), written on the final launch
    float *colors;     // ncols*H*4 final colour (nullable)
    int32_t final_pass;
    int32_t patches_x; // ceil(ncols / 8)
    int32_t patches;   // patches_x * ceil(H / 8)
    int32_t pad;
};

// Owned column c -> image column px (see jsrt.h jsrt_render_device).
__host__ __device__ inline int32_t owned_to_px(int32_t c, int32_t x_offset, int32_t x_delt, int32_t col_block) {
    if (col_block <= 1) return x_offset + c * x_delt;
    return ((c / col_block) * x_delt + x_offset) * col_block + (c % col_block);
}

hipError_t launch_render(const DScene &scene, const RenderArgs &args, hipStream_t stream);

}  // namespace jsrt
