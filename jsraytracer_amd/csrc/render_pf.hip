// render_pf.hip — one kernel profile of the wavefront renderer: compiled once per profile with
// -DJSRT_PF=<PF_*> (jsraytracer_amd/build.py), instantiating run_batch and every level kernel it launches.
#include "render_levels.h"

#ifndef JSRT_PF
#error "compile with -DJSRT_PF=<kernel profile>"
#endif

// -DJSRT_PART=0|1|2 splits a profile into three objects compiled in parallel (build.py): the chain
// schedule's kernels, the tree schedule's, and the single-cast entries (jsrt_cast / jsrt_material_data).
#ifndef JSRT_PART
#define JSRT_PART -1
#endif

namespace jsrt {
#if JSRT_PART < 0 || JSRT_PART == 0
template void run_batch<JSRT_PF, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t, KernelTimes *,
                                       const std::vector<size_t> &, const BatchSync *);
#endif
#if JSRT_PART < 0 || JSRT_PART == 1
template void run_batch<JSRT_PF, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t, KernelTimes *,
                                        const std::vector<size_t> &, const BatchSync *);
#endif
#if JSRT_PART < 0 || JSRT_PART == 2
template void cast_rays_pf<JSRT_PF>(const DScene &, const float *, uint32_t, double, double, int, double *, int32_t *,
                                   hipStream_t);
template void material_data_pf<JSRT_PF>(const DScene &, const float *, uint32_t, double *, int32_t *, float *, float *,
                                        float *, float *, float *, hipStream_t);
#endif
}  // namespace jsrt

#if defined(JSRT_X_STAMPS) && JSRT_PF == 0 && JSRT_PART == 0
// (timing experiment only) the per-phase cycle sums of the analytic chain k_shade (render_levels.h g_xst),
// and reset them
extern "C" int jsrt_x_stamps(unsigned long long *out) {
    std::vector<unsigned long long> h((size_t)jsrt::XST_SLOTS * 16);
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(jsrt::g_xst), h.size() * 8) != hipSuccess) return -1;
    for (int k = 0; k < 16; ++k) out[k] = 0;
    for (size_t i = 0; i < h.size(); ++i) out[i % 16] += h[i];
    std::fill(h.begin(), h.end(), 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(jsrt::g_xst), h.data(), h.size() * 8) == hipSuccess ? 0 : -1;
}
#endif
