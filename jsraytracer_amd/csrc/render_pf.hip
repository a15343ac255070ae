// render_pf.hip — one kernel profile of the wavefront renderer: compiled once per profile with
// -DJSRT_PF=<PF_*> (jsraytracer_amd/build.py), instantiating run_batch and every level kernel it launches.
#include "render_levels.h"

#ifndef JSRT_PF
#error "compile with -DJSRT_PF=<kernel profile>"
#endif

namespace jsrt {
template void run_batch<JSRT_PF, true>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t, KernelTimes *,
                                       const std::vector<size_t> &);
template void run_batch<JSRT_PF, false>(const DScene &, const RenderArgs &, const WArgs &, hipStream_t, KernelTimes *,
                                        const std::vector<size_t> &);
template void cast_rays_pf<JSRT_PF>(const DScene &, const float *, uint32_t, double, double, int, double *, int32_t *,
                                   hipStream_t);

// A/B instrumentation (variant builds with -DJSRT_DBG_COUNT for one profile): the counters live in
// this profile's code object, so they are read back from here (tools/dbg_counts.py)
#ifdef JSRT_DBG_COUNT
extern "C" int jsrt_debug_counters(unsigned long long *out, int n) {
    if (n > 256) n = 256;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), n * sizeof(unsigned long long)) != hipSuccess) return -1;
    static const unsigned long long zero[256] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), zero, sizeof zero) == hipSuccess ? 0 : -1;
}
#endif
}  // namespace jsrt
