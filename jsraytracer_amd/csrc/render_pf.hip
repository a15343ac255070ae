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
template void material_data_pf<JSRT_PF>(const DScene &, const float *, uint32_t, double *, int32_t *, float *, float *,
                                        float *, float *, float *, hipStream_t);
}  // namespace jsrt
