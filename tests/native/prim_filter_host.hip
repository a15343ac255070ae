// TEST INFRASTRUCTURE: the device's analytic-primitive pre-tests (csrc/prim_filter.h) and the exact
// intersections they stand in front of (csrc/device_common.h), compiled for the host so that
// tests/test_prim_filter.py can check every decision on millions of random rays.
#include "../../jsraytracer_amd/csrc/device_common.h"

using namespace jsrt;

// kind: JSRT_GEOM_*; rays: n x 6 floats (o, d, world space); lims: n x 3 (minD, maxD, lim).
// tout[i]: the exact distance; exact[i]: 1 if the exact test's distance is accepted (minD < t < lim), else 0; filt[i]: FLT_*.
extern "C" void filt_eval(int kind, const double *inv, const float *c, const float *h, const float *rays,
                          const double *lims, long n, int *exact, int *filt, double *tout) {
    FRows R;
    frows_build(inv, R);
    for (long i = 0; i < n; ++i) {
        const F3 o = f3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), d = f3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        const double minD = lims[3 * i], maxD = lims[3 * i + 1], lim = lims[3 * i + 2];
        const float oabs = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
        const float dabs = fmaxf(fabsf(d.x), fmaxf(fabsf(d.y), fabsf(d.z)));
        const FBounds B = fbounds(minD, maxD, lim);
        double t;
        int f;
        switch (kind) {
        case JSRT_GEOM_PLANE:
        case JSRT_GEOM_SQUARE:
        case JSRT_GEOM_CIRCLE:
            t = planar_intersect(kind, inv, o, d, minD, lim);
            f = planar_filter(kind, R, fray(R, o, d, oabs, dabs), B);
            break;
        case JSRT_GEOM_AABB:
            t = aabb_intersect(c, h, xf_point(inv, o), xf_dir(inv, d), minD, maxD);
            f = aabb_filter(R, c, h, fray(R, o, d, oabs, dabs), B);
            break;
        case JSRT_GEOM_SPHERE:
            t = sphere_static(xf_point(inv, o), xf_dir(inv, d), minD);
            f = sphere_filter(R, fray(R, o, d, oabs, dabs), B);
            break;
        default:
            t = -INFINITY;
            f = FLT_EXACT;
        }
        exact[i] = (t > minD && t < lim && t < maxD) ? 1 : 0;
        tout[i] = t;
        filt[i] = f;
    }
}
