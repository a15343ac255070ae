// Host build of the shadow cast's AABB any-hit filter (jsraytracer_amd/csrc/device_common.h box_any_f32) for
// the CPU tests (tests/test_box_any.py): its decisions against the exact aabb_intersect + World.cast bounds.
#include "../../jsraytracer_amd/csrc/device_common.h"

// boxes: n x 6 floats (center xyz, half xyz); rays: n x 6 floats (o xyz, d xyz).  Per case: exact[i] = 1 if the
// reference accepts the hit (minD < t < maxD), dec[i] = box_any_f32's decision, tf[i] = its distance estimate.
extern "C" void box_any(const float *boxes, const float *rays, long n, double minD, double maxD, int *exact,
                        int *dec, double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *b = boxes + 6 * i, *r = rays + 6 * i;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double t = jsrt::aabb_intersect(b, b + 3, o, d, minD, maxD);
        exact[i] = (t > minD && t < maxD) ? 1 : 0;
        double e = 0;
        dec[i] = jsrt::box_any_f32(b, b + 3, o, jsrt::box_ray(d), minD, maxD, e);
        tf[i] = e;
    }
}

// planar: n x 12 doubles (inv rows 0..2), kinds[i] (JSRT_GEOM_PLANE / SQUARE / CIRCLE), rays n x 6 floats
extern "C" void planar_any(const double *inv, const int *kinds, const float *rays, long n, double minD, double maxD,
                           int *exact, int *dec, double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *r = rays + 6 * i;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double t = jsrt::planar_intersect(kinds[i], inv + 12 * i, o, d, minD, maxD);
        exact[i] = (t > minD && t < maxD) ? 1 : 0;
        double e = 0;
        dec[i] = jsrt::planar_any_f32(kinds[i], inv + 12 * i, o, d, minD, maxD, e);
        tf[i] = e;
    }
}

// spheres (unit sphere, local rays): rays n x 6 floats
extern "C" void sphere_any(const float *rays, long n, double minD, double maxD, int *exact, int *dec, double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *r = rays + 6 * i;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double t = jsrt::sphere_static(o, d, minD);
        exact[i] = (t > minD && t < maxD) ? 1 : 0;
        double e = 0;
        dec[i] = jsrt::sphere_any_f32(o, d, minD, maxD, e);
        tf[i] = e;
    }
}

// triangles: n x 9 floats (3 vertices), rays n x 6 floats; the DTri fields as mesh_build.cpp computes them
extern "C" void tri_any(const float *verts, const float *rays, long n, double minD, double maxD, int *exact, int *dec,
                        double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *p = verts + 9 * i, *r = rays + 6 * i;
        jsrt::DTri T{};
        float a[3], b[3], h[3];
        for (int k = 0; k < 3; ++k) {
            a[k] = p[3 + k] - p[k];
            b[k] = p[6 + k] - p[k];
        }
        h[0] = (float)((double)a[1] * b[2] - (double)a[2] * b[1]);
        h[1] = (float)((double)a[2] * b[0] - (double)a[0] * b[2]);
        h[2] = (float)((double)a[0] * b[1] - (double)a[1] * b[0]);
        const double hn = sqrt((double)h[0] * h[0] + (double)h[1] * h[1] + (double)h[2] * h[2]);
        for (int k = 0; k < 3; ++k) T.n[k] = hn > 0.00001 ? (float)((double)h[k] * (1 / hn)) : h[k];
        for (int k = 0; k < 3; ++k) {
            T.p0[k] = p[k];
            T.v0[k] = a[k];
            T.v1[k] = b[k];
        }
        T.delta = (double)T.n[0] * p[0] + (double)T.n[1] * p[1] + (double)T.n[2] * p[2];
        T.d00 = (double)a[0] * a[0] + (double)a[1] * a[1] + (double)a[2] * a[2];
        T.d11 = (double)b[0] * b[0] + (double)b[1] * b[1] + (double)b[2] * b[2];
        T.d01 = (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2];
        T.denom = T.d00 * T.d11 - T.d01 * T.d01;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double t = jsrt::tri_intersect(T, o, d);
        exact[i] = (t > minD && t < maxD) ? 1 : 0;
        double e = 0;
        dec[i] = jsrt::tri_any_f32(T, o, d, minD, maxD, e);
        tf[i] = e;
    }
}

// closest-hit forms (World.cast's closest hit keeps minD < t < lim): exact[i] = 1 if the reference's distance
// t_ref is accepted, tref[i] = t_ref; dec[i] = the filter's decision, tf[i] = its (exact) distance when 1
extern "C" void box_closest(const float *boxes, const float *rays, const double *lims, long n, double minD, double maxD,
                            int *exact, double *tref, int *dec, double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *b = boxes + 6 * i, *r = rays + 6 * i;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double lim = lims[i] < maxD ? lims[i] : maxD;
        const double t = jsrt::aabb_intersect(b, b + 3, o, d, minD, maxD);
        exact[i] = (t > minD && t < lim) ? 1 : 0;
        tref[i] = t;
        double e = 0;
        dec[i] = jsrt::box_closest_f32(b, b + 3, o, d, jsrt::box_ray(d), minD, lim, e);
        tf[i] = e;
    }
}
extern "C" void sphere_closest(const float *rays, const double *lims, long n, double minD, double maxD, int *exact,
                               double *tref, int *dec, double *tf) {
    for (long i = 0; i < n; ++i) {
        const float *r = rays + 6 * i;
        const jsrt::F3 o = jsrt::f3(r[0], r[1], r[2]), d = jsrt::f3(r[3], r[4], r[5]);
        const double lim = lims[i] < maxD ? lims[i] : maxD;
        const double t = jsrt::sphere_static(o, d, minD);
        exact[i] = (t > minD && t < lim) ? 1 : 0;
        tref[i] = t;
        double e = 0;
        dec[i] = jsrt::sphere_closest_f32(o, d, minD, lim, e);
        tf[i] = e;
    }
}

// the spherePick stability test on the bits (device_common.h f32_stable_bits): out[i] = 1 if stable
extern "C" void stable_bits(const double *d, long n, int *out) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::f32_stable_bits(d[i]) ? 1 : 0;
}
