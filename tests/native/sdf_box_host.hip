// Host build of the box-union SDF (jsraytracer_amd/csrc/device_common.h sdf_minbox) for the CPU tests
// (tests/test_sdf_box.py): the one-square-root union against the reference's Math.min of BoxSDFs.
#include "../../jsraytracer_amd/csrc/device_common.h"

// boxes: n x 4 doubles (size xyz, pad); pts: m x 3 floats.  out_ref: Math.min chain of sdf_box, out: sdf_minbox
extern "C" void box_union(const double *boxes, int n, const float *pts, long m, double *out_ref, double *out) {
    for (long j = 0; j < m; ++j) {
        const jsrt::F3 P = jsrt::f3(pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]);
        double r = jsrt::sdf_box(boxes, P);
        for (int i = 1; i < n; ++i) r = jsrt::js_min(r, jsrt::sdf_box(boxes + 4 * i, P));
        out_ref[j] = r;
        out[j] = jsrt::sdf_minbox(boxes, n, P);
    }
}

// the Menger cross (sdf_cross, boxes: 3 x 4 doubles as the host matched them) against sdf_minbox
extern "C" void cross_union(const double *boxes, const float *pts, long m, double *out_ref, double *out) {
    for (long j = 0; j < m; ++j) {
        const jsrt::F3 P = jsrt::f3(pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]);
        out_ref[j] = jsrt::sdf_minbox(boxes, 3, P);
        out[j] = jsrt::sdf_cross(boxes, P);
    }
}
