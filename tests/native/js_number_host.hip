// Host build of jsraytracer_amd/csrc/js_number.h for the CPU test suite (tests/test_js_number.py):
// the device's toPrecision(8) fast path and its exact fallback, compiled for the host.
#include "../../jsraytracer_amd/csrc/js_number.h"

extern "C" void tp8_fast(const double *x, double *out, long n) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::to_precision8(x[i]);
}
extern "C" void tp8_sl(const double *x, double *out, long n) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::to_precision8_sl(x[i]);
}
extern "C" void tp8_exact(const double *x, double *out, long n) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::to_precision8_exact(x[i]);
}
extern "C" void js_fmod_n(const double *a, const double *b, double *out, long n) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::js_fmod(a[i], b[i]);
}
