// Host build of the device's Math.pow fast path (jsraytracer_amd/csrc/device_common.h pow_int_dd) for
// tests/test_pow_parity.py.
#include "../../jsraytracer_amd/csrc/device_common.h"

extern "C" void pow_dd(const double *x, const double *y, long n, double *out) {
    for (long i = 0; i < n; ++i) out[i] = jsrt::pow_int_dd(x[i], (int)y[i]);
}
