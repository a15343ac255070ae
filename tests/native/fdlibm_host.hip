// Host build of jsraytracer_amd/csrc/fdlibm.h for the CPU tests (tests/test_fdlibm.py).
#include "../../jsraytracer_amd/csrc/fdlibm.h"

extern "C" void trig_n(const double *x, double *out, long n) {  // per argument: sin, cos, acos
    for (long i = 0; i < n; ++i) {
        double s, c;
        jsrt::fdlibm::sin_cos(x[i], s, c);
        out[3 * i] = s;
        out[3 * i + 1] = c;
        out[3 * i + 2] = jsrt::fdlibm::acos(x[i]);
    }
}
// fdlibm's npio2_hw table against the high words fdlibm.h computes in its place
extern "C" int npio2_hw_ok(void) {
    const uint32_t tab[32] = {
        0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C, 0x4025FDBB, 0x402921FB,
        0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C, 0x40346B9C, 0x4035FDBB, 0x40378FDB, 0x403921FB,
        0x403AB41B, 0x403C463A, 0x403DD85A, 0x403F6A7A, 0x40407E4C, 0x4041475C, 0x4042106C, 0x4042D97C,
        0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB, 0x4046C6CB, 0x40478FDB, 0x404858EB, 0x404921FB};
    for (int n = 1; n <= 32; ++n)
        if (jsrt::fdlibm::hi_word((double)n * 1.57079632679489655800e+00) != tab[n - 1]) return 0;
    return 1;
}

extern "C" void uv_n(const double *xy, double *out, long n) {  // per (x, y): atan2(y, x), asin(x)
    for (long i = 0; i < n; ++i) {
        out[2 * i] = jsrt::fdlibm::atan2(xy[2 * i + 1], xy[2 * i]);
        out[2 * i + 1] = jsrt::fdlibm::asin(xy[2 * i]);
    }
}
