/*
 * js_fdlibm.h — TEST INFRASTRUCTURE ONLY (included by jsrt_oracle.c): Math.sin, Math.cos and Math.acos of
 * the reference's runtime, restated in C.  V8 (node 12) computes them with fdlibm 5.3
 * (v8/src/base/ieee754.cc: __kernel_sin, __kernel_cos, __ieee754_rem_pio2, __ieee754_acos); the C
 * library's sin / cos / acos differ from those in the last float64 bit on ~3 % of arguments.  Pinned bit
 * for bit to node's results on 3.3 M arguments (tests/golden/trig_v8.npz, tests/test_oracle_trig.py).
 * Arguments beyond 2^19 pi/2 (none on the render path) fall back to the C library.  Math.atan2 and Math.asin
 * (Vec.cartesianToSpherical, math.js:189-193, and the cylinder UV, geometry.js:479-487) likewise: fdlibm's
 * atan / __ieee754_atan2 / __ieee754_asin, pinned to node on 4 M argument pairs (tests/golden/uv_v8.npz);
 * the C library differs from them on 18 % / 6 % of unit-vector arguments.
 */
#ifndef JS_FDLIBM_H
#define JS_FDLIBM_H
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint32_t fd_hi(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)(u >> 32); }
static inline uint32_t fd_lo(double x) { uint64_t u; memcpy(&u, &x, 8); return (uint32_t)u; }
static inline double fd_words(uint32_t hi, uint32_t lo) { uint64_t u = ((uint64_t)hi << 32) | lo; double x; memcpy(&x, &u, 8); return x; }

static double fd_ksin(double x, double y, int iy) { /* __kernel_sin, |x| <= pi/4 */
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if ((fd_hi(x) & 0x7fffffffu) < 0x3e400000u && (int)x == 0) return x;
    const double z = x * x, v = z * x, r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

static double fd_kcos(double x, double y) { /* __kernel_cos, |x| <= pi/4 */
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const uint32_t ix = fd_hi(x) & 0x7fffffffu;
    if (ix < 0x3e400000u && (int)x == 0) return 1.0;
    const double z = x * x, r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - (z * r - x * y));
    const double qx = ix > 0x3fe90000u ? 0.28125 : fd_words(ix - 0x00200000u, 0u);
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

/* __ieee754_rem_pio2, small and medium paths (pi/4 < |x| <= 2^19 pi/2); 0 beyond */
static int fd_rem_pio2(double x, double *y, int *n) {
    static const uint32_t npio2_hw[32] = {
        0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C, 0x4025FDBB, 0x402921FB,
        0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C, 0x40346B9C, 0x4035FDBB, 0x40378FDB, 0x403921FB,
        0x403AB41B, 0x403C463A, 0x403DD85A, 0x403F6A7A, 0x40407E4C, 0x4041475C, 0x4042106C, 0x4042D97C,
        0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB, 0x4046C6CB, 0x40478FDB, 0x404858EB, 0x404921FB};
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const int32_t hx = (int32_t)fd_hi(x);
    const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
    if (ix < 0x4002d97cu) { /* |x| < 3pi/4 */
        double z;
        if (hx > 0) {
            z = x - pio2_1;
            if (ix != 0x3ff921fbu) { y[0] = z - pio2_1t; y[1] = (z - y[0]) - pio2_1t; }
            else { z -= pio2_2; y[0] = z - pio2_2t; y[1] = (z - y[0]) - pio2_2t; }
            *n = 1;
        } else {
            z = x + pio2_1;
            if (ix != 0x3ff921fbu) { y[0] = z + pio2_1t; y[1] = (z - y[0]) + pio2_1t; }
            else { z += pio2_2; y[0] = z + pio2_2t; y[1] = (z - y[0]) + pio2_2t; }
            *n = -1;
        }
        return 1;
    }
    if (ix > 0x413921fbu) return 0;
    double t = fabs(x);
    const int32_t nn = (int32_t)(t * invpio2 + 0.5);
    const double fn = (double)nn;
    double r = t - fn * pio2_1, w = fn * pio2_1t;
    if (nn < 32 && ix != npio2_hw[nn - 1]) {
        y[0] = r - w;
    } else {
        const int32_t j = (int32_t)(ix >> 20);
        y[0] = r - w;
        int32_t i = j - (int32_t)((fd_hi(y[0]) >> 20) & 0x7ff);
        if (i > 16) {
            t = r; w = fn * pio2_2; r = t - w; w = fn * pio2_2t - ((t - r) - w); y[0] = r - w;
            i = j - (int32_t)((fd_hi(y[0]) >> 20) & 0x7ff);
            if (i > 49) { t = r; w = fn * pio2_3; r = t - w; w = fn * pio2_3t - ((t - r) - w); y[0] = r - w; }
        }
    }
    y[1] = (r - y[0]) - w;
    if (hx < 0) { y[0] = -y[0]; y[1] = -y[1]; *n = -nn; } else *n = nn;
    return 1;
}

static double js_sin(double x) { /* ieee754::sin */
    const uint32_t ix = fd_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return fd_ksin(x, 0.0, 0);
    if (ix >= 0x7ff00000u) return x - x;
    double y[2]; int n;
    if (!fd_rem_pio2(x, y, &n)) return sin(x);
    switch (n & 3) {
    case 0: return fd_ksin(y[0], y[1], 1);
    case 1: return fd_kcos(y[0], y[1]);
    case 2: return -fd_ksin(y[0], y[1], 1);
    default: return -fd_kcos(y[0], y[1]);
    }
}

static double js_cos(double x) { /* ieee754::cos */
    const uint32_t ix = fd_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return fd_kcos(x, 0.0);
    if (ix >= 0x7ff00000u) return x - x;
    double y[2]; int n;
    if (!fd_rem_pio2(x, y, &n)) return cos(x);
    switch (n & 3) {
    case 0: return fd_kcos(y[0], y[1]);
    case 1: return -fd_ksin(y[0], y[1], 1);
    case 2: return -fd_kcos(y[0], y[1]);
    default: return fd_ksin(y[0], y[1], 1);
    }
}

static double js_acos(double x) { /* __ieee754_acos */
    const double pi = 3.14159265358979311600e+00, pio2_hi = 1.57079632679489655800e+00,
                 pio2_lo = 6.12323399573676603587e-17, pS0 = 1.66666666666666657415e-01,
                 pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05, qS1 = -2.40339491173441421878e+00,
                 qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const int32_t hx = (int32_t)fd_hi(x);
    const uint32_t ix = (uint32_t)hx & 0x7fffffffu;
    double z, p, q, r, s, w;
    if (ix >= 0x3ff00000u) {
        if (((ix - 0x3ff00000u) | fd_lo(x)) == 0) return hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000u) {
        if (ix <= 0x3c600000u) return pio2_hi + pio2_lo;
        z = x * x;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (hx < 0) {
        z = (1.0 + x) * 0.5;
        p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        s = sqrt(z);
        r = p / q;
        w = r * s - pio2_lo;
        return pi - 2.0 * (s + w);
    }
    z = (1.0 - x) * 0.5;
    s = sqrt(z);
    const double df = fd_words(fd_hi(s), 0u);
    const double c = (z - df * df) / (s + df);
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    w = r * s + c;
    return 2.0 * (df + w);
}
static double fd_atan(double x) { /* atan (s_atan.c) */
    static const double atanhi[] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static const double atanlo[] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17, 6.12323399573676603587e-17};
    static const double aT[] = {3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                                -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                                -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    double w, s1, s2, z;
    int32_t ix, hx, id;
    hx = (int32_t)fd_hi(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x44100000) {
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && (fd_lo(x) != 0))) return x + x;
        if (hx > 0) return atanhi[3] + atanlo[3];
        else return -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000) {
        if (ix < 0x3e200000) return x;
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    z = x * x;
    w = z * z;
    s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}
static double js_atan2(double y, double x) { /* __ieee754_atan2 (FreeBSD msun form, as V8) */
    const double tiny = 1.0e-300, zero = 0.0, pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
                 pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    double z;
    int32_t k, m, hx, hy, ix, iy;
    uint32_t lx, ly;
    hx = (int32_t)fd_hi(x); ix = hx & 0x7fffffff; lx = fd_lo(x);
    hy = (int32_t)fd_hi(y); iy = hy & 0x7fffffff; ly = fd_lo(y);
    if (((uint32_t)ix | ((lx | -lx) >> 31)) > 0x7ff00000u || ((uint32_t)iy | ((ly | -ly) >> 31)) > 0x7ff00000u) return x + y;
    if (((hx - 0x3ff00000) | (int32_t)lx) == 0) return fd_atan(y);
    m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | ly) == 0) {
        switch (m) {
        case 0: case 1: return y;
        case 2: return pi + tiny;
        case 3: return -pi - tiny;
        }
    }
    if ((ix | lx) == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0 * pi_o_4 + tiny;
            case 3: return -3.0 * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
            case 0: return zero;
            case 1: return -zero;
            case 2: return pi + tiny;
            case 3: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7ff00000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    k = (iy - ix) >> 20;
    if (k > 60) { z = pi_o_2 + 0.5 * pi_lo; m &= 1; }
    else if (hx < 0 && k < -60) z = 0.0;
    else z = fd_atan(fabs(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}
static double js_asin(double x) { /* __ieee754_asin */
    const double one = 1.0, huge = 1.0e300, pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
                 pio4_hi = 7.85398163397448278999e-01, pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04,
                 pS5 = 3.47933107596021167570e-05, qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    double t = 0, w, p, q, c, r, s;
    int32_t hx, ix;
    hx = (int32_t)fd_hi(x);
    ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (((ix - 0x3ff00000) | (int32_t)fd_lo(x)) == 0) return x * pio2_hi + x * pio2_lo;
        return (x - x) / (x - x);
    } else if (ix < 0x3fe00000) {
        if (ix < 0x3e400000) {
            if (huge + x > one) return x;
        } else {
            t = x * x;
        }
        p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
        q = one + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
        w = p / q;
        return x + x * w;
    }
    w = one - fabs(x);
    t = w * 0.5;
    p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    q = one + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    s = sqrt(t);
    if (ix >= 0x3FEF3333) {
        w = p / q;
        t = pio2_hi - (2.0 * (s + s * w) - pio2_lo);
    } else {
        w = fd_words(fd_hi(s), 0);
        c = (t - w * w) / (s + w);
        r = p / q;
        p = 2.0 * s * r - (pio2_lo - 2.0 * c);
        q = pio4_hi - 2.0 * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

#endif
