// js_number.h — the reference's Math.fmod rounding (math.js:27: Number(x.toPrecision(8))), on the
// host and the device.  SDFInfiniteRepetitionTransformer (sdf.js:471-473) and the checkerboard
// colour (materials.js:72-75) call it per evaluation, so it sits on the SDF march's inner loop.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace jsrt {

// Number(v.toPrecision(8)) — ECMA-262 toPrecision (ties -> larger n) then correctly rounded parse.
// Exact for 1e-12 <= |v| < 2^64 (128-bit products, no 128-bit division); outside that window the
// 8-digit rounding is applied in float64 (documented in DESIGN.md; no reference scene reaches it).
__host__ __device__ inline double to_precision8_exact(double v) {
    if (!__builtin_isfinite(v)) return v;
    if (v == 0.0) return 0.0;
    const bool neg = v < 0;
    const double x = fabs(v);
    int ex;
    const double f = frexp(x, &ex);
    const uint64_t M = (uint64_t)ldexp(f, 53);
    const int E = ex - 53;
    int e10 = (int)floor(log10(x));
    uint64_t n = 0;
    const uint64_t P10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                              100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull,
                              10000000000000ull, 100000000000000ull, 1000000000000000ull, 10000000000000000ull,
                              100000000000000000ull, 1000000000000000000ull, 10000000000000000000ull};
    bool ok = false;
    for (int it = 0; it < 4; ++it) {
        const int k = 7 - e10;
        uint64_t q;
        bool up;
        if (k >= 0) {
            if (k > 19 || E >= 0) break;
            const unsigned __int128 num = (unsigned __int128)M * P10[k];
            const int s = -E;
            if (s >= 127) break;
            const unsigned __int128 qq = num >> s;
            const unsigned __int128 rem = num - (qq << s);
            if (qq >= (unsigned __int128)1000000000ull) { e10 += 1; continue; }
            q = (uint64_t)qq;
            up = (rem << 1) >= ((unsigned __int128)1 << s);
        } else {
            const int m = -k;
            if (m > 19 || ex > 64) break;
            uint64_t num, den;
            if (E >= 0) { num = M << E; den = P10[m]; }
            else {
                num = M;
                if (-E > 63 || P10[m] > (~0ull >> -E)) break;
                den = P10[m] << -E;
            }
            q = num / den;
            const uint64_t rem = num - q * den;
            up = rem >= den - rem;  // 2*rem >= den without overflow
        }
        if (q < 10000000ull) { e10 -= 1; continue; }
        if (q >= 100000000ull) { e10 += 1; continue; }
        n = q + (up ? 1 : 0);
        if (n == 100000000ull) { n = 10000000ull; e10 += 1; }
        ok = true;
        break;
    }
    double r;
    if (!ok) {  // outside the exact window
        // 10^(7-e10) in two factors: a single one overflows for denormal x (5e-324 -> 10^331)
        const int k = 7 - e10, k1 = k / 2;
        const double s1 = pow(10.0, (double)k1), s2 = pow(10.0, (double)(k - k1));
        r = floor(x * s1 * s2 + 0.5) / s2 / s1;
    } else {
        const int k2 = e10 - 7;
        const double P10D[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        if (k2 >= 0 && k2 <= 22) r = (double)n * P10D[k2];
        else if (k2 < 0 && -k2 <= 22) r = (double)n / P10D[-k2];
        else r = (double)n * pow(10.0, (double)k2);
    }
    return neg ? -r : r;
}

// 10^k exactly for 0 <= k <= 22 (5^22 < 2^53: every partial product of the binary powers is itself an
// exact power of ten), from immediates: a per-lane table lookup would be a memory load on the SDF
// march's dependent chain.
__host__ __device__ inline double pow10_exact(int k) {
    double r = (k & 1) ? 1e1 : 1.0;
    r *= (k & 2) ? 1e2 : 1.0;
    r *= (k & 4) ? 1e4 : 1.0;
    r *= (k & 8) ? 1e8 : 1.0;
    r *= (k & 16) ? 1e16 : 1.0;
    return r;
}

// 10^k, 0 <= k <= 22, for to_precision8_sl on the device: a per-lane load of a constant table (an
// L1 hit) costs less than forming the power from immediates (five dependent multiplies behind selects): SDF_Menger
// 203.6 -> 206.3 M/s (profiles/r06_s15_tp8_menger.txt)
static __constant__ double p10_table[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                            1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Fast path for 1e-37 <= |v| < 1e8 (every value the reference scenes produce).  The product
// x * 10^k is carried as p + err: for k <= 22 one fma gives the exact rounding error; for k in
// 23..44 it is x * 1e22 * 10^(k-22) in double-double (err then carries ~2^-100 relative error,
// which decides a rounding only for a product within that distance of a half-integer; an exact
// tie needs x * 10^k to be a multiple of 1/2, impossible for x < 1e-15).  The 8-digit integer n
// (ties -> larger n, ECMA-262 toPrecision) follows without 128-bit arithmetic:
//   * p and r = floor(p) are multiples of ulp(p) <= 2^-26 and p - r is exact, so err only
//     matters when p - r == 0.5 (err > 0 rounds up, err < 0 down, 0 is a tie, rounded up);
//   * the decade test x * 10^k < 1e7 is p < 1e7, or p == 1e7 with err < 0 (likewise for 1e8).
// The parse n * 10^(e10-7) is one correctly rounded IEEE multiply or divide by an exact power of
// ten for |e10 - 7| <= 22, else a division by 1e22 * 10^j with a remainder correction.  The
// k <= 22 range is bit-identical to to_precision8_exact (tests/test_js_number.py).
__host__ __device__ inline double to_precision8(double v) {
    if (!__builtin_isfinite(v)) return v;
    if (v == 0.0) return 0.0;
    const double x = fabs(v);
    int ex;
    (void)frexp(x, &ex);  // x in [2^(ex-1), 2^ex)
    int e10 = (int)floor((double)(ex - 1) * 0.30102999566398120);  // floor(log10 x) or one less
    for (int it = 0; it < 3; ++it) {
        const int k = 7 - e10;
        if (k > 44 && it == 0) { e10 += 1; continue; }  // the estimate may be one decade low
        if (k < 0 || k > 44) break;
        double p, err;
        if (k <= 22) {
            const double P = pow10_exact(k);
            p = x * P;
            err = fma(x, P, -p);
        } else {
            const double B = pow10_exact(k - 22);
            const double p1 = x * 1e22, e1 = fma(x, 1e22, -p1);
            p = p1 * B;
            err = fma(p1, B, -p) + e1 * B;
        }
        if (p < 1e7 || (p == 1e7 && err < 0)) { e10 -= 1; continue; }
        if (p > 1e8 || (p == 1e8 && err >= 0)) { e10 += 1; continue; }
        const double r = floor(p), fr = p - r;
        double n = r + ((fr > 0.5 || (fr == 0.5 && err >= 0)) ? 1.0 : 0.0);
        int e = e10;
        if (n == 1e8) { n = 1e7; e += 1; }
        const int k2 = e - 7;
        double res;
        if (k2 >= 0) {
            res = n * pow10_exact(k2);  // k2 <= 0 here: e10 <= 7
#ifdef JSRT_RECIP_PARSE
        } else if (-k2 >= 7 && -k2 <= 9) {  // the SDF repetition range: RN(n / 10^m) as RN(n * RN(10^-m)) plus
            // one fma-exact remainder correction, bit-identical to the division for every 8-digit n and
            // m in 1..22 (tests/test_js_number.py::test_reciprocal_parse_exhaustive)
            const double R = -k2 == 7 ? 1e-7 : (-k2 == 8 ? 1e-8 : 1e-9);
            const double P = -k2 == 7 ? 1e7 : (-k2 == 8 ? 1e8 : 1e9);
            const double q0 = n * R;
            res = fma(fma(-q0, P, n), R, q0);
#endif
        } else if (-k2 <= 22) {
            res = n / pow10_exact(-k2);
        } else {  // n / (1e22 * B): quotient and exact remainders, one final rounding
            const double B = pow10_exact(-k2 - 22);
            const double q1 = n / 1e22, r1 = fma(-q1, 1e22, n);
            const double q = q1 / B, r = fma(-q, B, q1);
            res = q + (r + r1 / 1e22) / B;
        }
        return v < 0 ? -res : res;
    }
    return to_precision8_exact(v);
}

// to_precision8 without branches for 1e-15 <= |v| < 1e8 (the SDF repetition range and every checkerboard
// value), the same IEEE operations as the fast path above: the decade estimate e10 from the binary exponent
// is floor(log10 |v|) or one less, so the scaled value of the estimate and of the decade above are both
// formed and the one in [1e7, 1e8] kept (the fast path's loop, unrolled); the parse is one IEEE division by
// the kept power of ten (a division by 1 is exact), and that power is the only one formed per call (round 6:
// the parse's own two powers and the second scaled power cost SDF_Menger 16 %, profiles/r06_s14_tp8_menger.txt).
// Per lane this is straight-line code: no divergent branches, whose exec-mask bookkeeping made the SDF march
// SALU-heavy.  Bit-identical to to_precision8 (tests/test_js_number.py).
__host__ __device__ inline double to_precision8_sl(double v) {
    const double x = fabs(v);
    int ex;
    (void)frexp(x, &ex);
    const int e10 = (int)floor((double)(ex - 1) * 0.30102999566398120);
    if (!(x >= 1e-15 && x < 1e8) || e10 < -15) return to_precision8(v);  // (also 0, NaN, +-inf)
    const int kA = 7 - e10;  // 0..22 for e10 in [-15, 7]
    // 10^(kA - 1) and 10^kA = 10 * 10^(kA - 1), both exact (5^22 < 2^53)
#ifdef __HIP_DEVICE_COMPILE__
    const double PB = p10_table[kA > 0 ? kA - 1 : 0], PA = kA > 0 ? PB * 10.0 : 1.0;
#else
    const double PB = pow10_exact(kA > 0 ? kA - 1 : 0), PA = kA > 0 ? PB * 10.0 : 1.0;
#endif
    const double pA = x * PA, errA = fma(x, PA, -pA);
    // the estimate was a decade low when the scaled value reaches 1e8 (the fast path's second iteration)
    const bool hi = kA > 0 && (pA > 1e8 || (pA == 1e8 && errA >= 0));
    const double pB = x * PB, errB = fma(x, PB, -pB);
    const double p = hi ? pB : pA, err = hi ? errB : errA;
    const double r = floor(p), fr = p - r;
    const double n = r + ((fr > 0.5 || (fr == 0.5 && err >= 0)) ? 1.0 : 0.0);
    // the parse n * 10^(e - 7), e <= 7: one IEEE division by 10^(7 - e), the power already formed (PA or PB).  A
    // carry (n == 1e8, the 8 digits 1e7 of the next decade) keeps n = 1e8 and the divisor: 1e8 / 10^m and
    // 1e7 / 10^(m - 1) (or 1e7 * 10 at m = 0) are correctly rounded values of the same real number.
    const double res = n / (hi ? PB : PA);
    return v < 0 ? -res : res;
}

__host__ __device__ inline double js_fmod(double a, double b) {  // math.js:27
    return to_precision8(a - (floor(a / b) * b));
}

}  // namespace jsrt
