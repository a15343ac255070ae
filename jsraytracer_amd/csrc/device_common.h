// device_common.h — device-side building blocks shared by the render kernels: the reference's
// scalar semantics (Math.max/min/pow/round, toPrecision(8) fmod), the keyed RNG, f32-stored Vec
// arithmetic, ray transforms, geometry intersections, the SDF program VM, world casts with
// conservative culling, material colours and light-sample / scatter math.
//
// Numerics follow the reference's model: Vec components are float32 after every
// Vec op; scalars are float64; each binary op is one IEEE op (built with -ffp-contract=off).
// f32 (+,-,*,/) of two f32 operands is done natively in f32 (bit-identical to f64-then-round);
// f32 * f64 scalar is done in f64 then rounded.  Random numbers come from the keyed,
// ray-tree-addressed generator, identical to oracle/refharness/keyed_rng.js.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_scene.h"
#include "fdlibm.h"
#include "js_number.h"

// building blocks also compiled for the host (tests/native: filter-vs-exact checks on the CPU)
#define JSRT_HD __host__ __device__ __forceinline__

namespace jsrt {

#define JS_PI 3.141592653589793
#define DINF __builtin_inf()

// --------------------------------------------------------------------------------------------
// JS scalar semantics
JSRT_HD bool is_nan(double x) { return x != x; }
// Math.max / Math.min as compares and selects (no branches): NaN if either operand is NaN (a NaN `a`
// is returned as is, a NaN `b` is the select's fall-through); equal operands -- +-0 pairs included --
// give the AND (max) / OR (min) of their bit patterns: +0 unless both are -0 for max, -0 if either is
// for min, and the common value for equal non-zero operands (identical bits).
JSRT_HD double js_max(double a, double b) {  // Math.max
    double r = a > b ? a : b;
    if (a == b) r = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, a) & __builtin_bit_cast(uint64_t, b));
    return a != a ? a : r;
}
JSRT_HD double js_min(double a, double b) {  // Math.min
    double r = a < b ? a : b;
    if (a == b) r = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, a) | __builtin_bit_cast(uint64_t, b));
    return a != a ? a : r;
}
// the same on f32 values (exact: the result is an operand, +-0 or NaN)
JSRT_HD float js_maxf(float a, float b) {
    float r = a > b ? a : b;
    if (a == b) r = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, a) & __builtin_bit_cast(uint32_t, b));
    return a != a ? a : r;
}
JSRT_HD float js_max0f(float x) { return (x > 0.0f || x != x) ? x : 0.0f; }  // Math.max(x, 0)
JSRT_HD float js_min0f(float x) { return x > 0.0f ? 0.0f : x; }              // Math.min(x, 0)
JSRT_HD double js_sign(double x) {
    if (is_nan(x) || x == 0.0) return x;
    return x > 0 ? 1.0 : -1.0;
}
// (ah + al) * (bh + bl) in double-double (Dekker / fma two-product): relative error ~2^-104
JSRT_HD void dd_mul(double ah, double al, double bh, double bl, double &rh, double &rl) {
    const double p = ah * bh;
    const double e = fma(ah, bh, -p) + (ah * bl + al * bh);
    rh = p + e;
    rl = e - (rh - p);
}
// x^n, integer 1 <= n <= 64, 0 <= x <= 2, by binary powering in double-double and one final rounding:
// the correctly rounded power except for a value within ~2^-100 relative of a rounding boundary (libm's
// f64 pow -- V8's fdlibm, glibc, OCML -- is itself only within ~1 ulp there).  A third of the VALU
// of OCML's general pow for the Phong exponents the reference scenes use (10, 100).
JSRT_HD double pow_int_dd(double x, int n) {
    double bh = x, bl = 0.0, rh = 1.0, rl = 0.0;
    bool first = true;  // the first factor is copied, not multiplied into (1, 0): dd_mul's outputs are
                        // normalised, so 1 x (bh, bl) would return (bh, bl) unchanged
    for (;;) {
        if (n & 1) {
            if (first) { rh = bh; rl = bl; first = false; }
            else dd_mul(rh, rl, bh, bl, rh, rl);
        }
        n >>= 1;
        if (!n) break;
        dd_mul(bh, bl, bh, bl, bh, bl);
    }
    return rh + rl;
}
// Math.pow.  The fast path takes x in [+0, 2] (never -0: pow_int_dd(-0, odd n) would return +0 where
// Math.pow gives -0) and an integral y in [1, 64]; its result is the correctly rounded power, which V8's
// fdlibm pow is only within an ulp of, so parity there is pinned by the goldens, not by construction.
__device__ __forceinline__ double js_pow(double x, double y) {
    if (is_nan(y)) return __builtin_nan("");
    if (y == 0.0) return 1.0;
    if ((x == 1.0 || x == -1.0) && __builtin_isinf(y)) return __builtin_nan("");
#ifndef JSRT_LIBM_POW
    if ((x > 0.0 || (x == 0.0 && !__builtin_signbit(x))) && x <= 2.0 && y >= 1.0 && y <= 64.0 && y == floor(y))
        return pow_int_dd(x, (int)y);
#endif
    return pow(x, y);
}
__device__ __forceinline__ double js_round(double x) {  // Math.round (half toward +inf)
    if (!__builtin_isfinite(x) || x == 0.0) return x;
    double r = floor(x);
    if (x - r >= 0.5) r += 1.0;
    return r;
}
JSRT_HD float or0(float x) { return (x != x || x == 0.0f) ? 0.0f : x; }  // `x || 0`

// --------------------------------------------------------------------------------------------
// keyed RNG (oracle/refharness/keyed_rng.js)
__device__ __forceinline__ uint32_t mix32(uint32_t h, uint32_t v) {
    h = (h ^ v) * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    return h;
}
// the draw of hash h = mix(mix(pixkey, node), call)
__device__ __forceinline__ double uniform_of(uint32_t h) {
    const uint32_t hi = mix32(h, 0xA5A5A5A5u) >> 5;  // 27 bits
    const uint32_t lo = mix32(h, 0x5A5A5A5Au) >> 6;  // 26 bits
    // (hi * 2^26 + lo) * 2^-53 with every step exact in f64 (hi * 2^-27 and lo * 2^-53 are exact, their sum
    // has at most 53 significant bits): the same double as the reference generator's, without the u64
    // multiply and the u64 -> f64 conversion sequence
    return fma((double)hi, 1.0 / 134217728.0, (double)lo * (1.0 / 9007199254740992.0));
}
// pixkey = mix(mix(seed, pixel), sample), hoisted per sample
__device__ __forceinline__ double keyed_uniform(uint32_t pixkey, uint32_t node, uint32_t call) {
    return uniform_of(mix32(mix32(pixkey, node), call));
}
struct Rng {
    uint32_t key, node, calls;
    __device__ __forceinline__ double next() { return keyed_uniform(key, node, calls++); }
};
// the same stream from the frame hash h0 = mix(pixkey, node), computed once per ray-tree node (the shadow
// hand-off carries it in place of the key and the node address)
struct RngH {
    uint32_t h0, calls;
    __device__ __forceinline__ double next() { return uniform_of(mix32(h0, calls++)); }
};

// --------------------------------------------------------------------------------------------
// 3-component Vec with an implicit w (1 for points, 0 for directions; colours are 3-vectors)
struct F3 {
    float x, y, z;
};
JSRT_HD F3 f3(float x, float y, float z) { return F3{x, y, z}; }
JSRT_HD F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
JSRT_HD F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
JSRT_HD F3 mul(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
JSRT_HD F3 scale(F3 a, double s) {  // Vec.times(scalar): f32(x * s) in f64
    return f3((float)((double)a.x * s), (float)((double)a.y * s), (float)((double)a.z * s));
}
JSRT_HD F3 neg(F3 a) { return f3(-a.x, -a.y, -a.z); }  // times(-1) is exact
// Vec.dot (math.js:252-260) of two f32 vectors: ((x x' + y y') + z z') in f64.  A product of two f32 values is
// exact in f64 (24 + 24 <= 53 significant bits; no overflow or underflow to a subnormal), so the fused form
// fma(z, z', fma(x, x', y y')) rounds exactly the sums the reference rounds, bit for bit (signed zeros and
// NaN / Infinity included): three f64 operations instead of five.
JSRT_HD double dot3(F3 a, F3 b) {
    return fma((double)a.z, (double)b.z, fma((double)a.x, (double)b.x, (double)a.y * (double)b.y));
}
// normalized() of a Vec whose 4th component is (+/-)0 or absent: the 4th term only adds a zero
JSRT_HD F3 normalized(F3 a) {
    const double n = sqrt(dot3(a, a));
    return (n > 0.00001) ? scale(a, 1 / n) : a;
}
JSRT_HD double average3(F3 a) {  // Vec.average (math.js:261-266)
    return ((((0.0 + (double)a.x) + (double)a.y) + (double)a.z)) / 3;
}

// Mat(3x4 rows, implicit row 3 = 0,0,0,1) * Vec (math.js:392-397): f64 dot in order, f32 store.
template <class T>
JSRT_HD F3 xf_point(const T *m, F3 o) {  // w = 1 (T: double in any address space)
    return f3((float)((((double)o.x * m[0] + (double)o.y * m[1]) + (double)o.z * m[2]) + m[3]),
              (float)((((double)o.x * m[4] + (double)o.y * m[5]) + (double)o.z * m[6]) + m[7]),
              (float)((((double)o.x * m[8] + (double)o.y * m[9]) + (double)o.z * m[10]) + m[11]));
}
template <class T>
JSRT_HD F3 xf_dir(const T *m, F3 d) {  // w = 0: the 4th term only adds a zero
    return f3((float)(((double)d.x * m[0] + (double)d.y * m[1]) + (double)d.z * m[2]),
              (float)(((double)d.x * m[4] + (double)d.y * m[5]) + (double)d.z * m[6]),
              (float)(((double)d.x * m[8] + (double)d.y * m[9]) + (double)d.z * m[10]));
}
// Ray.getPoint (math.js:297-299): origin.plus(direction.times(t))
JSRT_HD F3 ray_point(F3 o, F3 d, double t) {
    return f3(o.x + (float)((double)d.x * t), o.y + (float)((double)d.y * t), o.z + (float)((double)d.z * t));
}
// Math.sin and Math.cos of one argument: V8's own algorithm (fdlibm.h, pinned bit for bit to node's results
// on 3.3 M arguments, tests/test_fdlibm.py), one argument reduction for the pair.  (OCML's sin / cos / acos
// differ from V8 in the last bit on ~3 % of arguments, as glibc's do.)
__device__ __forceinline__ void sin_cos(double x, double &s, double &c) { fdlibm::sin_cos(x, s, c); }
// Vec.spherePick() (math.js:180-185): theta = 2 pi r0, phi = acos(2 r1 - 1), the point (cos theta sin phi,
// cos phi, sin theta sin phi) as f32, with V8's sin / cos / acos (fdlibm.h).  Only the three f32 roundings
// reach the image, so estimates are evaluated first -- OCML's sincos of theta, and sin / cos of phi from
// sin_cos_of_acos (no acos, no second sincos) -- and kept when every value within SPHERE_PICK_EPS = 2^-44 of
// each product rounds to the same f32: tests/test_gpu_trig.py bounds |OCML - V8| by 2^-50 on the spherePick
// arguments of node's fixture and tests/test_sphere_pick_identity.py the phi estimates by 2^-50, so a product
// is within 3 * 2^-50 + 2^-52 of V8's, 19x inside the margin, and a kept result is V8's.  The rest (|value|
// below ~2^-20, or within 2^-44 of an f32 rounding boundary: about one pick in 10^5) are recomputed with
// fdlibm, out of line.
constexpr double SPHERE_PICK_EPS = 0x1p-44;
// Whether every value within SPHERE_PICK_EPS of d rounds to d's f32, on the bits of d (|d| <= 2; integer
// operations, no f64 temporaries; tests/test_box_any.py::test_f32_stable_bits): the f32
// rounding of d is decided by its low 29 fraction bits against the midpoint 2^28, and 2^-44 is 2^(8 - e)
// units of d's last place for d in [2^e, 2^(e+1)).  Stable iff the distance to the midpoint exceeds that
// (|d| < 2^-20: never, the margin reaches half an f32 unit).
JSRT_HD bool f32_stable_bits(double d) {
    const uint64_t b = __builtin_bit_cast(uint64_t, d);
    const int e = (int)((uint32_t)(b >> 52) & 0x7FFu) - 1023;
    const int sh = 8 - e;
    const uint32_t m = (uint32_t)b & 0x1FFFFFFFu;
    const uint32_t dist = m > 0x10000000u ? m - 0x10000000u : 0x10000000u - m;
    return sh <= 28 && dist > (1u << (sh < 0 ? 0 : sh));
}
struct SinCos2 {
    double st, ct, sp, cp;
};
// sin(phi) and cos(phi) of phi = acos(a) for the filter (not V8's values): sqrt((1 - a)(1 + a)) and a.  Both
// factors of 1 - a^2 are exact where it matters (Sterbenz: the small one near a = +-1), so the root is within
// ~2^-52 relative of the real sin(acos(a)), and V8's sin(acos(a)) / cos(acos(a)) are within ~2^-51 of the real
// values (acos's last-bit error carried through slopes <= 1, plus their own rounding): the approximation is
// within 2^-50 of V8's, as OCML's acos + sincos were (tests/test_sphere_pick_identity.py checks it against the
// oracle's fdlibm on 4 M arguments and the poles), so the 2^-44 stability margin still decides exactly.  An
// acos and a sincos less per pick.
__device__ __forceinline__ void sin_cos_of_acos(double a, double &sin_phi, double &cos_phi) {
    sin_phi = sqrt((1.0 - a) * (1.0 + a));
    cos_phi = a;
}
__device__ __forceinline__ SinCos2 sphere_pick_exact(double theta, double a) {
    SinCos2 r;
    fdlibm::sin_cos(theta, r.st, r.ct);
    fdlibm::sin_cos(fdlibm::acos(a), r.sp, r.cp);
    return r;
}
template <class R>
__device__ __forceinline__ F3 sphere_pick(R &rng) {
    const double theta = 2.0 * JS_PI * rng.next();
    const double a = 2.0 * rng.next() - 1.0;
    double sin_t, cos_t, sin_phi, cos_phi;
#ifdef JSRT_EXACT_TRIG  // A/B: fdlibm only
    const bool fast = false;
#else
    sincos(theta, &sin_t, &cos_t);
    sin_cos_of_acos(a, sin_phi, cos_phi);
    const bool fast = f32_stable_bits(cos_t * sin_phi) && f32_stable_bits(cos_phi) && f32_stable_bits(sin_t * sin_phi);
#endif
    if (__builtin_expect(!fast, 0)) {  // out of line: the hot path keeps OCML's register footprint
        const SinCos2 r = sphere_pick_exact(theta, a);
        sin_t = r.st, cos_t = r.ct, sin_phi = r.sp, cos_phi = r.cp;
    }
    return f3((float)(cos_t * sin_phi), or0((float)cos_phi), or0((float)(sin_t * sin_phi)));
}
// spherePick for a caller that finishes the unstable picks itself (k_shade, at its tail, where the registers
// are free: the fallback inline in the scatter cost k_shade ~50 spilled VGPRs and 25 % of its time):
// OCML's values, with `unstable` set when a product's f32 rounding is not decided within SPHERE_PICK_EPS;
// sphere_pick_v8 then gives the reference's point from the same two draws.
template <class R>
__device__ __forceinline__ F3 sphere_pick_fast(R &rng, bool &unstable) {
    const double theta = 2.0 * JS_PI * rng.next();
    const double a = 2.0 * rng.next() - 1.0;
    double sin_t, cos_t, sin_phi, cos_phi;
    sincos(theta, &sin_t, &cos_t);
    sin_cos_of_acos(a, sin_phi, cos_phi);
    const double px = cos_t * sin_phi, pz = sin_t * sin_phi;
    unstable = !(f32_stable_bits(px) && f32_stable_bits(cos_phi) && f32_stable_bits(pz));  // (forced: JSRT_FORCE_EXACT_PICK)
    return f3((float)px, or0((float)cos_phi), or0((float)pz));
}
template <class R>
__device__ __forceinline__ F3 sphere_pick_v8(R &rng) {
    const double theta = 2.0 * JS_PI * rng.next();
    const double a = 2.0 * rng.next() - 1.0;
    double sin_t, cos_t, sin_phi, cos_phi;
    fdlibm::sin_cos(theta, sin_t, cos_t);
    fdlibm::sin_cos(fdlibm::acos(a), sin_phi, cos_phi);
    return f3((float)(cos_t * sin_phi), or0((float)cos_phi), or0((float)(sin_t * sin_phi)));
}
// Vec.cartesianToSpherical (math.js:189-193)
__device__ __forceinline__ void cart_to_sph(F3 n, float &u, float &v) {
    u = (float)(0.5 + fdlibm::atan2((double)n.z, (double)n.x) / (2 * JS_PI));  // V8's atan2 / asin (fdlibm.h)
    v = (float)(0.5 - fdlibm::asin((double)n.y) / JS_PI);
}

// --------------------------------------------------------------------------------------------
// geometry (geometry.js), local space
JSRT_HD bool aabb_slab(float cx, float cy, float cz, float hx, float hy, float hz, F3 o, F3 d,
                                          double minD, double maxD, double &tmin, double &tmax) {
    // AABB.get_intersects (geometry.js:189-209)
    double t_min = -DINF, t_max = DINF;
    const float p[3] = {cx - o.x, cy - o.y, cz - o.z};
    const float h[3] = {hx, hy, hz};
    const float dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double di = (double)dd[i];
        if (fabs(di) > 0.0000001) {
            double t1 = ((double)p[i] + (double)h[i]) / di, t2 = ((double)p[i] - (double)h[i]) / di;
            if (t1 > t2) { const double tmp = t1; t1 = t2; t2 = tmp; }
            if (t1 > t_min) t_min = t1;
            if (t2 < t_max) t_max = t2;
            if (t_min > t_max || t_max < minD || t_min > maxD) return false;
        } else if (fabs((double)p[i]) > (double)h[i])
            return false;
    }
    tmin = t_min;
    tmax = t_max;
    return true;
}

// The BVH entry test (aggregates.js:208-209: AABB.get_intersects, then ts.min <= maxD, ts.max >= minD,
// ts.min <= ret.distance) evaluated in f32 with an error bound; only a decision too close to call runs
// the exact f64 slab (aabb_slab: six correctly rounded divisions).
//
// Exactness: the reference's result is a boolean of comparisons between the quotients (p_i +- h_i) /
// d_i (f64, p = center - origin in f32 as Vec.minus stores it) and the doubles minD, lim =
// min(maxD, best).  Swaps, running max / min and the per-axis early outs reduce to: enter iff every
// skipped axis (|d_i| <= 1e-7) has |p_i| <= h_i, and max_i lo_i <= min_i hi_i, min_i hi_i >= minD,
// max_i lo_i <= lim.  Here each quotient is (p_i +- h_i) * (1 / d_i) in f32: within 3 f32 roundings
// (3u, u = 2^-24) of the real quotient, which the f64 quotient is within 2^-53 of.  A comparison is
// decided only when its operands are apart by more than EPS = 2^-21 (> 8u) of their magnitudes
// (+ 1e-30 absolute, for underflow); then it has the exact outcome.  Overflow / NaN is "too close".
struct BoxRay {       // per ray: the f32 reciprocals and the reference's epsilon test per axis
    float inv[3];
    uint32_t skip;    // bit i: |d_i| <= 1e-7 (geometry.js:194, compared in f64)
};
JSRT_HD BoxRay box_ray(F3 d) {
    BoxRay r;
    const float dd[3] = {d.x, d.y, d.z};
    r.skip = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const bool sk = !(fabs((double)dd[i]) > 0.0000001);
        r.skip |= (sk ? 1u : 0u) << i;
        r.inv[i] = sk ? 0.0f : 1.0f / dd[i];
    }
    return r;
}
// 1: enter, 0: skip, -1: too close to call (run the exact test)
__device__ __forceinline__ int box_enter_f32(float cx, float cy, float cz, float hx, float hy, float hz, F3 o,
                                             const BoxRay &r, float fmin_d, float flim) {
    constexpr float EPS = 4.76837158203125e-7f, TINY = 1e-30f;  // 2^-21
    const float c[3] = {cx, cy, cz}, h[3] = {hx, hy, hz}, oo[3] = {o.x, o.y, o.z};
    float tmin = -__builtin_inff(), tmax = __builtin_inff();
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float p = c[i] - oo[i];
        if ((r.skip >> i) & 1u) {
            out = out || fabsf(p) > h[i];  // exact: both f32
        } else {
            const float a = (p + h[i]) * r.inv[i], b = (p - h[i]) * r.inv[i];
            tmin = fmaxf(tmin, fminf(a, b));
            tmax = fminf(tmax, fmaxf(a, b));
        }
    }
    if (out) return 0;
    if (r.skip == 7u) return 1;  // no slab: (-inf, inf) always enters
    // finite unless an axis overflowed (a skipped axis never sets them, a used one always does)
    if (!__builtin_isfinite(tmin) || !__builtin_isfinite(tmax)) return -1;
    const float en = EPS * fabsf(tmin) + TINY, ex = EPS * fabsf(tmax) + TINY;
    const float em = EPS * fabsf(fmin_d) + TINY;
    // c1: tmin <= tmax, c2: tmax >= minD, c3: tmin <= lim (lim may be +inf: always true)
    if (tmin - en > tmax + ex || tmax + ex < fmin_d - em) return 0;
    const bool c3_true = !__builtin_isfinite(flim) ? flim > 0 : tmin + en < flim - (EPS * fabsf(flim) + TINY);
    const bool c3_false = __builtin_isfinite(flim) ? tmin - en > flim + (EPS * fabsf(flim) + TINY) : flim < 0;
    if (c3_false) return 0;
    if (tmin + en < tmax - ex && tmax - ex > fmin_d + em && c3_true) return 1;
    return -1;
}

// Any-hit acceptance of an AABB geometry in a shadow cast (AABB.intersect, geometry.js:173-179, then
// World.cast's minD < t < maxD; a shadow cast stops at its first accepted hit, so `best` is +inf on every
// lane that still casts), decided in f32 with box_enter_f32's error bound: 1 = accepted (t_out = the f32
// estimate of the distance, inside (minD, maxD) by the margin), 0 = not accepted, -1 = too close to call
// (the caller runs the exact aabb_intersect).  The exact outcome: the slab passes (box_enter_f32's
// conditions with lim = maxD) and t = tmin >= minD ? tmin : tmax lies in (minD, maxD), i.e.
//   minD < tmin < maxD and tmin <= tmax,  or  tmin < minD < tmax < maxD
// (tmin == minD gives t = minD: rejected, and too close to call here).  The six correctly rounded f64
// divisions of the exact slab run only for a decision within 2^-21 of a boundary.
template <class T>  // T: float in any address space
JSRT_HD int box_any_f32(const T *c, const T *h, F3 o, const BoxRay &r, double minD, double maxD, double &t_out) {
    constexpr float EPS = 4.76837158203125e-7f, TINY = 1e-30f;  // 2^-21
    const float oo[3] = {o.x, o.y, o.z};
    float tmin = -__builtin_inff(), tmax = __builtin_inff();
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float p = c[i] - oo[i];
        if ((r.skip >> i) & 1u) {
            out = out || fabsf(p) > h[i];  // exact: both f32
        } else {
            const float a = (p + h[i]) * r.inv[i], b = (p - h[i]) * r.inv[i];
            tmin = fmaxf(tmin, fminf(a, b));
            tmax = fminf(tmax, fmaxf(a, b));
        }
    }
    if (out) return 0;
    if (!__builtin_isfinite(tmin) || !__builtin_isfinite(tmax)) return -1;  // (also every axis skipped)
    const float f0 = (float)minD, f1 = (float)maxD;
    if (!__builtin_isfinite(f0)) return -1;
    const bool inf1 = !__builtin_isfinite(f1) && f1 > 0;  // maxD = +inf: every finite t is below it
    const float en = EPS * fabsf(tmin) + TINY, ex = EPS * fabsf(tmax) + TINY;
    const float e0 = EPS * fabsf(f0) + TINY, e1 = inf1 ? 0.0f : EPS * fabsf(f1) + TINY;
    if (tmin - en > f0 + e0) {  // tmin > minD: t = tmin
        const bool lt1 = inf1 || tmin + en < f1 - e1, gt1 = !inf1 && tmin - en > f1 + e1;
        if (gt1 || tmin - en > tmax + ex) return 0;
        if (lt1 && tmin + en < tmax - ex) {
            t_out = tmin;
            return 1;
        }
        return -1;
    }
    if (tmin + en < f0 - e0) {  // tmin < minD: t = tmax
        const bool lt1 = inf1 || tmax + ex < f1 - e1, gt1 = !inf1 && tmax - ex > f1 + e1;
        if (tmax + ex < f0 - e0 || gt1) return 0;
        if (tmax - ex > f0 + e0 && lt1) {
            t_out = tmax;
            return 1;
        }
        return -1;
    }
    return -1;
}

template <class T>
JSRT_HD double aabb_intersect(const T *c, const T *h, F3 o, F3 d, double minD, double maxD) {  // geometry.js:173-179
    double tmin, tmax;
    if (aabb_slab(c[0], c[1], c[2], h[0], h[1], h[2], o, d, minD, maxD, tmin, tmax)) return (tmin >= minD) ? tmin : tmax;
    return -(double)__builtin_inf();
}

// Closest-hit form of the AABB test (World.cast's closest hit, world.js:7-15: a distance is kept only when
// minD < t < lim, lim = min(maxD, the closest hit so far)), decided in f32 as box_any_f32 with maxD := lim:
// 0 = not accepted (t_out untouched; the exact test's distance would be rejected), 1 = accepted with the EXACT
// distance in t_out, -1 = too close to call (the caller runs aabb_intersect).  An accepted distance is one slab
// quotient -- tmin, the largest lower quotient, when it is above minD, else tmax, the smallest upper one -- so
// when the f32 estimates single out that axis by more than their error bounds, the exact distance is that
// axis's correctly rounded f64 quotient (p -+ h) / d: one division instead of aabb_slab's six.  The lower
// quotient of an axis is (p - h) / d for d > 0 and (p + h) / d for d < 0 (division rounds monotonically, and
// h >= 0), as aabb_slab's swap leaves it; p = c - o in f32 and p +- h exact in f64, as aabb_slab forms them.
template <class T>  // T: float in any address space
JSRT_HD int box_closest_f32(const T *c, const T *h, F3 o, F3 d, const BoxRay &r, double minD, double lim, double &t_out) {
    constexpr float EPS = 4.76837158203125e-7f, TINY = 1e-30f;  // 2^-21
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    float lo[3], hi[3];
    float tmin = -__builtin_inff(), tmax = __builtin_inff();
    int kmin = -1, kmax = -1;
    bool out = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float p = c[i] - oo[i];
        lo[i] = -__builtin_inff();
        hi[i] = __builtin_inff();
        if ((r.skip >> i) & 1u) {
            out = out || fabsf(p) > h[i];  // exact: both f32
        } else {
            const float a = (p + h[i]) * r.inv[i], b = (p - h[i]) * r.inv[i];
            lo[i] = fminf(a, b);
            hi[i] = fmaxf(a, b);
            if (kmin < 0 || lo[i] > tmin) { tmin = lo[i]; kmin = i; }
            if (kmax < 0 || hi[i] < tmax) { tmax = hi[i]; kmax = i; }
        }
    }
    if (out) return 0;
    if (!__builtin_isfinite(tmin) || !__builtin_isfinite(tmax)) return -1;  // (also every axis skipped)
    const float f0 = (float)minD, f1 = (float)lim;
    if (!__builtin_isfinite(f0)) return -1;
    const bool inf1 = !__builtin_isfinite(f1) && f1 > 0;
    const float en = EPS * fabsf(tmin) + TINY, ex = EPS * fabsf(tmax) + TINY;
    const float e0 = EPS * fabsf(f0) + TINY, e1 = inf1 ? 0.0f : EPS * fabsf(f1) + TINY;
    int k = -1;
    bool lower = true;
    if (tmin - en > f0 + e0) {  // tmin > minD: t = tmin
        const bool lt1 = inf1 || tmin + en < f1 - e1, gt1 = !inf1 && tmin - en > f1 + e1;
        if (gt1 || tmin - en > tmax + ex) return 0;
        if (!(lt1 && tmin + en < tmax - ex)) return -1;
        k = kmin;
    } else if (tmin + en < f0 - e0) {  // tmin < minD: t = tmax
        const bool lt1 = inf1 || tmax + ex < f1 - e1, gt1 = !inf1 && tmax - ex > f1 + e1;
        if (tmax + ex < f0 - e0 || gt1) return 0;
        if (!(tmax - ex > f0 + e0 && lt1)) return -1;
        k = kmax;
        lower = false;
    } else {
        return -1;
    }
    // the extreme quotient's axis, separated from the others by the error bounds
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (j == k || ((r.skip >> j) & 1u)) continue;
        if (lower ? !(lo[j] + (EPS * fabsf(lo[j]) + TINY) < tmin - en) : !(hi[j] - (EPS * fabsf(hi[j]) + TINY) > tmax + ex))
            return -1;
    }
    const double p = (double)(c[k] - oo[k]), hh = (double)h[k], di = (double)dd[k];
    t_out = ((di > 0) == lower) ? (p - hh) / di : (p + hh) / di;
    return 1;
}

JSRT_HD double plane_t(F3 o, F3 d) {  // geometry.js:246-248
    return (d.z != 0.0f) ? -(double)o.z / (double)d.z : -DINF;
}

JSRT_HD double sphere_static(F3 o, F3 d, double minD) {  // geometry.js:429-442
    const double a = dot3(d, d), b = dot3(d, o), c = dot3(o, o) - 1;
    double big = b * b - a * c;
    if (big < 0 || a == 0) return -DINF;
    big = sqrt(big);
    const double t1 = (-b + big) / a, t2 = (-b - big) / a;
    if (t1 >= minD && t2 >= minD) return js_min(t1, t2);
    return (t2 < minD) ? t1 : t2;
}

JSRT_HD double tri_intersect(const DTri &T, F3 o, F3 d) {  // geometry.js:368-375
    const F3 n = f3(T.n[0], T.n[1], T.n[2]);
    const double denom = dot3(n, d);
    const double distance = (denom != 0) ? (T.delta - dot3(n, o)) / denom : -DINF;
    if (!__builtin_isfinite(distance) || distance < 0) return distance;
    const F3 p = ray_point(o, d, distance);
    const F3 v2 = f3(p.x - T.p0[0], p.y - T.p0[1], p.z - T.p0[2]);
    const double d20 = dot3(v2, f3(T.v0[0], T.v0[1], T.v0[2])), d21 = dot3(v2, f3(T.v1[0], T.v1[1], T.v1[2]));
    const double v = (T.d11 * d20 - T.d01 * d21) / T.denom, w = (T.d00 * d21 - T.d01 * d20) / T.denom;
    const float b0 = (float)(1 - v - w), b1 = (float)v, b2 = (float)w;
    return (b0 >= 0 && b0 <= 1 && b1 >= 0 && b1 <= 1 && b2 >= 0 && b2 <= 1) ? distance : -DINF;
}


// f32 reciprocal within 1 ulp (v_rcp_f32 on the device; the host build of the tests divides, inside the same
// bound)
JSRT_HD float rcp_f32(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// Any-hit acceptance of a Triangle in a shadow cast (tri_intersect's result accepted by minD < t < maxD),
// decided in f32: 1 / 0 / -1 as planar_any_f32.  The plane distance num / denom (num and denom the exact
// path's own f64 values) is estimated as f32(num) * rcp(f32(denom)), within 2^-20 relative; the hit point
// then moves by at most 2^-18 (|d t| + |o|) per component (planar_any_f32), v2 = p - p0 by that plus
// 2^-22 (|p| + |p0|), and the dots, Cramer numerators and quotients, evaluated in f32 from the f64 Gram
// terms, carry the propagated bound plus 2^-20 of their magnitudes (at most ~8 f32 roundings of 2^-24
// each).  A barycentric b = f32(x) is in [0, 1] whenever x is (f32 rounding is monotone and keeps 0 and
// 1), below 0 when x < -1e-30 and above 1 when x > 1 + 2^-22; a decision outside the margins is therefore
// the exact test's outcome.  The three correctly rounded f64 divisions run only when it is too close.
JSRT_HD int tri_any_f32(const DTri &T, F3 o, F3 d, double minD, double maxD, double &t_out) {
    constexpr float EPS = 4.76837158203125e-7f, EPST = 9.5367431640625e-7f, EPSP = 3.814697265625e-6f;
    constexpr float E22 = 2.384185791015625e-7f, TINY = 1e-30f;  // 2^-21, 2^-20, 2^-18, 2^-22
    const F3 n = f3(T.n[0], T.n[1], T.n[2]);
    const double denom = dot3(n, d);
    if (denom == 0) return 0;  // tri_intersect: -inf
    const double num = T.delta - dot3(n, o);
    const float fd = (float)denom, fn = (float)num;
    if (!(fabsf(fd) >= 1e-30f && fabsf(fd) <= 1e30f) || !(fabsf(fn) <= 1e30f) || (fn != 0.0f && fabsf(fn) < 1e-20f))
        return -1;
    const float t = fn * rcp_f32(fd);
    const float f0 = (float)minD, f1 = (float)maxD;
    if (!__builtin_isfinite(t) || !__builtin_isfinite(f0)) return -1;
    const bool inf1 = !__builtin_isfinite(f1) && f1 > 0;
    const float et = EPST * fabsf(t) + TINY, e0 = EPS * fabsf(f0) + TINY, e1 = inf1 ? 0.0f : EPS * fabsf(f1) + TINY;
    if (t + et < f0 - e0 || (!inf1 && t - et > f1 + e1)) return 0;
    if (!(t - et > f0 + e0 && (inf1 || t + et < f1 - e1))) return -1;
    // the hit point and v2 = p - p0, with per-component bounds
    const float s[3] = {d.x * t, d.y * t, d.z * t}, oo[3] = {o.x, o.y, o.z};
    float v2[3], ev[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float pk = oo[k] + s[k];
        v2[k] = pk - T.p0[k];
        ev[k] = EPSP * (fabsf(s[k]) + fabsf(oo[k])) + E22 * (fabsf(pk) + fabsf(T.p0[k])) + TINY;
    }
    const float d20 = v2[0] * T.v0[0] + v2[1] * T.v0[1] + v2[2] * T.v0[2];
    const float d21 = v2[0] * T.v1[0] + v2[1] * T.v1[1] + v2[2] * T.v1[2];
    const float a20 = fabsf(v2[0] * T.v0[0]) + fabsf(v2[1] * T.v0[1]) + fabsf(v2[2] * T.v0[2]);
    const float a21 = fabsf(v2[0] * T.v1[0]) + fabsf(v2[1] * T.v1[1]) + fabsf(v2[2] * T.v1[2]);
    const float e20 = ev[0] * fabsf(T.v0[0]) + ev[1] * fabsf(T.v0[1]) + ev[2] * fabsf(T.v0[2]) + EPST * a20 + TINY;
    const float e21 = ev[0] * fabsf(T.v1[0]) + ev[1] * fabsf(T.v1[1]) + ev[2] * fabsf(T.v1[2]) + EPST * a21 + TINY;
    const float d00 = (float)T.d00, d11 = (float)T.d11, d01 = (float)T.d01, fden = (float)T.denom;
    if (!(fabsf(fden) >= 1e-30f) || !__builtin_isfinite(fden)) return -1;
    const float ia = fabsf(rcp_f32(fden));
    const float vn = d11 * d20 - d01 * d21, wn = d00 * d21 - d01 * d20;
    const float mv = fabsf(d11 * d20) + fabsf(d01 * d21), mw = fabsf(d00 * d21) + fabsf(d01 * d20);
    const float v = vn * rcp_f32(fden), w = wn * rcp_f32(fden);
    const float ebv = (fabsf(d11) * e20 + fabsf(d01) * e21 + EPST * mv) * ia + EPST * fabsf(v) + TINY;
    const float ebw = (fabsf(d00) * e21 + fabsf(d01) * e20 + EPST * mw) * ia + EPST * fabsf(w) + TINY;
    const float b0 = 1.0f - v - w, eb0 = ebv + ebw + EPST * (1.0f + fabsf(v) + fabsf(w));
    if (!__builtin_isfinite(b0) || !__builtin_isfinite(eb0) || !__builtin_isfinite(ebv) || !__builtin_isfinite(ebw))
        return -1;
    const float x[3] = {b0, v, w}, e[3] = {eb0, ebv, ebw};
    bool in = true, out = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        out = out || x[k] + e[k] < -1e-30f || x[k] - e[k] > 1.0f + E22;
        in = in && x[k] - e[k] >= 0.0f && x[k] + e[k] <= 1.0f;
    }
    if (out) return 0;
    if (in) {
        t_out = t;
        return 1;
    }
    return -1;
}
// a Triangle's distance as a shadow cast reads it (tri_any_f32, the exact test only when too close to call)
// (opt-in, -DJSRT_TRI_ANY: it raises the mesh k_shadow's spills from 42 to 95 and loses -- bunny k_shadow
// 26.3 -> 37.2 ms, the dragon 789 -> 749 M/s, profiles/r04_s10_ab.txt)
JSRT_HD double tri_any(const DTri &T, F3 o, F3 d, double minD, double maxD) {
#if !defined(JSRT_NO_ANY_FILTER) && defined(JSRT_TRI_ANY)
    double t = 0;
    const int dec = tri_any_f32(T, o, d, minD, maxD, t);
    if (dec >= 0) return dec ? t : -DINF;
#endif
    return tri_intersect(T, o, d);
}

// --------------------------------------------------------------------------------------------
// SDF program VM (sdf_program.h).  P is the 4-vector point with w == 1.
//
// Every lane that runs the VM runs the same program in lockstep (the wave marches one SDF), so the
// program counter, the stack pointers and the loop counters are wave-uniform: they are kept in
// SGPRs (readfirstlane), instruction fetch is a scalar load and the opcode switch is a scalar
// branch.  The stacks are small fixed register files indexed by those uniform values.
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// read-only scene data addressed by a wave-uniform index, viewed in the constant address space so the
// compiler may load it with scalar loads (generic pointers get per-lane vector loads)
#define CONST_AS __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const CONST_AS T *as_const(const T *p) {
    return (const CONST_AS T *)p;
}

// BoxSDF.distanceComp (sdf.js:276-279): q = p.abs().minus(size).to4(0);
// Vec.max(q, 0).norm() + min(max(q0, q1, q2), 0)
template <class T>
JSRT_HD double sdf_box(const T *k, F3 P) {
    const float qx = fabsf(P.x) - (float)k[0];
    const float qy = or0(fabsf(P.y) - (float)k[1]);
    const float qz = or0(fabsf(P.z) - (float)k[2]);
    // Math.max / Math.min of f32 values are f32 values: evaluated in f32 (js_maxf)
    const F3 m = f3(js_max0f(qx), js_max0f(qy), js_max0f(qz));
    return sqrt(dot3(m, m)) + (double)js_min0f(js_maxf(js_maxf(qx, qy), qz));
}

// UnionSDF of n BoxSDFs (k: 4 doubles apart), Math.min(d_0, ..., d_n-1) (sdf.js:83-85), with ONE square
// root.  A box's distance is sqrt(a) + c, a = |max(q, 0)|^2 (f64), c = min(max(q), 0) (f32):
//   outside (a > 0): c is +0 and the distance sqrt(a) > 0;  inside or on it (a == 0): 0 + c <= 0.
// So an inside box's distance is below every outside one, and among outside boxes the correctly rounded
// square root is monotone: min_i RN(sqrt(a_i)) = RN(sqrt(min_i a_i)).  The minimum is therefore the
// smallest inside distance if there is one, else the root of the smallest a -- bit for bit Math.min's
// value (no -0 arises: +0 + -0 is +0), with a NaN from any box kept (tests/test_sdf_box.py).
template <class T>
JSRT_HD double sdf_minbox(const T *k, int n, F3 P) {
    double amin = __builtin_inf(), din = 0.0;
    bool inside = false, nan = false;
    for (int i = 0; i < n; ++i) {
        const T *b = k + 4 * i;
        const float qx = fabsf(P.x) - (float)b[0];
        const float qy = or0(fabsf(P.y) - (float)b[1]);
        const float qz = or0(fabsf(P.z) - (float)b[2]);
        const F3 m = f3(js_max0f(qx), js_max0f(qy), js_max0f(qz));
        const double a = dot3(m, m);
        const float c = js_min0f(js_maxf(js_maxf(qx, qy), qz));
        nan = nan || a != a || c != c;
        if (a == 0.0) {
            const double d = 0.0 + (double)c;
            din = inside ? (d < din ? d : din) : d;
            inside = true;
        } else {
            amin = a < amin ? a : amin;
        }
    }
    const double r = inside ? din : sqrt(amin);
    return nan ? __builtin_nan("") : r;
}

// sdf_minbox of the Menger sponge's cross (MINBOX pad 1: the host matched three boxes, box i infinite along axis
// i, every other half size the same f32 h; tests/SDF_Menger/test.mjs:27-36), bit for bit.  For finite P the bars
// share q_i = |p_i| - h (or0 changes nothing: no NaN, and a zero difference of two non-negative values is +0),
// and a bar's infinite axis has q = -inf: max(q, 0) = +0 and js_maxf(-inf, v) = js_maxf(v, -inf) = v.  So bar x
// has a = |m|^2 = fma(mz, mz, my^2) (dot3 with a zero term: fma(0, 0, c) = c for c >= +0; the squares of f32
// values are exact) and c = min(max(qy, qz), 0), and likewise y, z -- one subtraction, one max0 and one square
// per axis instead of per box and axis.  No -0 or NaN arises, so the plain comparisons are Math.max / min.  A
// non-finite P (|p| - inf is NaN there) takes sdf_minbox.
template <class T>
JSRT_HD double sdf_cross(const T *k, F3 P) {
    if (!(fabsf(P.x) <= __FLT_MAX__ && fabsf(P.y) <= __FLT_MAX__ && fabsf(P.z) <= __FLT_MAX__)) return sdf_minbox(k, 3, P);
    const float h = (float)k[1];
    const float qx = fabsf(P.x) - h, qy = fabsf(P.y) - h, qz = fabsf(P.z) - h;
    const double mx = qx > 0.0f ? qx : 0.0f, my = qy > 0.0f ? qy : 0.0f, mz = qz > 0.0f ? qz : 0.0f;
    const double sx = mx * mx, sy = my * my;
    const double a[3] = {fma(mz, mz, sy), fma(mz, mz, sx), fma(mx, mx, sy)};
    const float c[3] = {qy > qz ? qy : qz, qx > qz ? qx : qz, qx > qy ? qx : qy};
    double amin = __builtin_inf(), din = 0.0;
    bool inside = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (a[i] == 0.0) {
            const double d = 0.0 + (double)(c[i] > 0.0f ? 0.0f : c[i]);
            din = inside ? (d < din ? d : din) : d;
            inside = true;
        } else {
            amin = a[i] < amin ? a[i] : amin;
        }
    }
    return inside ? din : sqrt(amin);
}

// SDFInfiniteRepetitionTransformer.transform (sdf.js:471-473): Math.fmod(p + s/2, s) - s/2 per axis.
// k[3..5]: 1/s when s is a power of two (x / s and x * (1 / s) are then the same rounding of the
// same real number), else 0.
template <class T>
__device__ __forceinline__ float sdf_rep1(const T *k, int i, float p) {  // axis i, before sdf_xrep's `|| 0`
    const double s = k[i], inv = k[3 + i], a = (double)p + s / 2;
    const double q = floor(inv != 0.0 ? a * inv : a / s);
    return (float)(to_precision8_sl(a - (q * s)) - s / 2);  // math.js:27 (branch-free form, js_number.h)
}
template <class T>
__device__ __forceinline__ F3 sdf_xrep(const T *k, F3 P) {
    return f3(sdf_rep1(k, 0, P.x), or0(sdf_rep1(k, 1, P.y)), or0(sdf_rep1(k, 2, P.z)));
}

template <int N>
struct RegFile {  // per-lane doubles addressed by a wave-uniform index
    double r[N];
    __device__ __forceinline__ double get(int i) const {
        double v = r[0];
#pragma unroll
        for (int k = 1; k < N; ++k)
            if (i == k) v = r[k];
        return v;
    }
    __device__ __forceinline__ void set(int i, double v) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (i == k) r[k] = v;
    }
};

#include "sdf_forms.h"

__device__ __forceinline__ double sdf_run(const DScene &S, int pc, int end, F3 P) {
    RegFile<SDF_MAX_D> dst;
    RegFile<SDF_MAX_S> sst;
    F3 pst0 = P, pst1 = P;  // SDF_MAX_P == 2
    int lc0 = 0, lc1 = 0;   // SDF_MAX_LOOP == 2
    int dsp = 0, psp = 0, ssp = 0, lsp = 0;
    // The program and its constants are read-only and every index is wave-uniform: through the
    // constant address space the loads are scalar (s_load, scalar cache) instead of a vector load per
    // lane on the interpreter's dependent chain.
    const CONST_AS SdfInsn *code = as_const(S.sdf_insn);
    const CONST_AS double *K = as_const(S.sdf_const);
    pc = uni(pc);  // uniform among the active lanes (sdf_node_dist's waterfall)
    end = uni(end);
    if (uni(code[pc].op) == SOP_FORM) return sdf_form_any(K, code, pc, P);  // straight-line code (sdf_forms.h)
    while (pc < end) {
        const int op = uni(code[pc].op), ia = uni(code[pc].a), ib = uni(code[pc].b);
        switch (op) {
        case SOP_END: pc = end; continue;
        case SOP_BOX: dst.set(dsp++, sdf_box(K + ia, P)); break;
        case SOP_SPHERE: {  // p.to4(0).norm() - radius (sdf.js:232-234)
            const F3 q = f3(P.x, or0(P.y), or0(P.z));
            dst.set(dsp++, sqrt(dot3(q, q)) - K[ia]);
            break;
        }
        case SOP_TETRA:  // sdf.js:305-308
            dst.set(dsp++, (js_max(fabs((double)P.x + (double)P.y) - (double)P.z,
                                   fabs((double)P.x - (double)P.y) + (double)P.z) - 1) / sqrt(3.0));
            break;
        case SOP_MIN: {
            double r = dst.get(dsp - ia);
            for (int i = 1; i < ia; ++i) r = js_min(r, dst.get(dsp - ia + i));
            dsp -= ia;
            dst.set(dsp++, r);
            break;
        }
        case SOP_MAX: {
            double r = dst.get(dsp - ia);
            for (int i = 1; i < ia; ++i) r = js_max(r, dst.get(dsp - ia + i));
            dsp -= ia;
            dst.set(dsp++, r);
            break;
        }
        case SOP_NEG: dst.set(dsp - 1, -dst.get(dsp - 1)); break;
        case SOP_SUBK: dst.set(dsp - 1, dst.get(dsp - 1) - K[ia]); break;
        case SOP_SMIN: {  // smoothMin (sdf.js:128-131)
            const double b = dst.get(--dsp), a = dst.get(dsp - 1), k = K[ia];
            const double h = js_max(k - fabs(a - b), 0.0) / k;
            dst.set(dsp - 1, js_min(a, b) - h * h * h * k * (1.0 / 6.0));
            break;
        }
        case SOP_PUSHP:
            if (psp == 0) pst0 = P;
            else pst1 = P;
            ++psp;
            break;
        case SOP_POPP:
            --psp;
            P = psp == 0 ? pst0 : pst1;
            break;
        case SOP_TPUSH: sst.set(ssp++, 1.0); break;
        case SOP_TPOP: --ssp; break;
        case SOP_TPOP_MUL: {
            const double st = sst.get(--ssp);
            sst.set(ssp - 1, sst.get(ssp - 1) * st);
            break;
        }
        case SOP_MULS: dst.set(dsp - 1, dst.get(dsp - 1) * sst.get(ssp - 1)); break;
        case SOP_XMAT:  // SDFMatrixTransformer.transform (sdf.js:433-435)
            P = xf_point(K + ia, P);
            sst.set(ssp - 1, sst.get(ssp - 1) * K[ib]);
            break;
        case SOP_XREF: {  // SDFReflectionTransformer.transformComp (sdf.js:450-455)
            const F3 n = f3((float)K[ia], (float)K[ia + 1], (float)K[ia + 2]);
            const double dt = dot3(n, P) - K[ia + 3];
            if (dt < 0) P = sub(P, scale(n, 2 * dt));
            break;
        }
        case SOP_XREP: P = sdf_xrep(K + ia, P); break;
        case SOP_MINBOX:  // BOX x ib, MIN ib (pad 1: the Menger cross)
            dst.set(dsp++, uni(code[pc].pad) ? sdf_cross(K + ia, P) : sdf_minbox(K + ia, ib, P));
            break;
        case SOP_XMATS:  // TPUSH XMAT TPOP_MUL
            P = xf_point(K + ia, P);
            sst.set(ssp - 1, sst.get(ssp - 1) * (1.0 * K[ib]));
            break;
        case SOP_XMATREP: {  // TPUSH XMATS XREP TPOP_MUL
            const int ic = uni(code[pc].pad);
            P = sdf_xrep(K + ic, xf_point(K + ia, P));
            sst.set(ssp - 1, sst.get(ssp - 1) * (1.0 * (1.0 * K[ib])));
            break;
        }
        case SOP_MULSMIN: {  // MULS, MIN 2
            const double d = dst.get(dsp - 1) * sst.get(ssp - 1);
            --dsp;
            dst.set(dsp - 1, js_min(dst.get(dsp - 1), d));
            break;
        }
        case SOP_LOOP:
            if (ia <= 0) { pc = ib + 1; continue; }
            if (lsp == 0) lc0 = ia;
            else lc1 = ia;
            ++lsp;
            break;
        case SOP_ENDLOOP: {
            int c = (lsp == 1 ? lc0 : lc1) - 1;
            if (lsp == 1) lc0 = c;
            else lc1 = c;
            if (c > 0) { pc = ia + 1; continue; }
            --lsp;
            break;
        }
        default: break;
        }
        ++pc;
    }
    return dst.get(0);
}

// Lanes may ask for different nodes (getMaterialData picks children per lane, a BVH leaf may hold
// different SDF primitives): a waterfall runs the VM once per distinct program among the active
// lanes, each time with a uniform program counter.
__device__ __forceinline__ double sdf_node_dist(const DScene &S, int n, F3 p) {
    const int pc = S.sdf_range[2 * n], end = S.sdf_range[2 * n + 1];
    double r = 0;
    for (;;) {
        const int pcu = uni(pc);
        if (pc == pcu) {
            r = sdf_run(S, pcu, end, p);
            break;
        }
    }
    return r;
}

// SDF node n's distance when its program is a recognised form (DScene::sdf_all_forms: every geometry
// root is one): the form's straight-line code only, so a kernel that needs no VM does not carry its
// register files (the persistent marches: k_extend_q / k_shadow_cast).
__device__ __forceinline__ double sdf_form_dist(const DScene &S, int n, F3 p) {
    const CONST_AS SdfInsn *code = as_const(S.sdf_insn);
    const CONST_AS double *K = as_const(S.sdf_const);
    const int pc = S.sdf_range[2 * n];
    double r = 0;
    for (;;) {  // waterfall over the lanes' nodes (a wave marches one SDF in every reference scene)
        const int pcu = uni(pc);
        if (pc == pcu) {
            r = sdf_form_any(K, code, pcu, p);
            break;
        }
    }
    return r;
}

__device__ __forceinline__ double sdf_intersect(const DScene &S, int g, F3 o, F3 d, double minD, double maxD) {  // sdf.js:12-40
    const jsrt_rec_sdfgeom &G = S.sdfg[g];
    double bmin, bmax;
    if (!aabb_slab(G.center[0], G.center[1], G.center[2], G.half[0], G.half[1], G.half[2], o, d, minD, maxD, bmin,
                   bmax))
        return -DINF;
    minD = js_max(minD, bmin);
    maxD = js_min(maxD, bmax);
    double t = minD;
    const double rd_norm = sqrt(dot3(d, d));
    for (int i = 0; i < G.max_samples; ++i) {
        const F3 p = ray_point(o, d, t);
        const double distance = sdf_node_dist(S, G.root, p);
        if (!__builtin_isfinite(distance)) break;
        if (distance <= G.eps) return t;
        t += distance / rd_norm;
        if (t < minD || t > maxD || (t - minD) * rd_norm > G.max_trace) break;
    }
    return -DINF;
}

// SDF getMaterialData (sdf.js:87-360).  Smooth combinators blend both subtrees' data, so the walk
// keeps a small explicit stack of pending blends.
struct SdfMD {
    F3 bc;
    float u, v;
    int has_bc, has_uv;
};

__device__ __forceinline__ SdfMD sdf_leaf_md(const DScene &S, const jsrt_rec_sdfnode &N, F3 p) {
    SdfMD r;
    r.bc = f3(N.basecolor[0], N.basecolor[1], N.basecolor[2]);
    r.has_bc = 1;
    r.has_uv = 0;
    r.u = r.v = 0;
    if (N.kind == JSRT_SDF_SPHERE) {  // UV: cartesianToSpherical(p.to4(0).normalized())
        r.has_uv = 1;
        cart_to_sph(normalized(f3(p.x, or0(p.y), or0(p.z))), r.u, r.v);
    }
    return r;
}

// hint (sdf_forms.h sdf_form_normal4): the root Difference's two operand distances at p, already evaluated
__device__ __forceinline__ SdfMD sdf_material(const DScene &S, int root, F3 p, const double *hint = nullptr) {
    // Iterative post-order over the (binary) blend nodes; simple selector nodes are followed in place.
    struct Pending {
        int node;      // smooth node waiting for its children
        double mixf;
        int stage;     // 0: evaluating child a, 1: evaluating child b
        SdfMD a;
    };
    Pending stk[8];
    int sp = 0;
    int n = root;
    SdfMD res;
    for (int guard = 0; guard < 256; ++guard) {
        const jsrt_rec_sdfnode &N = S.sdf_nodes[n];
        bool leaf = false;
        switch (N.kind) {
        case JSRT_SDF_UNION:
        case JSRT_SDF_INTERSECTION: {  // Math.indexOfMin / indexOfMax (math.js:53-70)
            int best = 0;
            double bv = N.kind == JSRT_SDF_UNION ? DINF : -DINF;
            for (int i = 0; i < N.count; ++i) {
                const double d = sdf_node_dist(S, S.sdf_child[N.first + i], p);
                if (N.kind == JSRT_SDF_UNION ? (d < bv) : (d > bv)) { bv = d; best = i; }
            }
            n = S.sdf_child[N.first + best];
            continue;
        }
        case JSRT_SDF_DIFFERENCE:
            if (hint && n == root) {
                n = (hint[0] > -hint[1]) ? N.a : N.b;
                continue;
            }
            n = (sdf_node_dist(S, N.a, p) > -sdf_node_dist(S, N.b, p)) ? N.a : N.b;
            continue;
        case JSRT_SDF_ROUND:
        case JSRT_SDF_TRANSFORM:
        case JSRT_SDF_RECURSIVE_UNION: n = N.a; continue;
        case JSRT_SDF_SMOOTH_UNION:
        case JSRT_SDF_SMOOTH_INTERSECTION:
        case JSRT_SDF_SMOOTH_DIFFERENCE: {
            const double da = sdf_node_dist(S, N.a, p), db = sdf_node_dist(S, N.b, p), k = N.k;
            double x, y;  // smoothMinBlend arguments (sdf.js:133-137, 151, 172, 193)
            if (N.kind == JSRT_SDF_SMOOTH_UNION) { x = da; y = db; }
            else if (N.kind == JSRT_SDF_SMOOTH_INTERSECTION) { x = -da; y = -db; }
            else { x = -da; y = db; }
            const double h = js_max(k - fabs(x - y), 0.0) / k;
            const double m = h * h * h * 0.5;
            double mixf = (x < y) ? m : (1.0 - m);
            if (N.kind == JSRT_SDF_SMOOTH_INTERSECTION) mixf = 1.0 - mixf;
            if (sp >= 8) return res;
            stk[sp].node = n;
            stk[sp].mixf = mixf;
            stk[sp].stage = 0;
            ++sp;
            n = N.a;
            continue;
        }
        default: leaf = true; res = sdf_leaf_md(S, N, p); break;
        }
        if (!leaf) break;
        // unwind finished subtrees into pending blends (SDF.blendMaterialData, sdf.js:66-73)
        while (sp > 0) {
            Pending &T = stk[sp - 1];
            if (T.stage == 0) {
                T.a = res;
                T.stage = 1;
                n = S.sdf_nodes[T.node].b;
                break;
            }
            const SdfMD a = T.a, b = res;
            const double mixf = T.mixf;
            --sp;
            if (mixf <= 0.0) res = a;
            else if (mixf >= 1.0) res = b;
            else {
                const F3 ca = a.has_bc ? a.bc : f3(1, 1, 1), cb = b.has_bc ? b.bc : f3(1, 1, 1);
                const float ua = a.has_uv ? a.u : 0.0f, va = a.has_uv ? a.v : 0.0f;
                const float ub = b.has_uv ? b.u : 0.0f, vb = b.has_uv ? b.v : 0.0f;
                res.bc = f3((float)((1 - mixf) * ca.x + mixf * cb.x), (float)((1 - mixf) * ca.y + mixf * cb.y),
                            (float)((1 - mixf) * ca.z + mixf * cb.z));
                res.u = (float)((1 - mixf) * ua + mixf * ub);
                res.v = (float)((1 - mixf) * va + mixf * vb);
                res.has_bc = res.has_uv = 1;
            }
        }
        if (sp == 0) return res;
    }
    return res;
}

// --------------------------------------------------------------------------------------------
// world intersection (world.js:7-15, 116-124; aggregates.js:14-18, 43-49, 207-225)
struct Hit {
    double t;
    int prim;
    int ctx;
};

template <int PF, class PT>  // PT: DPrim in any address space
__device__ __forceinline__ double prim_intersect_local(const DScene &S, const PT &P, F3 o, F3 d, double minD,
                                                       double maxD) {
    switch (P.gkind) {
    case JSRT_GEOM_PLANE: return plane_t(o, d);
    case JSRT_GEOM_SQUARE: {  // geometry.js:287-291
        const double t = plane_t(o, d);
        const F3 p = ray_point(o, d, t);
        return (-0.5f <= p.x && p.x <= 0.5f && -0.5f <= p.y && p.y <= 0.5f) ? t : -DINF;
    }
    case JSRT_GEOM_CIRCLE: {  // geometry.js:310-314; the w term of p - (0,0,0,1) is 0 for finite t
        const double t = plane_t(o, d);
        const F3 p = ray_point(o, d, t);
        return (dot3(p, p) <= 1) ? t : -DINF;
    }
    case JSRT_GEOM_SPHERE: return sphere_static(o, d, minD);
    case JSRT_GEOM_CYLINDER: {  // geometry.js:473-478 (rays masked by Vec.of(1,1,0,1))
        const double oz = o.z, dz = d.z;
        if (fabs(oz) > 1 && dz != 0) minD = js_max(minD, -(oz - js_sign(oz)) / dz);
        const double t = sphere_static(f3(o.x, o.y, o.z * 0.0f), f3(d.x, d.y, d.z * 0.0f), minD);
        return (fabs(oz + t * dz) <= 1) ? t : -DINF;
    }
    case JSRT_GEOM_AABB: return aabb_intersect(P.center, P.half, o, d, minD, maxD);
    case JSRT_GEOM_TRIANGLE:
        if (PF & PF_TRI) return tri_intersect(S.tris[P.gindex], o, d);
        return -DINF;
    case JSRT_GEOM_SDF:
        if (PF & PF_SDF) return sdf_intersect(S, P.gindex, o, d, minD, maxD);
        return -DINF;
    default: return -DINF;
    }
}

// one row of Mat x Vec (math.js:392-397), the same operations as xf_point / xf_dir
template <class T>
JSRT_HD float xf_row_point(const T *r, F3 o) {
    return (float)((((double)o.x * r[0] + (double)o.y * r[1]) + (double)o.z * r[2]) + r[3]);
}
template <class T>
JSRT_HD float xf_row_dir(const T *r, F3 d) {
    return (float)(((double)d.x * r[0] + (double)d.y * r[1]) + (double)d.z * r[2]);
}

// SimplePlane / Square / Circle .intersect of a world ray through the primitive's inverse transform
// `inv` (rows 0..2), for a caller that accepts minD < t < lim: a planar primitive whose plane
// distance already fails that test may return it without transforming the x/y rows or testing its
// bounds; the caller's decision is unchanged.
template <class T>
JSRT_HD double planar_intersect(int k, const T *inv, F3 o, F3 d, double minD, double lim) {
    // SimplePlane.intersect (geometry.js:246-248) needs only the local z row
    const float oz = xf_row_point(inv + 8, o), dz = xf_row_dir(inv + 8, d);
    const double t = (dz != 0.0f) ? -(double)oz / (double)dz : -(double)__builtin_inf();
    if (k == JSRT_GEOM_PLANE || !(t > minD && t < lim)) return t;
    const float ox = xf_row_point(inv, o), oy = xf_row_point(inv + 4, o);
    const float dx = xf_row_dir(inv, d), dy = xf_row_dir(inv + 4, d);
    const F3 p = ray_point(f3(ox, oy, oz), f3(dx, dy, dz), t);
    if (k == JSRT_GEOM_SQUARE)  // geometry.js:287-291
        return (-0.5f <= p.x && p.x <= 0.5f && -0.5f <= p.y && p.y <= 0.5f) ? t : -(double)__builtin_inf();
    return (dot3(p, p) <= 1) ? t : -(double)__builtin_inf();  // Circle, geometry.js:310-314
}

#ifdef JSRT_X_F32XF
// (timing experiment only) the any-hit filters' local rays from an f32 transform
template <class T>
__device__ __forceinline__ float xf_row_point_x(const T *r, F3 o) {
    return fmaf(o.x, (float)r[0], fmaf(o.y, (float)r[1], fmaf(o.z, (float)r[2], (float)r[3])));
}
template <class T>
__device__ __forceinline__ float xf_row_dir_x(const T *r, F3 d) {
    return fmaf(d.x, (float)r[0], fmaf(d.y, (float)r[1], d.z * (float)r[2]));
}
#define XROWP xf_row_point_x
#define XROWD xf_row_dir_x
#else
#define XROWP xf_row_point
#define XROWD xf_row_dir
#endif

// Any-hit acceptance of a SimplePlane / Square / Circle in a shadow cast (planar_intersect's result accepted
// by minD < t < maxD; `best` is +inf on every lane still casting), decided in f32: 1 = accepted (t_out = the
// f32 estimate of the distance, inside the bounds by the margin), 0 = not accepted, -1 = too close to call
// (the caller runs planar_intersect).  The plane distance -oz / dz is estimated as -oz * rcp(dz) (within
// 2^-21 relative: rcp's 1 ulp and the product's rounding); the hit point p = o + (f32)(d * t), which the exact
// path forms from the f64 distance with two f32 roundings, moves by at most 2^-18 (|d t| + |o|) per
// component under the estimate, so a bound test decided outside that margin is the exact test's outcome.
template <class T>
JSRT_HD int planar_any_f32(int k, const T *inv, F3 o, F3 d, double minD, double maxD, double &t_out) {
    constexpr float EPS = 4.76837158203125e-7f, EPSP = 3.814697265625e-6f, TINY = 1e-30f;  // 2^-21, 2^-18
    const float oz = XROWP(inv + 8, o), dz = XROWD(inv + 8, d);
    if (dz == 0.0f) return 0;  // t = -inf (planar_intersect's dz == 0 case): never accepted
#ifdef __HIP_DEVICE_COMPILE__
    const float ta = -oz * __builtin_amdgcn_rcpf(dz);  // v_rcp_f32: within 1 ulp
#else
    const float ta = -oz * (1.0f / dz);  // (host build of the tests: correctly rounded, inside the same bound)
#endif
    const float f0 = (float)minD, f1 = (float)maxD;
    if (!__builtin_isfinite(ta) || !__builtin_isfinite(f0) || !(fabsf(dz) >= 1e-30f)) return -1;
    const bool inf1 = !__builtin_isfinite(f1) && f1 > 0;
    const float et = EPS * fabsf(ta) + TINY, e0 = EPS * fabsf(f0) + TINY, e1 = inf1 ? 0.0f : EPS * fabsf(f1) + TINY;
    if (ta + et < f0 - e0 || (!inf1 && ta - et > f1 + e1)) return 0;
    if (!(ta - et > f0 + e0 && (inf1 || ta + et < f1 - e1))) return -1;
    if (k == JSRT_GEOM_PLANE) {
        t_out = ta;
        return 1;
    }
    const float ox = XROWP(inv, o), oy = XROWP(inv + 4, o);
    const float dx = XROWD(inv, d), dy = XROWD(inv + 4, d);
    const double td = (double)ta;
    const float sx = (float)((double)dx * td), sy = (float)((double)dy * td);
    const float px = ox + sx, py = oy + sy;
    const float ex = EPSP * (fabsf(sx) + fabsf(ox)) + TINY, ey = EPSP * (fabsf(sy) + fabsf(oy)) + TINY;
    if (!__builtin_isfinite(px) || !__builtin_isfinite(py) || !__builtin_isfinite(ex) || !__builtin_isfinite(ey))
        return -1;
    if (k == JSRT_GEOM_SQUARE) {  // -0.5 <= p.x <= 0.5 && -0.5 <= p.y <= 0.5
        if (fabsf(px) - ex > 0.5f || fabsf(py) - ey > 0.5f) return 0;
        if (fabsf(px) + ex < 0.5f && fabsf(py) + ey < 0.5f) {
            t_out = ta;
            return 1;
        }
        return -1;
    }
    // Circle: dot3(p, p) <= 1, with p.z = oz + (f32)(dz t) (the residual of the plane itself)
    const float sz = (float)((double)dz * td), pz = oz + sz;
    const float ez = EPSP * (fabsf(sz) + fabsf(oz)) + TINY;
    const double r2 = dot3(f3(px, py, pz), f3(px, py, pz));
    const double m = 2.0 * ((double)fabsf(px) * ex + (double)fabsf(py) * ey + (double)fabsf(pz) * ez) +
                     ((double)ex * ex + (double)ey * ey + (double)ez * ez) + 1e-15;
    if (!__builtin_isfinite(r2)) return -1;
    if (r2 - m > 1.0) return 0;
    if (r2 + m < 1.0) {
        t_out = ta;
        return 1;
    }
    return -1;
}

// Any-hit acceptance of a Sphere in a shadow cast (sphere_static's result accepted by minD < t < maxD),
// decided in f32: 1 / 0 / -1 as planar_any_f32.  a, b, c and the discriminant are the reference's f64
// values (the exact path's own operations); the square root and the two quotients are estimated in f32.
// Since a > 0, t1 >= t2 and sphere_static returns t = t2 >= minD ? t2 : t1.  Each estimate is within
// 2^-19 (sqrt(disc) / a + |t|) of the exact quotient: the f32 roundings of b, a and the discriminant
// (2^-24 each), sqrt and rcp (1 ulp each) and the f32 sum (2^-24 (|b| + sqrt(disc))), whose cancellation
// term is covered by sqrt(disc) / a when it is large and by |t| ~ |b| / a when sqrt(disc) is small.
JSRT_HD int sphere_any_f32(F3 o, F3 d, double minD, double maxD, double &t_out, bool *second = nullptr) {
    constexpr float EPS = 4.76837158203125e-7f, EPSS = 1.9073486328125e-6f, TINY = 1e-30f;  // 2^-21, 2^-19
    const double a = dot3(d, d), b = dot3(d, o), c = dot3(o, o) - 1;
    const double big = b * b - a * c;
    if (big < 0 || a == 0) return 0;  // sphere_static: -inf
    if (!(big >= 1e-30) || !(a >= 1e-30) || !(a <= 1e30) || !(fabs(b) <= 1e30) || !(big <= 1e30)) return -1;
    const float fa = (float)a, fb = (float)b;
#ifdef __HIP_DEVICE_COMPILE__
    const float sq = __builtin_amdgcn_sqrtf((float)big), ia = __builtin_amdgcn_rcpf(fa);
#else
    const float sq = sqrtf((float)big), ia = 1.0f / fa;
#endif
    const float t1 = (-fb + sq) * ia, t2 = (-fb - sq) * ia;
    const float base = EPSS * (sq * ia);
    const float e1 = base + EPSS * fabsf(t1) + TINY, e2 = base + EPSS * fabsf(t2) + TINY;
    const float f0 = (float)minD, f1 = (float)maxD;
    if (!__builtin_isfinite(f0)) return -1;
    const bool inf1 = !__builtin_isfinite(f1) && f1 > 0;
    const float em = EPS * fabsf(f0) + TINY, eM = inf1 ? 0.0f : EPS * fabsf(f1) + TINY;
    float t, et;
    if (t2 - e2 > f0 + em) {  // t2 > minD: t = t2
        t = t2;
        et = e2;
        if (second) *second = true;
    } else if (t2 + e2 < f0 - em) {  // t2 < minD: t = t1
        t = t1;
        et = e1;
        if (second) *second = false;
    } else {
        return -1;
    }
    if (t + et < f0 - em || (!inf1 && t - et > f1 + eM)) return 0;
    if (t - et > f0 + em && (inf1 || t + et < f1 - eM)) {
        t_out = t;
        return 1;
    }
    return -1;
}

// Closest-hit form of the Sphere test (sphere_static's distance kept when minD < t < lim), decided by
// sphere_any_f32 with maxD := lim: 0 = not accepted, 1 = accepted with the EXACT distance in t_out -- the root
// sphere_any_f32 settled on (t2 when it is above minD, else t1), from the reference's own f64 a, b and the
// correctly rounded square root, one division instead of two -- -1 = too close to call.  sphere_static returns
// min(t1, t2) when both are >= minD, t1 / t2 when only that one is, which for a > 0 (t1 >= t2) is t2 when
// t2 >= minD, else t1: the root sphere_any_f32 separated from minD by its margin.
JSRT_HD int sphere_closest_f32(F3 o, F3 d, double minD, double lim, double &t_out) {
    double te = 0;
    bool second = false;
    const int dec = sphere_any_f32(o, d, minD, lim, te, &second);
    if (dec != 1) return dec;
    const double a = dot3(d, d), b = dot3(d, o), c = dot3(o, o) - 1;
    const double big = sqrt(b * b - a * c);  // (sphere_any_f32 decided: b * b - a * c >= 1e-30, a >= 1e-30)
    t_out = second ? (-b - big) / a : (-b + big) / a;
    return 1;
}

// Primitive.intersect: Infinity for a non-shadow-casting primitive in a shadow cast.
// `lim` = the caller's acceptance bound min(best, maxD): every caller accepts a distance only when
// minD < t < lim, so a planar primitive whose plane distance already fails that test may return it
// without transforming the x/y rows or testing its bounds; the caller's decision is unchanged.
template <int PF, class PT>  // PT: DPrim in any address space
__device__ __forceinline__ double prim_intersect(const DScene &S, const PT &P, F3 o, F3 d, double minD, double maxD,
                                                 bool transp, double lim) {
    if (!transp && !P.casts_shadow) return DINF;
    const int k = P.gkind;
    if (k == JSRT_GEOM_PLANE || k == JSRT_GEOM_SQUARE || k == JSRT_GEOM_CIRCLE) return planar_intersect(k, P.inv, o, d, minD, lim);
    return prim_intersect_local<PF>(S, P, xf_point(P.inv, o), xf_dir(P.inv, d), minD, maxD);
}

// A Primitive's distance as a shadow cast reads it (accepted or not): for an AABB, planar, sphere or triangle geometry the f32
// decisions above (an accepted distance is the f32 estimate, a rejected one -inf), the exact test only for
// a decision too close to call; every other kind through prim_intersect.
template <int PF, class PT>
__device__ __forceinline__ double prim_any(const DScene &S, const PT &P, F3 o, F3 d, double minD, double maxD,
                                           bool transp) {
#ifndef JSRT_NO_ANY_FILTER
    if (!transp && !P.casts_shadow) return DINF;  // Primitive.intersect (as prim_intersect)
    const int k = P.gkind;
    double t = 0;
    if (k == JSRT_GEOM_AABB) {
#ifdef JSRT_X_F32XF
        const F3 lo = f3(XROWP(P.inv, o), XROWP(P.inv + 4, o), XROWP(P.inv + 8, o)),
                 ld = f3(XROWD(P.inv, d), XROWD(P.inv + 4, d), XROWD(P.inv + 8, d));
#else
        const F3 lo = xf_point(P.inv, o), ld = xf_dir(P.inv, d);
#endif
        const int dec = box_any_f32(P.center, P.half, lo, box_ray(ld), minD, maxD, t);
        if (dec >= 0) return dec ? t : -DINF;
        return aabb_intersect(P.center, P.half, lo, ld, minD, maxD);
    }
    if (k == JSRT_GEOM_PLANE || k == JSRT_GEOM_SQUARE || k == JSRT_GEOM_CIRCLE) {
        const int dec = planar_any_f32(k, P.inv, o, d, minD, maxD, t);
        if (dec >= 0) return dec ? t : -DINF;
        return planar_intersect(k, P.inv, o, d, minD, maxD);
    }
    if ((PF & PF_TRI) && k == JSRT_GEOM_TRIANGLE)
        return tri_any(S.tris[P.gindex], xf_point(P.inv, o), xf_dir(P.inv, d), minD, maxD);
    if (k == JSRT_GEOM_SPHERE) {
        const F3 lo = xf_point(P.inv, o), ld = xf_dir(P.inv, d);
        const int dec = sphere_any_f32(lo, ld, minD, maxD, t);
        if (dec >= 0) return dec ? t : -DINF;
        return sphere_static(lo, ld, minD);
    }
#endif
    return prim_intersect<PF>(S, P, o, d, minD, maxD, transp, maxD);
}

// Primitive.intersect for a closest-hit cast (world.js:7-15): the caller keeps a distance only when
// minD < t < lim (lim = min(maxD, the closest hit so far)), so for an AABB or Sphere geometry the f32 filters
// above decide that first; an accepted distance comes back exact (one division, box_closest_f32 /
// sphere_closest_f32), a rejected one as -Infinity, and only a decision too close to call runs the exact test.
// Not in the BVH profiles: there the top-level primitives are few and the filters' ~960 static instructions cost
// the latency-bound mesh k_extend more than they save (bunny k_extend 25.4 -> 25.0 ms, dragon 3,804 -> 3,756 ms
// without them, profiles/r05_s22_ab.txt)
template <int PF, class PT>  // PT: DPrim in any address space
__device__ __forceinline__ double prim_closest(const DScene &S, const PT &P, F3 o, F3 d, double minD, double maxD,
                                               bool transp, double lim) {
#if !defined(JSRT_NO_ANY_FILTER) && !defined(JSRT_NO_CLOSEST_FILTER)
    if constexpr (!(PF & PF_BVH)) {
        if (!transp && !P.casts_shadow) return DINF;  // Primitive.intersect (as prim_intersect)
        const int k = P.gkind;
        double t = 0;
        if (k == JSRT_GEOM_AABB) {
            const F3 lo = xf_point(P.inv, o), ld = xf_dir(P.inv, d);
            const int dec = box_closest_f32(P.center, P.half, lo, ld, box_ray(ld), minD, lim, t);
            if (dec >= 0) return dec ? t : -DINF;
            return aabb_intersect(P.center, P.half, lo, ld, minD, maxD);
        }
        if (k == JSRT_GEOM_SPHERE) {
            const F3 lo = xf_point(P.inv, o), ld = xf_dir(P.inv, d);
            const int dec = sphere_closest_f32(lo, ld, minD, lim, t);
            if (dec >= 0) return dec ? t : -DINF;
            return sphere_static(lo, ld, minD);
        }
    }
#endif
    return prim_intersect<PF>(S, P, o, d, minD, maxD, transp, lim);
}

// BVHAggregateNode.intersect with the BVH-local `ret` (aggregates.js:43-49, 207-225)
template <int PF, bool ANY>
__device__ __forceinline__ Hit bvh_cast(const DScene &S, const DInst &I, F3 o, F3 d, double minD, double maxD, bool transp) {
    Hit best{DINF, -1, I.ctx};
    const bool fast = I.count != 0;
    // Traversal stack in LDS, one column per lane ([entry * blockDim + lane]: lanes at the same depth
    // hit distinct banks): S.bvh_stack entries (deepest node + 2 >= the D + 1 a greater-first
    // traversal can hold) of the launch's dynamic LDS (bvh_lds_bytes).  A per-lane array would live
    // in scratch, and every push/pop would be a memory round trip on the traversal's critical path.
    extern __shared__ int bvh_lds_stack[];
    int *const stack = bvh_lds_stack + threadIdx.x;
    const int stride = (int)blockDim.x;
    const BoxRay br = box_ray(d);
    const float fmin_d = (float)minD;
    float flim = (float)maxD;  // (float)min(maxD, best)
    int sp = 0;
    stack[0] = I.first;
    ++sp;
    while (sp > 0) {
        --sp;
        const DBvhNode N = S.bvh[stack[sp * stride]];
#ifndef JSRT_NO_BOX_FILTER
        int en = box_enter_f32(N.cx, N.cy, N.cz, N.hx, N.hy, N.hz, o, br, fmin_d, flim);
#else
        int en = -1;
#endif
        if (en < 0) {
            double tmn, tmx;
            en = aabb_slab(N.cx, N.cy, N.cz, N.hx, N.hy, N.hz, o, d, minD, maxD, tmn, tmx) && tmn <= maxD &&
                 tmx >= minD && tmn <= best.t;
        }
        if (en) {
            if (N.b < 0) {
                const int cnt = ~N.b;
                for (int k = 0; k < cnt; ++k) {
                    double t;
                    if (fast) t = ANY ? tri_any(S.ltris[N.a + k], o, d, minD, maxD)  // leaf-ordered copy: no index load
                                      : tri_intersect(S.ltris[N.a + k], o, d);
                    else if (ANY) t = prim_any<PF>(S, S.prims[S.leaf_prims[N.a + k]], o, d, minD, maxD, transp);
                    else t = prim_intersect<PF>(S, S.prims[S.leaf_prims[N.a + k]], o, d, minD, maxD, transp, fmin(maxD, best.t));
                    if (t > minD && t < maxD && t < best.t) {
                        best.t = t;
                        best.prim = S.leaf_prims[N.a + k];
                        if (ANY) return best;
                        flim = (float)fmin(maxD, best.t);
                    }
                }
            } else {
                stack[sp * stride] = N.a;  // lesser, visited after the greater subtree
                stack[(sp + 1) * stride] = N.b;
                sp += 2;
            }
        }
    }
    return best;
}

// Aggregate / BVH instance below the top level (aggregates.js:14-18): members flattened in DFS
// order into the caller's running closest hit (equivalent to nested first-minimum selection).
template <int PF, bool ANY>
__device__ __forceinline__ void nested_cast(const DScene &S, int inst, F3 o, F3 d, double minD, double maxD, bool transp, Hit &best) {
    struct Fr {
        int inst, next;
        F3 o, d;
    };
    Fr st[8];
    int sp = 0;
    {
        const DInst &I = S.insts[inst];
        st[sp++] = Fr{inst, 0, xf_point(S.mats + 12 * I.matrix, o), xf_dir(S.mats + 12 * I.matrix, d)};
    }
    while (sp > 0) {
        Fr &f = st[sp - 1];
        const DInst &I = S.insts[f.inst];
        if (I.kind == INST_BVH) {
            const Hit h = bvh_cast<PF, ANY>(S, I, f.o, f.d, minD, maxD, transp);
            --sp;
            if (h.prim >= 0 && h.t > minD && h.t < best.t && h.t < maxD) {
                best = h;
                if (ANY) return;
            }
            continue;
        }
        if (f.next >= I.count) { --sp; continue; }
        const int c = S.inst_child[I.first + f.next++];
        const DInst &C = S.insts[c];
        if (C.kind == INST_PRIM) {
            const double t = ANY ? prim_any<PF>(S, S.prims[C.prim], f.o, f.d, minD, maxD, transp)
                                 : prim_intersect<PF>(S, S.prims[C.prim], f.o, f.d, minD, maxD, transp, fmin(maxD, best.t));
            if (t > minD && t < best.t && t < maxD) {
                best = Hit{t, C.prim, I.ctx};
                if (ANY) return;
            }
        } else if (sp < 8) {
            const double *m = S.mats + 12 * C.matrix;
            const F3 no = xf_point(m, f.o), nd = xf_dir(m, f.d);
            st[sp++] = Fr{c, 0, no, nd};
        }
    }
}

// Conservative cull of one top-level object: false only when the object provably
// cannot produce an accepted hit on the segment (minD, flim): the ray misses its world box inflated
// by k|o| + e0 (flim = (float) of the far limit min(best, maxD)).
template <class RBT>  // RootBound in any address space
__device__ __forceinline__ bool root_needed(const RBT &RB, F3 o, float ix, float iy, float iz, float oabs,
                                            float fminD, float flim) {
    if (!RB.bounded) return true;
    const float e = RB.k * oabs + RB.e0;
    float a0 = (RB.lo[0] - e - o.x) * ix, a1 = (RB.hi[0] + e - o.x) * ix;
    float tn = fminf(a0, a1), tf = fmaxf(a0, a1);
    a0 = (RB.lo[1] - e - o.y) * iy;
    a1 = (RB.hi[1] + e - o.y) * iy;
    tn = fmaxf(tn, fminf(a0, a1));
    tf = fminf(tf, fmaxf(a0, a1));
    a0 = (RB.lo[2] - e - o.z) * iz;
    a1 = (RB.hi[2] + e - o.z) * iz;
    tn = fmaxf(tn, fminf(a0, a1));
    tf = fminf(tf, fmaxf(a0, a1));
    return (tn <= tf) && (tf >= fminD) && (tn <= flim);
}

// World.cast (world.js:28-30); ANY = shadow query (only `0 < d < 1` of the closest is read,
// materials.js:250-252, so the first accepted hit decides).
//
// Culling: every top-level object carries a world-space box inflated by a margin
// >= 1e3 x the f32 rounding bound of any point the exact test can accept.  A lane skips an object
// when its ray segment (minD, min(best, maxD)) provably misses that box, and the wave skips the
// object when no lane needs it.  Skipped objects could not have produced an accepted hit, so the
// closest hit (first minimum in World.objects order) is unchanged bit for bit.
//
// mask (wave-uniform, shadow casts): bit i clear = root i (< 64) cannot produce an accepted hit on any lane's
// segment (scene_load.cpp shadow_grid), so the loop skips it without loading its record.
template <int PF, bool ANY>
__device__ __forceinline__ Hit world_cast(const DScene &S, F3 o, F3 d, double minD, double maxD, bool transp,
                                          uint64_t mask = ~0ull) {
    Hit best{DINF, -1, 0};
    const float ix = __builtin_amdgcn_rcpf(d.x), iy = __builtin_amdgcn_rcpf(d.y), iz = __builtin_amdgcn_rcpf(d.z);
    const float oabs = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    const float fminD = (float)minD;
    bool live = true;
    float flim = (float)maxD;  // (float)min(best, maxD): the cull's far limit, updated with best
    for (int i = 0; i < S.n_roots; ++i) {
        if (i < 64 && !((mask >> i) & 1ull)) continue;
        // the record of a wave-uniform root through the constant address space: scalar loads into SGPRs
        // (a generic pointer gets a vector load per field, each waited for on the loop's critical path)
        const auto &R = as_const(S.rootrec)[i];
        const bool need = live && root_needed(R.rb, o, ix, iy, iz, oabs, fminD, flim);
        if (!__any(need)) continue;
#ifdef JSRT_X_CULLONLY  // (timing experiment only) any-hit casts run the culls but no test: nothing accepted
        if (ANY) continue;
#endif
        if (!need) {  // (a divergent if, not a divergent continue: the loop itself stays uniform)
        } else if (R.kind == INST_PRIM) {
            // Primitive.intersect: Infinity for a non-shadow-casting primitive in a shadow cast
            if (transp || R.p.casts_shadow) {
                const double t = ANY ? prim_any<PF>(S, R.p, o, d, minD, maxD, transp)
                                     : prim_closest<PF>(S, R.p, o, d, minD, maxD, transp, fmin(maxD, best.t));
                if (t > minD && t < best.t && t < maxD) {
                    best = Hit{t, R.prim, 0};
                    flim = (float)best.t;
                    if (ANY) live = false;
                }
            }
        } else if ((PF & PF_BVH) && R.kind == INST_BVH) {
            const auto *m = R.p.inv;
            const Hit h = bvh_cast<PF, ANY>(S, S.insts[R.inst], xf_point(m, o), xf_dir(m, d), minD, maxD, transp);
            if (h.prim >= 0 && h.t > minD && h.t < best.t && h.t < maxD) {
                best = h;
                flim = (float)best.t;
                if (ANY) live = false;
            }
        } else if (PF & PF_AGG) {
            nested_cast<PF, ANY>(S, R.inst, o, d, minD, maxD, transp, best);
            flim = (float)(best.t < maxD ? best.t : maxD);
            if (ANY && best.prim >= 0) live = false;
        }
    }
    return best;
}

// The flat shadow loop (DScene::sroot): World.cast(P, delta, 1e-4, 1, false) as materials.js:250-252 reads it --
// only whether some object accepts a hit in (minD, maxD) -- over the shadow-casting top-level Primitives of a
// flat scene, grouped by geometry class.  Same culls and same any-hit tests (prim_any) as world_cast, so the
// answer is the same bit for bit; only the visiting order differs, which an any-hit answer does not see.
// What it saves is the generic loop's scalar bookkeeping: one root there is a chain of dependent scalar loads
// and branches (bounded?, kind?, casts_shadow?, gkind?, then the matrix), each waited for on the wave's
// critical path.  Here a record's 40 dwords arrive in three loads issued together and waited for once, the
// class is a compile-time constant, and `mask` (over records, DScene::grid_smask) is walked by its set bits.
// Returns true when some record accepts a hit (the lane's sample is shadowed).
template <int C>
__device__ __forceinline__ bool sroot_class(const DScene &S, uint64_t m, F3 o, F3 d, double minD, double maxD,
                                            float ix, float iy, float iz, float oabs, bool &live) {
    typedef uint32_t u16v __attribute__((ext_vector_type(16)));
    typedef uint32_t u8v __attribute__((ext_vector_type(8)));
    const float fminD = (float)minD, flim = (float)maxD;
    while (m) {
        if (!__any(live)) break;
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        // the record in three loads issued together: [0, 16) inv 0..7, [16, 32) inv 8..11 + bounds, [32, 40)
        const CONST_AS uint32_t *w = reinterpret_cast<const CONST_AS uint32_t *>(as_const(S.sroot) + j);
        u16v a = *reinterpret_cast<const CONST_AS u16v *>(w);
        u16v b = *reinterpret_cast<const CONST_AS u16v *>(w + 16);
        u8v c = *reinterpret_cast<const CONST_AS u8v *>(w + 32);
        __asm__ volatile("" : "+s"(a), "+s"(b), "+s"(c));  // all three in flight before the first use
        double inv[12];
#pragma unroll
        for (int k = 0; k < 8; ++k) inv[k] = __hiloint2double((int)a[2 * k + 1], (int)a[2 * k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) inv[8 + k] = __hiloint2double((int)b[2 * k + 1], (int)b[2 * k]);
        RootBound rb;
        rb.lo[0] = __uint_as_float(b[8]);
        rb.lo[1] = __uint_as_float(b[9]);
        rb.lo[2] = __uint_as_float(b[10]);
        rb.k = __uint_as_float(b[11]);
        rb.hi[0] = __uint_as_float(b[12]);
        rb.hi[1] = __uint_as_float(b[13]);
        rb.hi[2] = __uint_as_float(b[14]);
        rb.e0 = __uint_as_float(b[15]);
        rb.bounded = (int32_t)c[7];
        const bool need = live && root_needed(rb, o, ix, iy, iz, oabs, fminD, flim);
        if (!__any(need)) continue;
        if (!need) continue;  // (a divergent if: the loop itself stays uniform)
        double t = 0;
        if constexpr (C == SR_BOX) {  // prim_any's AABB branch
            const float ce[3] = {__uint_as_float(c[0]), __uint_as_float(c[1]), __uint_as_float(c[2])};
            const float ha[3] = {__uint_as_float(c[4]), __uint_as_float(c[5]), __uint_as_float(c[6])};
            const F3 lo = xf_point(inv, o), ld = xf_dir(inv, d);
            const int dec = box_any_f32(ce, ha, lo, box_ray(ld), minD, maxD, t);
            if (dec < 0) t = aabb_intersect(ce, ha, lo, ld, minD, maxD);
            else if (!dec) t = -DINF;
        } else if constexpr (C == SR_PLANE || C == SR_SQUARE || C == SR_CIRCLE) {  // prim_any's planar branch
            const int k = C == SR_PLANE ? JSRT_GEOM_PLANE : C == SR_SQUARE ? JSRT_GEOM_SQUARE : JSRT_GEOM_CIRCLE;
            const int dec = planar_any_f32(k, inv, o, d, minD, maxD, t);
            if (dec < 0) t = planar_intersect(k, inv, o, d, minD, maxD);
            else if (!dec) t = -DINF;
        } else if constexpr (C == SR_SPHERE) {  // prim_any's Sphere branch
            const F3 lo = xf_point(inv, o), ld = xf_dir(inv, d);
            const int dec = sphere_any_f32(lo, ld, minD, maxD, t);
            if (dec < 0) t = sphere_static(lo, ld, minD);
            else if (!dec) t = -DINF;
        } else {  // any other geometry: prim_any on the primitive itself
            t = prim_any<PF_ANALYTIC>(S, S.prims[(int)c[3]], o, d, minD, maxD, false);
        }
        if (t > minD && t < maxD) live = false;  // accepted (world_cast: t > minD && t < best.t && t < maxD)
    }
    return false;
}

__device__ __forceinline__ bool shadow_cast_flat(const DScene &S, F3 o, F3 d, double minD, double maxD, uint64_t m) {
    const float ix = __builtin_amdgcn_rcpf(d.x), iy = __builtin_amdgcn_rcpf(d.y), iz = __builtin_amdgcn_rcpf(d.z);
    const float oabs = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    bool live = true;
    auto part = [&](int c) {  // the mask's bits of class c (records [sr_first[c], sr_first[c + 1]))
        const int a = S.sr_first[c], b = S.sr_first[c + 1];
        const uint64_t hi = b >= 64 ? ~0ull : ((1ull << b) - 1), lo = a >= 64 ? ~0ull : ((1ull << a) - 1);
        return m & hi & ~lo;
    };
    sroot_class<SR_BOX>(S, part(SR_BOX), o, d, minD, maxD, ix, iy, iz, oabs, live);
    sroot_class<SR_PLANE>(S, part(SR_PLANE), o, d, minD, maxD, ix, iy, iz, oabs, live);
    sroot_class<SR_SQUARE>(S, part(SR_SQUARE), o, d, minD, maxD, ix, iy, iz, oabs, live);
    sroot_class<SR_CIRCLE>(S, part(SR_CIRCLE), o, d, minD, maxD, ix, iy, iz, oabs, live);
    sroot_class<SR_SPHERE>(S, part(SR_SPHERE), o, d, minD, maxD, ix, iy, iz, oabs, live);
    sroot_class<SR_OTHER>(S, part(SR_OTHER), o, d, minD, maxD, ix, iy, iz, oabs, live);
    return !live;
}

// --------------------------------------------------------------------------------------------
// Persistent casts for SDF scenes (world.js:7-15 + sdf.js:12-40 with lane refill).
//
// A sphere-traced SDF takes anywhere from a few to max_samples steps per ray, so a wave that casts
// 64 rays together idles most lanes while its slowest ray marches (measured: 15 % VALU lane use on
// SDF_Menger).  Here each lane runs a resumable World.cast: it walks the top-level objects in
// World.objects order (culling and exact tests exactly as world_cast), suspends at an SDF
// primitive to march it, and every iteration of the kernel's loop performs ONE march step for all
// marching lanes together (one uniform SDF program, sdf_node_dist).  A lane whose cast finishes
// stores its hit and takes the next ray from a work counter (one atomic per wave and round).
// Objects are still visited in order with the same acceptance tests, so the closest hit (first
// minimum) is unchanged bit for bit.  Top level must be primitives only (all_roots_prims).
struct MarchState {
    F3 o, d;          // world ray
    F3 lo, ld;        // ray in the SDF primitive's frame
    double t, tmin, tmax, rdn;
    Hit best;
    float flim;
    int root;         // next top-level object to visit
    int steps, g, prim;
    bool marching;
};

// Advance a lane's cast through the top-level objects until it must march an SDF primitive
// (returns with m.marching) or the cast is complete (m.root == n_roots).
template <int PF, bool ANY>
__device__ __forceinline__ void march_advance(const DScene &S, MarchState &m, double minD, double maxD, bool transp) {
    const float ix = __builtin_amdgcn_rcpf(m.d.x), iy = __builtin_amdgcn_rcpf(m.d.y), iz = __builtin_amdgcn_rcpf(m.d.z);
    const float oabs = fmaxf(fabsf(m.o.x), fmaxf(fabsf(m.o.y), fabsf(m.o.z)));
    const float fminD = (float)minD;
    while (m.root < S.n_roots) {
        const DRoot &R = S.rootrec[m.root++];
        if (!root_needed(R.rb, m.o, ix, iy, iz, oabs, fminD, m.flim)) continue;
        const DPrim &P = R.p;
        if ((PF & PF_SDF) && P.gkind == JSRT_GEOM_SDF) {  // Primitive.intersect -> SDFGeometry.intersect
            if (!transp && !P.casts_shadow) continue;   // Infinity: never accepted
            const F3 lo = xf_point(P.inv, m.o), ld = xf_dir(P.inv, m.d);
            const jsrt_rec_sdfgeom &G = S.sdfg[P.gindex];
            double bmin, bmax;
            if (!aabb_slab(G.center[0], G.center[1], G.center[2], G.half[0], G.half[1], G.half[2], lo, ld, minD, maxD,
                           bmin, bmax))
                continue;
            if (G.max_samples <= 0) continue;
            m.lo = lo;
            m.ld = ld;
            m.tmin = js_max(minD, bmin);
            m.tmax = js_min(maxD, bmax);
            m.t = m.tmin;
            m.rdn = sqrt(dot3(ld, ld));
            m.steps = 0;
            m.g = P.gindex;
            m.prim = R.prim;
            m.marching = true;
            return;
        }
        const double t = prim_intersect<PF>(S, P, m.o, m.d, minD, maxD, transp, fmin(maxD, m.best.t));
        if (t > minD && t < m.best.t && t < maxD) {
            m.best = Hit{t, R.prim, 0};
            m.flim = (float)m.best.t;
            if (ANY) m.root = S.n_roots;
        }
    }
}

// One sphere-tracing step of a marching lane (the body of sdf_intersect's loop).
template <bool ANY, bool FO>
__device__ __forceinline__ void march_step(const DScene &S, MarchState &m, double minD, double maxD) {
    const jsrt_rec_sdfgeom &G = S.sdfg[m.g];
    const F3 p = ray_point(m.lo, m.ld, m.t);
    const double distance = FO ? sdf_form_dist(S, G.root, p) : sdf_node_dist(S, G.root, p);
    bool end = false, hit = false;
    if (!__builtin_isfinite(distance)) end = true;
    else if (distance <= G.eps) end = hit = true;
    else {
        m.t += distance / m.rdn;
        if (m.t < m.tmin || m.t > m.tmax || (m.t - m.tmin) * m.rdn > G.max_trace || ++m.steps >= G.max_samples)
            end = true;
    }
    if (!end) return;
    m.marching = false;
    if (hit && m.t > minD && m.t < m.best.t && m.t < maxD) {
        m.best = Hit{m.t, m.prim, 0};
        m.flim = (float)m.best.t;
        if (ANY) m.root = S.n_roots;
    }
}

// The persistent loop.  Src: bool load(uint32_t job, F3 &o, F3 &d) (false: no ray in that slot),
// void store(uint32_t job, const Hit &h).  Jobs [0, count) are taken from *ctr.  FO: every SDF root
// of the scene is a recognised form (sdf_form_dist), no stack VM.
#ifndef JSRT_MARCH_STEPS
#define JSRT_MARCH_STEPS 8
#endif
#ifndef JSRT_MARCH_KEEP  // closest-hit marches (k_extend_q)
#define JSRT_MARCH_KEEP 48
#endif
#ifndef JSRT_MARCH_KEEP_ANY  // shadow marches (k_shadow_cast)
#define JSRT_MARCH_KEEP_ANY 36
#endif
template <int PF, bool ANY, bool FO, class Src>
__device__ __forceinline__ void persistent_cast(const DScene &S, uint32_t *ctr, uint32_t count, double minD,
                                                double maxD, bool transp, Src &src) {
    MarchState m;
    m.marching = false;
    bool have = false, drained = false;
    uint32_t job = 0;
    const int lane = (int)__lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (;;) {
        const bool want = !have && !drained;
        const uint64_t wb = __ballot(want);
        if (wb) {
            const int leader = __builtin_ctzll(wb);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(wb));
            base = __shfl(base, leader);
            if (want) {
                job = base + (uint32_t)__popcll(wb & lt);
                if (job >= count) drained = true;
                else if (src.load(job, m.o, m.d)) {
                    have = true;
                    m.best = Hit{DINF, -1, 0};
                    m.flim = (float)maxD;
                    m.root = 0;
                    m.marching = false;
                }
            }
        }
        if (!__any(have || !drained)) break;
        if (have && !m.marching) {
            march_advance<PF, ANY>(S, m, minD, maxD, transp);
            if (!m.marching) {
                src.store(job, m.best);
                have = false;
            }
        }
        // up to JSRT_MARCH_STEPS march steps per refill round while at least JSRT_MARCH_KEEP lanes still march:
        // the refill (ballot, atomic, ray loads) and the root walk of the lanes that finished run once per
        // round instead of once per step, at the price of a finished lane idling for the rest of its round
        // (SDF_Menger: 1 step 118.8 M/s, 2 steps 150.7 / 147.6, 4 steps 127.6, 8 steps 99.1; up to 8 steps while
        // >= 56 lanes march 151.7, >= 48 149.4; profiles/r04_s13_ab.txt, r04_s14_ab.txt.  Round 6, with the
        // evaluation ~1.5x cheaper, the refill costs relatively more: keep 56 / 48 / 40 / 32 / 24 read 225.8 / 239.1 /
        // 239.3 / 232.7 / 223.3 M/s, the closest-hit march best at 48 (k_extend_q 75.0 ms) and the shadow march at
        // 32-40 (k_shadow_cast 40.3 ms); profiles/r06_s19_march_knobs_menger.txt, r06_s20_march_keep_menger.txt)
        if (__any(have && m.marching)) {
#pragma unroll 1
            for (int k = 0; k < JSRT_MARCH_STEPS; ++k) {
                if (have && m.marching) march_step<ANY, FO>(S, m, minD, maxD);
                const uint64_t mb = __ballot(have && m.marching);
                if (!mb || (k > 0 && __popcll(mb) < (ANY ? JSRT_MARCH_KEEP_ANY : JSRT_MARCH_KEEP))) break;
            }
        }
    }
}

// --------------------------------------------------------------------------------------------
// materials (materials.js)
__device__ __forceinline__ F3 mc_eval(const DScene &S, int m, float u, float v) {  // MaterialColor.color(data)
    {  // a chain that does not read (u, v): its colour, computed by the loader (scene_load.cpp mc_constants)
        const float4 cc = *reinterpret_cast<const float4 *>(S.mc_const + 4 * m);
        if (cc.w != 0.0f) return f3(cc.x, cc.y, cc.z);
    }
    // walk Scaled* wrappers (and checkerboard choices) down to the solid colour, then apply the
    // scales innermost first: ScaledMaterialColor.color = child.color(data).times(scale)
    auto step = [&](int x) {  // next record below x (checkerboards resolved by (u, v))
        const jsrt_rec_mcolor &M = S.mc[x];
        if (M.kind == JSRT_MC_CHECKER) {  // materials.js:72-75
            // Math.fmod(a, 2) % 2 < 1 for a = floor(u) + floor(v): a is integral (or +-inf/NaN), so
            // a - floor(a / 2) * 2 is exactly 0, 1 or NaN, on which toPrecision(8) and % 2 are the identity
            const double a = floor((double)u) + floor((double)v);
            const double r = a - floor(a / 2) * 2;
            return (r < 1) ? M.a : M.b;
        }
        return M.a;
    };
    int n = 0, x = m;  // n = number of Scaled wrappers on the way down
    for (int g = 0; g < 16; ++g) {
        const int k = S.mc[x].kind;
        if (k == JSRT_MC_SOLID) break;
        if (k != JSRT_MC_CHECKER) ++n;
        x = step(x);
    }
    const jsrt_rec_mcolor &B = S.mc[x];
    F3 c = f3(B.vec[0], B.vec[1], B.vec[2]);
    for (int i = n - 1; i >= 0; --i) {  // the i-th wrapper from the top (usually n <= 1)
        int y = m, seen = 0;
        for (int g = 0; g < 16; ++g) {
            const int k = S.mc[y].kind;
            if (k != JSRT_MC_CHECKER) {
                if (seen == i) break;
                ++seen;
            }
            y = step(y);
        }
        const jsrt_rec_mcolor &M = S.mc[y];
        if (M.kind == JSRT_MC_SCALED_SCALAR) c = scale(c, M.scalar);
        else c = mul(c, f3(M.vec[0], M.vec[1], M.vec[2]));
    }
    return c;
}

struct Child {
    F3 dir, col, w;
    double k;
};

struct ShadeData {    // material_data after getBaseFactors (materials.js:210-238, 302-308)
    F3 pos, V, N, R, refr, ambient, diff, spec, refl, trans;
    double vdotn, kr, smoothness;
    bool backside, has_refr;
};

// PhongMaterial.colorFromLightSample / FresnelPhongMaterial.colorFromLightSample
// L = the sample direction normalised (light_sample computes it once for both uses).
// spec_zero: the specular colour is (+0, +0, +0), the smoothness in [0, 1e5] and R finite (the loader's
// MATF_SPEC_ZERO and k_shade's check).  Then every specular power the reference would compute is finite
// (its base is a dot of two unit f32 vectors, at most 1 + 3e-7), spec.times(specular) is +0 and the
// specular term is lcol * +0 whatever its value: the power is skipped.  Its one other effect, a NaN from a
// NaN L, is kept: for Phong, L.dot(R) is NaN exactly when L.dot(N) is (R and N finite), and a NaN L.dot(N)
// already makes the diffuse term NaN; the Fresnel terms are guarded by ldotn comparisons a NaN fails.
__device__ __forceinline__ F3 light_sample_color(int mkind, const ShadeData &d, F3 L, F3 lcol, bool spec_zero = false) {
    double diffuse, specular;
    if (mkind == JSRT_MAT_PHONG) {  // materials.js:261-269
        const double ldotn = dot3(L, d.N);
        diffuse = js_max(ldotn, 0);
        specular = spec_zero ? (is_nan(ldotn) ? ldotn : 0.0) : js_pow(js_max(dot3(L, d.R), 0), d.smoothness);
    } else {  // materials.js:340-356
        const double ldotn = dot3(L, d.N);
        diffuse = 0;
        specular = 0;
        if (d.kr > 0 && ldotn >= 0) {
            diffuse += d.kr * ldotn;
            if (!spec_zero) specular += d.kr * js_pow(js_max(dot3(L, d.R), 0), d.smoothness);
        }
        if (d.kr < 1 && ldotn <= 0) {
            diffuse += (1 - d.kr) * -ldotn;
            if (!spec_zero) specular += (1 - d.kr) * js_pow(js_max(dot3(L, d.refr), 0), d.smoothness);
        }
    }
    return add(mul(lcol, scale(d.diff, diffuse)), mul(lcol, scale(d.spec, specular)));
}

// One sample of lights.js sampleIterator for `Lt` seen from world point P: the direction (delta, NOT
// normalised: the shadow ray's t in (1e-4, 1) spans the segment) and the sample colour.
// LT: DLight in any address space (a wave-uniform record is read through the constant one: scalar loads)
// SPH: the scene may have a sphere area light (DScene::sphere_lights); without one the spherePick and its
// fdlibm fallback are not compiled into the caller (k_shadow: never executed, they cost it 5 ms on cornell)
template <bool SPH = true, class LT, class RNG>
__device__ __forceinline__ void light_sample(const DScene &S, const LT &Lt, F3 P, RNG &rng, F3 &delta, F3 &L,
                                             F3 &lcol) {
    if (Lt.kind == JSRT_LIGHT_POINT) {  // SimplePointLight.sampleIterator (lights.js:45-53)
        delta = sub(f3(Lt.pos[0], Lt.pos[1], Lt.pos[2]), P);
        L = normalized(delta);
        float u = 0, v = 0;
        if (Lt.needs_uv) cart_to_sph(L, u, v);
        lcol = scale(mc_eval(S, Lt.color, u, v), 1 / (4 * JS_PI * dot3(delta, delta)));
    } else {  // RandomSampleAreaLight.sampleIterator (lights.js:80-92)
        F3 local;
        if (SPH && Lt.gkind == JSRT_GEOM_SPHERE) {  // Vec.spherePick().to4(1)
            local = sphere_pick(rng);
        } else {  // Square / Circle.sampleSurface (geometry.js:295-300, 326-331)
            const double a = rng.next() - 0.5;
            const double b = rng.next() - 0.5;
            local = f3((float)a, (float)b, 0.0f);
        }
        const auto *T = Lt.T;
        const F3 wpos = f3((float)((((double)local.x * T[0] + (double)local.y * T[1]) + (double)local.z * T[2]) + T[3]),
                           (float)((((double)local.x * T[4] + (double)local.y * T[5]) + (double)local.z * T[6]) + T[7]),
                           (float)((((double)local.x * T[8] + (double)local.y * T[9]) + (double)local.z * T[10]) + T[11]));
        delta = sub(wpos, P);
        F3 wn;
        float u, v;
        if (SPH && Lt.gkind == JSRT_GEOM_SPHERE) {  // Sphere.materialData: local.normalized() (w = 1 term included)
            const double nn = sqrt(dot3(local, local) + 1.0);
            F3 n = local;
            float nw = 1.0f;
            if (nn > 0.00001) { n = scale(local, 1 / nn); nw = (float)(1.0 * (1 / nn)); }
            cart_to_sph(n, u, v);
            const auto *Ti = Lt.Ti;  // inv_transform.transposed().times(n).to4(0).normalized()
            const float wx = (float)((((double)n.x * Ti[0] + (double)n.y * Ti[4]) + (double)n.z * Ti[8]) + (double)nw * Ti[12]);
            const float wy = (float)((((double)n.x * Ti[1] + (double)n.y * Ti[5]) + (double)n.z * Ti[9]) + (double)nw * Ti[13]);
            const float wz = (float)((((double)n.x * Ti[2] + (double)n.y * Ti[6]) + (double)n.z * Ti[10]) + (double)nw * Ti[14]);
            wn = normalized(f3(wx, or0(wy), or0(wz)));
        } else {
            wn = f3(Lt.wn[0], Lt.wn[1], Lt.wn[2]);
            u = local.x;
            v = local.y;
        }
        L = normalized(delta);
        const double sc = (1 / (4 * JS_PI * dot3(delta, delta))) * fabs(dot3(L, wn));
        lcol = scale(mc_eval(S, Lt.color, u, v), sc);
    }
}

// PhongPathTracingMaterial.scatter (materials.js:398-412)
// fix (out): 0, or 1 + the RNG call index of the diffuse pick's first draw when the pick was unstable
// (sphere_pick_fast): the caller recomputes the direction with sphere_pick_v8 before it is cast
__device__ __forceinline__ bool path_scatter(double mirror_prob, bool has_r, F3 R, F3 N, const ShadeData &d, Rng &rng,
                                             F3 &dir, F3 &col, uint32_t &fix, bool force) {
    fix = 0;
    if (rng.next() < mirror_prob) {
        dir = R;
        col = f3(1, 1, 1);
        return has_r;
    }
    const double dp = average3(d.diff), sp = average3(d.spec);
    const double probSum = dp + sp;
    if (probSum == 0) return false;
    if (rng.next() < (dp / probSum)) {  // scatterDiffuse: N.plus(Vec.spherePick().to4()).normalized()
        const uint32_t call = rng.calls;
        bool unstable;
        const F3 sp3 = sphere_pick_fast(rng, unstable);
        if (unstable || force) fix = call + 1;
        dir = normalized(add(N, sp3));
        col = scale(d.diff, 1 / JS_PI);
        return true;
    }
    dir = R;  // scatterSpecular: finite smoothness returns R (materials.js:444-445)
    col = d.spec;
    return has_r;
}


// --------------------------------------------------------------------------------------------
// Camera.getRayForPixel (cameras.js:29-34, 46-52)
__device__ __forceinline__ void camera_ray(const DCamera &C, double x, double y, Rng &rng, F3 &o, F3 &d) {
    const double *T = C.T;
    const F3 dir = f3((float)(x * C.tan_fov * C.aspect), (float)(y * C.tan_fov), -1.0f);
    o = f3((float)T[3], (float)T[7], (float)T[11]);
    d = f3((float)((((double)dir.x * T[0] + (double)dir.y * T[1]) + (double)dir.z * T[2]) + 0.0 * T[3]),
           (float)((((double)dir.x * T[4] + (double)dir.y * T[5]) + (double)dir.z * T[6]) + 0.0 * T[7]),
           (float)((((double)dir.x * T[8] + (double)dir.y * T[9]) + (double)dir.z * T[10]) + 0.0 * T[11]));
    if (C.kind == JSRT_CAMERA_DOF) {
        const double a = rng.next() * 2 * JS_PI, rr = sqrt(rng.next());  // Vec.circlePick (math.js:175-179)
        double sa, ca;
        sin_cos(a, sa, ca);
        const float cx = (float)(rr * ca), cy = (float)(rr * sa);
        const float sx = (float)((double)cx * C.sensor), sy = or0((float)((double)cy * C.sensor));
        const F3 off = f3((float)((((double)sx * T[0] + (double)sy * T[1]) + 0.0 * T[2]) + 0.0 * T[3]),
                          (float)((((double)sx * T[4] + (double)sy * T[5]) + 0.0 * T[6]) + 0.0 * T[7]),
                          (float)((((double)sx * T[8] + (double)sy * T[9]) + 0.0 * T[10]) + 0.0 * T[11]));
        o = add(o, off);
        d = normalized(sub(scale(d, C.focus), off));
    }
}

__device__ __forceinline__ uint32_t set_color_rgba(F3 c) {  // PixelBuffer.setColor (pixelbuffer.js:39-49)
    const float v[3] = {c.x, c.y, c.z};
    uint32_t out = 0xFF000000u;  // alpha: colour length 3 -> comp 1 -> 255
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double comp = js_min(js_max((double)v[k], 0), 1);
        const double r = js_round(255 * comp);
        const uint32_t b = (r != r) ? 0u : (uint32_t)r;
        out |= b << (8 * k);
    }
    return out;
}


}  // namespace jsrt
