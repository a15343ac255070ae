// prim_filter.h — f32 interval pre-tests in front of the exact (f64) analytic-primitive intersections.
// Included by device_common.h inside its namespace jsrt (needs F3 and the exact functions above the
// include point).
//
// A caller of Primitive.intersect only ever asks one question: is the returned distance t accepted,
// minD < t < lim (world.js:10-13, aggregates.js:212-213, lim = min(maxD, best))?  These filters
// answer it from f32 arithmetic carrying an absolute error bound for every value the reference
// computes (local ray rows, plane distance, slab quotients, quadratic roots):
//   FLT_NO    the exact test provably rejects (miss, or t outside (minD, lim));
//   FLT_YES   the exact test provably accepts (t is not known exactly, only that it is accepted);
//   FLT_EXACT too close to call: run the exact test.
// A decision is taken only when the compared quantities are apart by more than their bounds, so the
// outcome is the reference's bit for bit.  Shadow casts (any-hit) stop at FLT_YES; closest-hit casts
// skip FLT_NO objects and run the exact test otherwise (they need the exact t).
//
// Error model.  A local row is evaluated as m_r . (o - T) + c_r, with T the primitive's world position
// (f32) and c_r the f64 residual m_r . T + m_r3 rounded to f32, so magnitudes are those of o - T, not
// of o and the translation separately.  Each bound is REL * (magnitudes) + TINY with REL = 2^-21:
// 8 units of 2^-24 against at most 7 roundings of that size (o - T; the coefficients and residual
// rounded to f32; three fma of partial sums bounded by the magnitude sum; the reference's final f32
// store; its f64 ops are 2^-51 of its own magnitudes, far below), and likewise for the derived values
// (rcp / sqrt approximations <= 1 ulp, each f32 op 2^-24).  TINY = 1e-30 covers underflow.  NaN or
// infinity anywhere makes every decisive comparison false, hence FLT_EXACT.
// tests/test_prim_filter.py checks the decisions against the exact functions on rays built to sit on
// every decision boundary.
#pragma once


enum : int { FLT_NO = 0, FLT_YES = 1, FLT_EXACT = -1 };

constexpr float FLT_REL = 4.76837158203125e-07f;  // 2^-21
constexpr float FLT_TINY = 1e-30f;

JSRT_HD float frcp(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
JSRT_HD float fsqrt(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}

struct FV {  // approximation v of a value the reference computes, |v - reference| <= e
    float v, e;
};

// The ray relative to the primitive: o - T and its max norm (shared by the rows of one primitive).
struct FRay {
    F3 o, d;       // o - T, d
    float q, dq;   // max |o_i - T_i|, max |d_i|
    float ea;      // absolute error term of the point rows
};
JSRT_HD FRay fray(const FRows &R, F3 o, F3 d, float oabs, float dabs) {
    const F3 u = f3(o.x - R.T[0], o.y - R.T[1], o.z - R.T[2]);
    return FRay{u, d, fmaxf(fabsf(u.x), fmaxf(fabsf(u.y), fabsf(u.z))), dabs, fmaf(oabs, R.ga, R.gb) + FLT_TINY};
}

// Row r of Mat x Vec as the reference rounds it (f64 dot in order, f32 store, math.js:392-397).
JSRT_HD FV frow_point(const FRows &R, int r, const FRay &Y) {
    const float *m = R.m + 3 * r;
    const float v = fmaf(Y.o.z, m[2], fmaf(Y.o.y, m[1], fmaf(Y.o.x, m[0], R.c[r])));
    return FV{v, FLT_REL * (fmaf(Y.q, R.rn[r], fabsf(R.c[r])) + fabsf(v)) + Y.ea};
}
JSRT_HD FV frow_dir(const FRows &R, int r, const FRay &Y) {
    const float *m = R.m + 3 * r;
    const float v = fmaf(Y.d.z, m[2], fmaf(Y.d.y, m[1], Y.d.x * m[0]));
    return FV{v, FLT_REL * (Y.dq * R.rn[r] + fabsf(v)) + FLT_TINY};
}

// The caller's bounds, with their slack: t > minD decided by lo > min_hi / hi < min_lo, t < lim by
// hi < lim_lo / lo > lim_hi (lim may be +inf; both are >= 0).
struct FBounds {
    float min_lo, min_hi, lim_lo, lim_hi, max_lo, max_hi;
};
JSRT_HD FBounds fbounds(double minD, double maxD, double lim) {
    const float a = (float)minD, b = (float)lim, c = (float)maxD;
    return FBounds{a * (1 - FLT_REL) - FLT_TINY, a * (1 + FLT_REL) + FLT_TINY, b * (1 - FLT_REL) - FLT_TINY,
                   b * (1 + FLT_REL) + FLT_TINY, c * (1 - FLT_REL) - FLT_TINY, c * (1 + FLT_REL) + FLT_TINY};
}

// decision on an accepted-distance interval [lo, hi]
JSRT_HD int faccept(float lo, float hi, const FBounds &B) {
    if (hi < B.min_lo || lo > B.lim_hi) return FLT_NO;
    if (lo > B.min_hi && hi < B.lim_lo) return FLT_YES;
    return FLT_EXACT;
}

// planar_intersect (SimplePlane / Square / Circle, geometry.js:246-248, 287-291, 310-314)
JSRT_HD int planar_filter(int k, const FRows &R, const FRay &Y, const FBounds &B) {
    const FV oz = frow_point(R, 2, Y), dz = frow_dir(R, 2, Y);
    const float adz = fabsf(dz.v) - dz.e;
    if (!(adz > 0.0f)) return FLT_EXACT;  // dz may be 0 (t = -inf) or of unknown sign
    // t = -oz / dz (f64 division of the f32 rows)
    // |t_ref - t| <= |oz_ref + t dz_ref| / |dz_ref| <= (e_oz + |t| (e_dz + rounding of t |dz|)) / (|dz| - e_dz)
    const float t = -oz.v * frcp(dz.v);
    const float et = (oz.e + fabsf(t) * (dz.e + FLT_REL * fabsf(dz.v))) * frcp(adz) * 1.001f + FLT_TINY;
    const int in = faccept(t - et, t + et, B);
    if (in != FLT_YES || k == JSRT_GEOM_PLANE) return in;
    // p = o + f32(d * t) in local space (Ray.getPoint); bound: |dp| <= e_o + (|d| + e_d) e_t + |t| e_d + roundings
    const FV ox = frow_point(R, 0, Y), oy = frow_point(R, 1, Y);
    const FV dx = frow_dir(R, 0, Y), dy = frow_dir(R, 1, Y);
    const float px = fmaf(dx.v, t, ox.v), py = fmaf(dy.v, t, oy.v);
    const float epx = ox.e + (fabsf(dx.v) + dx.e) * et + fabsf(t) * dx.e + FLT_REL * (fabsf(ox.v) + fabsf(dx.v * t) + fabsf(px)) + FLT_TINY;
    const float epy = oy.e + (fabsf(dy.v) + dy.e) * et + fabsf(t) * dy.e + FLT_REL * (fabsf(oy.v) + fabsf(dy.v * t) + fabsf(py)) + FLT_TINY;
    if (k == JSRT_GEOM_SQUARE) {  // -0.5 <= p.x, p.y <= 0.5
        if (fabsf(px) - epx > 0.5f || fabsf(py) - epy > 0.5f) return FLT_NO;
        if (fabsf(px) + epx < 0.5f && fabsf(py) + epy < 0.5f) return FLT_YES;
        return FLT_EXACT;
    }
    // Circle: dot3(p, p) <= 1 with p.z = oz + f32(dz * t)
    const float pz = fmaf(dz.v, t, oz.v);
    const float epz = oz.e + (fabsf(dz.v) + dz.e) * et + fabsf(t) * dz.e + FLT_REL * (fabsf(oz.v) + fabsf(dz.v * t) + fabsf(pz)) + FLT_TINY;
    const float q = fmaf(pz, pz, fmaf(py, py, px * px));
    const float eq = 2 * (fabsf(px) * epx + fabsf(py) * epy + fabsf(pz) * epz) + (epx * epx + epy * epy + epz * epz) +
                     FLT_REL * q + FLT_TINY;
    if (q - eq > 1.0f) return FLT_NO;
    if (q + eq < 1.0f) return FLT_YES;
    return FLT_EXACT;
}

// AABB.intersect (geometry.js:173-179, 189-209): the slab test, then t = tmin >= minD ? tmin : tmax
JSRT_HD int aabb_filter(const FRows &R, const float *c, const float *h, const FRay &Y, const FBounds &B) {
    constexpr float SKIP = 1e-7f;  // |d_i| > 0.0000001 (f64 compare of the f32 component)
    float tn_lo = -__builtin_inff(), tn_hi = -__builtin_inff(), tx_lo = __builtin_inff(), tx_hi = __builtin_inff();
    int used = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const FV oi = frow_point(R, i, Y), di = frow_dir(R, i, Y);
        const float p = c[i] - oi.v;  // Vec.minus: f32(c - o)
        const float ep = oi.e + FLT_REL * fabsf(p) + FLT_TINY;
        const float ad = fabsf(di.v);
        if (ad - di.e > SKIP * (1 + FLT_REL)) {
            const float r = frcp(di.v), adl = ad - di.e;
            const float a = (p + h[i]) * r, b = (p - h[i]) * r;
            // |(p_ref + h) / d_ref - a| <= (e_p + |a| (e_d + rounding of a |d|)) / (|d| - e_d)
            const float ea = (ep + fabsf(a) * (di.e + FLT_REL * ad)) * frcp(adl) * 1.001f + FLT_TINY;
            const float eb = (ep + fabsf(b) * (di.e + FLT_REL * ad)) * frcp(adl) * 1.001f + FLT_TINY;
            if (!(fabsf(a) + ea + fabsf(b) + eb < 1e38f)) return FLT_EXACT;  // overflow / NaN (fminf drops NaN)
            tn_lo = fmaxf(tn_lo, fminf(a - ea, b - eb));
            tn_hi = fmaxf(tn_hi, fminf(a + ea, b + eb));
            tx_lo = fminf(tx_lo, fmaxf(a - ea, b - eb));
            tx_hi = fminf(tx_hi, fmaxf(a + ea, b + eb));
            ++used;
        } else if (ad + di.e < SKIP * (1 - FLT_REL)) {  // skipped axis: false when |p| > h
            if (fabsf(p) - ep > h[i]) return FLT_NO;
            if (!(fabsf(p) + ep < h[i])) return FLT_EXACT;
        } else {
            return FLT_EXACT;
        }
    }
    if (used == 0) return FLT_EXACT;
    // slab fails: t_min > t_max || t_max < minD || t_min > maxD
    if (tn_lo > tx_hi || tx_hi < B.min_lo || tn_lo > B.max_hi) return FLT_NO;
    if (!(tn_hi < tx_lo && tx_lo > B.min_hi && tn_hi < B.max_lo)) return FLT_EXACT;
    if (tn_lo > B.min_hi) return faccept(tn_lo, tn_hi, B);  // t = t_min (>= minD)
    if (tn_hi < B.min_lo) return faccept(tx_lo, tx_hi, B);  // t = t_max
    return FLT_EXACT;
}

// Sphere.intersect (geometry.js:429-442, sphere_static): roots of |o + t d|^2 = 1,
// t = t2 >= minD ? t2 : t1 (t2 <= t1)
JSRT_HD int sphere_filter(const FRows &R, const FRay &Y, const FBounds &B) {
    const FV ox = frow_point(R, 0, Y), oy = frow_point(R, 1, Y), oz = frow_point(R, 2, Y);
    const FV dx = frow_dir(R, 0, Y), dy = frow_dir(R, 1, Y), dz = frow_dir(R, 2, Y);
    const float a = fmaf(dz.v, dz.v, fmaf(dy.v, dy.v, dx.v * dx.v));
    const float ea = (2 * (fabsf(dx.v) * dx.e + fabsf(dy.v) * dy.e + fabsf(dz.v) * dz.e) + dx.e * dx.e + dy.e * dy.e +
                      dz.e * dz.e) + FLT_REL * a + FLT_TINY;
    const float b = fmaf(dz.v, oz.v, fmaf(dy.v, oy.v, dx.v * ox.v));
    const float eb = (fabsf(dx.v) * ox.e + fabsf(ox.v) * dx.e + dx.e * ox.e) + (fabsf(dy.v) * oy.e + fabsf(oy.v) * dy.e + dy.e * oy.e) +
                     (fabsf(dz.v) * oz.e + fabsf(oz.v) * dz.e + dz.e * oz.e) +
                     FLT_REL * (fabsf(dx.v * ox.v) + fabsf(dy.v * oy.v) + fabsf(dz.v * oz.v)) + FLT_TINY;
    const float oo = fmaf(oz.v, oz.v, fmaf(oy.v, oy.v, ox.v * ox.v));
    const float c = oo - 1.0f;
    const float ec = (2 * (fabsf(ox.v) * ox.e + fabsf(oy.v) * oy.e + fabsf(oz.v) * oz.e) + ox.e * ox.e + oy.e * oy.e +
                      oz.e * oz.e) + FLT_REL * (oo + 1.0f) + FLT_TINY;
    if (!(a - ea > 0.0f)) return FLT_EXACT;  // a == 0 -> -inf in the reference
    const float big = b * b - a * c;
    const float ebig = (2 * fabsf(b) * eb + eb * eb + fabsf(a) * ec + fabsf(c) * ea + ea * ec +
                        FLT_REL * (b * b + fabsf(a * c))) * 1.001f + FLT_TINY;
    if (big + ebig < 0.0f) return FLT_NO;  // big < 0: no intersection
    if (!(big - ebig > 0.0f)) return FLT_EXACT;
    const float s_lo = fsqrt(big - ebig) * (1 - FLT_REL), s_hi = fsqrt(big + ebig) * (1 + FLT_REL);
    const float a_lo = a - ea, a_hi = a + ea;
    // t1 = (-b + s) / a, t2 = (-b - s) / a with a in [a_lo, a_hi] > 0
    const float n1_lo = -(b + eb) + s_lo, n1_hi = -(b - eb) + s_hi;
    const float n2_lo = -(b + eb) - s_hi, n2_hi = -(b - eb) - s_lo;
    const float ra_lo = frcp(a_hi) * (1 - FLT_REL), ra_hi = frcp(a_lo) * (1 + FLT_REL);  // 1/a in [ra_lo, ra_hi]
    auto div_lo = [&](float n) { return (n >= 0 ? n * ra_lo : n * ra_hi) * (n >= 0 ? 1 - FLT_REL : 1 + FLT_REL) - FLT_TINY; };
    auto div_hi = [&](float n) { return (n >= 0 ? n * ra_hi : n * ra_lo) * (n >= 0 ? 1 + FLT_REL : 1 - FLT_REL) + FLT_TINY; };
    const float t1_lo = div_lo(n1_lo), t1_hi = div_hi(n1_hi), t2_lo = div_lo(n2_lo), t2_hi = div_hi(n2_hi);
    if (t2_lo > B.min_hi) return faccept(t2_lo, t2_hi, B);  // t = t2
    if (t2_hi < B.min_lo) return faccept(t1_lo, t1_hi, B);  // t = t1
    return FLT_EXACT;
}

