// sdf_forms.h — straight-line device code for SDF program shapes the host recognises (scene_load.cpp
// match_sdf_forms), in place of the stack VM (device_common.h sdf_run).
//
// The VM dispatches every instruction through a wave-uniform switch and keeps its stacks in register
// files addressed by uniform indices (select chains): on SDF_Menger that is ~4 M scalar and ~1.2 M branch
// instructions per wave beside 6.2 M VALU (profiles/pmc_r02_s1_SDF_Menger).  A recognised shape runs the
// same IEEE operations in the same order as the VM would on its instructions, with the stack slots as
// named registers and the loop as a plain loop; the instructions are still read for their constants.
// Included by device_common.h inside namespace jsrt, after the VM's building blocks (sdf_box, sdf_xrep).
#pragma once

// SFORM_RUNION: RecursiveTransformUnion(Union(Box x n), Sequence(Matrix, Repetition), iterations)
// (sdf.js:349-357), the Menger sponge's hole pattern.  Fused program (pc: after the SOP_FORM marker):
//   [0] PUSHP
//   [1] MINBOX a, b, x     d1 = Union(boxes)(P)  (x: the Menger cross)     sdf.js:83-85
//   [2] TPUSH              s = 1
//   [3] LOOP a             iterations
//   [4] XMATREP a, b, pad    Q = rep(M Q), s = s * (1 * (1 * k))            sdf.js:387-394, 433-435, 471-473
//   [5] MINBOX a, b, x       d = Union(boxes)(Q)
//   [6] MULSMIN              d1 = min(d1, d * s)                           sdf.js:354-356
//   [7] ENDLOOP  [8] TPOP  [9] POPP
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_runion(const KT *K, const CT *code, int pc, F3 P) {
    const int u0 = uni(code[pc + 1].a), un0 = uni(code[pc + 1].b);
    const int iters = uni(code[pc + 3].a);
    const int xm = uni(code[pc + 4].a), xs = uni(code[pc + 4].b), xr = uni(code[pc + 4].pad);
    const int u1 = uni(code[pc + 5].a), un1 = uni(code[pc + 5].b);
    const bool x0 = uni(code[pc + 1].pad) != 0, x1 = uni(code[pc + 5].pad) != 0;  // the Menger cross (sdf_cross)
    double d1 = x0 ? sdf_cross(K + u0, P) : sdf_minbox(K + u0, un0, P);
    double s = 1.0;
    F3 Q = P;
    for (int it = 0; it < iters; ++it) {
        Q = sdf_xrep(K + xr, xf_point(K + xm, Q));
        s = s * (1.0 * (1.0 * K[xs]));
        const double d = x1 ? sdf_cross(K + u1, Q) : sdf_minbox(K + u1, un1, Q);
        d1 = js_min(d1, d * s);
    }
    return d1;
}

// SFORM_RUNION_DIFF: Difference(Box, <SFORM_RUNION>) -- the Menger sponge of tests/SDF_Menger/test.mjs:27-36:
//   [0] BOX a   d0 = BoxSDF(P) (sdf.js:276-279)   [1..10] SFORM_RUNION   [11] NEG  [12] MAX 2
//   max(d0, -d1) (DifferenceSDF, sdf.js:117-119; Math.max, sdf.js:99-101)
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_runion_diff(const KT *K, const CT *code, int pc, F3 P) {
    const double d0 = sdf_box(K + uni(code[pc].a), P);
    const double d1 = sdf_form_runion(K, code, pc + 1, P);
    return js_max(d0, -d1);
}

// SDFGeometry.materialData's four distances (sdf.js:41-47: at P and at P + step along each axis, every other
// coordinate + 0.0f) of an SFORM_RUNION_DIFF whose loop matrix is diagonal (marker b & 1, scene_load.cpp
// runion_flags) and whose unions are both the Menger cross (MINBOX pad).  With finite coordinates the matrix row i
// is x_i m_ii + 0.0 (the zero products and the +0 translation leave a non-zero product and turn a zero sum into
// +0, as the reference's sum does) and the repetition is per axis, so coordinate i's chain through the loop
// depends on coordinate i alone: the four points share it, and each axis runs two chains (the point's and the
// offset one) instead of four -- half the toPrecision(8) steps.  The boxes, the crosses and the min / max run per
// point as sdf_form_runion_diff runs them.  -0 and +0 give the same chain (every use is |x| or x + c).  Returns
// false (nothing written) unless every coordinate entering a matrix row is finite: the caller then evaluates
// the four points one by one.  ab: the box's and the union's distances at P, which DifferenceSDF.getMaterialData
// compares (sdf.js:117-125): the child nodes' own programs are the same box and SFORM_RUNION code.
template <class KT, class CT>
__device__ __forceinline__ bool sdf_form_normal4(const KT *K, const CT *code, int pc, F3 P, float step, double dd[4],
                                                 double ab[2]) {
    if (!(uni(code[pc].op) == SOP_FORM && uni(code[pc].a) == SFORM_RUNION_DIFF && (uni(code[pc].b) & 1) &&
          uni(code[pc + 3].pad) && uni(code[pc + 7].pad)))
        return false;
    const int r = pc + 2;  // the SFORM_RUNION at [r, r + 10): MINBOX r + 1, LOOP r + 3, XMATREP r + 4, MINBOX r + 5
    const int bx = uni(code[pc + 1].a), u0 = uni(code[r + 1].a), iters = uni(code[r + 3].a);
    const int xm = uni(code[r + 4].a), xs = uni(code[r + 4].b), xr = uni(code[r + 4].pad), u1 = uni(code[r + 5].a);
    float cx[2] = {P.x + 0.0f, P.x + step}, cy[2] = {P.y + 0.0f, P.y + step}, cz[2] = {P.z + 0.0f, P.z + step};
    double d0[4], d1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const F3 q = f3(cx[k == 1], cy[k == 2], cz[k == 3]);
        d0[k] = sdf_box(K + bx, q);
        d1[k] = sdf_cross(K + u0, q);
    }
    bool fin = true;
    double sc = 1.0;
    const double m0 = K[xm], m5 = K[xm + 5], m10 = K[xm + 10];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            fin = fin && fabsf(cx[j]) <= __FLT_MAX__ && fabsf(cy[j]) <= __FLT_MAX__ && fabsf(cz[j]) <= __FLT_MAX__;
            cx[j] = sdf_rep1(K + xr, 0, (float)((double)cx[j] * m0 + 0.0));
            cy[j] = or0(sdf_rep1(K + xr, 1, (float)((double)cy[j] * m5 + 0.0)));
            cz[j] = or0(sdf_rep1(K + xr, 2, (float)((double)cz[j] * m10 + 0.0)));
        }
        sc = sc * (1.0 * (1.0 * K[xs]));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double d = sdf_cross(K + u1, f3(cx[k == 1], cy[k == 2], cz[k == 3]));
            d1[k] = js_min(d1[k], d * sc);
        }
    }
    if (!fin) return false;
#pragma unroll
    for (int k = 0; k < 4; ++k) dd[k] = js_max(d0[k], -d1[k]);
    ab[0] = d0[0];  // the Difference's two operands at P: getMaterialData's choice (sdf_material's hint)
    ab[1] = d1[0];
    return true;
}

// One primitive of a form: BOX / SPHERE / TETRA at instruction `pc` (the VM's cases, sdf.js:232-234,
// 276-279, 305-308), the opcode read uniform.
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_prim(const KT *K, const CT *code, int pc, F3 P) {
    const int op = uni(code[pc].op), ia = uni(code[pc].a);
    if (op == SOP_BOX) return sdf_box(K + ia, P);
    if (op == SOP_SPHERE) {
        const F3 q = f3(P.x, or0(P.y), or0(P.z));
        return sqrt(dot3(q, q)) - K[ia];
    }
    return (js_max(fabs((double)P.x + (double)P.y) - (double)P.z, fabs((double)P.x - (double)P.y) + (double)P.z) - 1) /
           sqrt(3.0);
}

// SFORM_PAIR: TransformSDF(primitive, Matrix) twice, combined (sdf.js:83-85, 99-101, 117-119, 128-131,
// 330-333; SDF_Combinations).  Each operand is [0] PUSHP [1] TPUSH [2] XMAT a b [3] PRIM [4] MULS [5] TPOP
// [6] POPP: prim(M P) * (1 * k); the flags say which of the operands and the result the program negates
// and which combiner follows (MIN 2, MAX 2 or SMIN k at pc + cb).  The VM's operations in its order.
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_tprim(const KT *K, const CT *code, int pc, F3 P) {
    const int xa = uni(code[pc + 2].a), xb = uni(code[pc + 2].b);
    return sdf_form_prim(K, code, pc + 3, xf_point(K + xa, P)) * (1.0 * K[xb]);
}
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_pair(const KT *K, const CT *code, int pc, int flags, int off_b, F3 P) {
    double a = sdf_form_tprim(K, code, pc, P);
    if (flags & SPAIR_NEG_A) a = -a;
    double b = sdf_form_tprim(K, code, pc + off_b, P);
    if (flags & SPAIR_NEG_B) b = -b;
    const int cb = off_b + 7 + ((flags & SPAIR_NEG_B) ? 1 : 0);
    double r;
    if (flags & SPAIR_SMIN) {  // smoothMin (sdf.js:128-131)
        const double k = K[uni(code[pc + cb].a)];
        const double h = js_max(k - fabs(a - b), 0.0) / k;
        r = js_min(a, b) - h * h * h * k * (1.0 / 6.0);
    } else {
        r = (flags & SPAIR_MAX) ? js_max(a, b) : js_min(a, b);
    }
    return (flags & SPAIR_NEG_OUT) ? -r : r;
}

// SFORM_TXREC: TransformSDF(primitive, SDFRecursiveTransformer(Sequence(Matrix, Reflection x m), n)) --
// SDF_Sierpinski (tests/SDF_Sierpinski/test.mjs: a tetrahedron folded 10 times by a scaling and three
// reflections).  Program: [0] PUSHP [1] TPUSH [2] LOOP n [3] TPUSH [4] XMATS a b [5 .. 5+m) XREF [5+m]
// TPOP_MUL [6+m] ENDLOOP [7+m] PRIM [8+m] MULS [9+m] TPOP [10+m] POPP.  Per iteration P = M P, then each
// reflection (sdf.js:450-455: P - n * 2 (n.P - delta) when n.P - delta < 0), the iteration's scale
// 1 * (1 * k) multiplied into the outer one; the result prim(P) * scale.
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_txrec(const KT *K, const CT *code, int pc, int m, F3 P) {
    const int iters = uni(code[pc + 2].a);
    const int xa = uni(code[pc + 4].a), xb = uni(code[pc + 4].b);
    double s0 = 1.0;
    F3 Q = P;
    for (int it = 0; it < iters; ++it) {
        double s1 = 1.0;
        Q = xf_point(K + xa, Q);
        s1 = s1 * (1.0 * K[xb]);
        for (int j = 0; j < m; ++j) {
            const int ra = uni(code[pc + 5 + j].a);
            const F3 n = f3((float)K[ra], (float)K[ra + 1], (float)K[ra + 2]);
            const double dt = dot3(n, Q) - K[ra + 3];
            if (dt < 0) Q = sub(Q, scale(n, 2 * dt));
        }
        s0 = s0 * s1;
    }
    return sdf_form_prim(K, code, pc + 7 + m, Q) * s0;
}

// SFORM_TX1: TransformSDF(primitive, one Matrix or Repetition transformer) (sdf.js:330-333; SDF_SphereRepetition):
// [0] PUSHP [1] TPUSH [2] XMAT a b | XREP a [3] PRIM [4] MULS [5] TPOP [6] POPP.  XMAT: prim(M P) * (1 * k); XREP
// (sdf.js:471-473, the scale untouched): prim(rep(P)) * 1.
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_tx1(const KT *K, const CT *code, int pc, F3 P) {
    if (uni(code[pc + 2].op) == SOP_XMAT) return sdf_form_tprim(K, code, pc, P);
    return sdf_form_prim(K, code, pc + 3, sdf_xrep(K + uni(code[pc + 2].a), P)) * 1.0;
}

// Any recognised form at the marker pc (uniform): its straight-line code
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_any(const KT *K, const CT *code, int pc, F3 P) {
    const int form = uni(code[pc].a);
    if (form == SFORM_RUNION_DIFF) return sdf_form_runion_diff(K, code, pc + 1, P);
    if (form == SFORM_RUNION) return sdf_form_runion(K, code, pc + 1, P);
    if (form == SFORM_PAIR) return sdf_form_pair(K, code, pc + 1, uni(code[pc].b), uni(code[pc].pad), P);
    if (form == SFORM_TXREC) return sdf_form_txrec(K, code, pc + 1, uni(code[pc].b), P);
    if (form == SFORM_PRIM) return sdf_form_prim(K, code, pc + 1, P);
    return sdf_form_tx1(K, code, pc + 1, P);
}
