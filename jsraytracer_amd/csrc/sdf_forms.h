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
//   [1] MINBOX a, b        d1 = Union(boxes)(P)                             sdf.js:83-85
//   [2] TPUSH              s = 1
//   [3] LOOP a             iterations
//   [4] XMATREP a, b, pad    Q = rep(M Q), s = s * (1 * (1 * k))            sdf.js:387-394, 433-435, 471-473
//   [5] MINBOX a, b          d = Union(boxes)(Q)
//   [6] MULSMIN              d1 = min(d1, d * s)                           sdf.js:354-356
//   [7] ENDLOOP  [8] TPOP  [9] POPP
template <class KT, class CT>
__device__ __forceinline__ double sdf_form_runion(const KT *K, const CT *code, int pc, F3 P) {
    const int u0 = uni(code[pc + 1].a), un0 = uni(code[pc + 1].b);
    const int iters = uni(code[pc + 3].a);
    const int xm = uni(code[pc + 4].a), xs = uni(code[pc + 4].b), xr = uni(code[pc + 4].pad);
    const int u1 = uni(code[pc + 5].a), un1 = uni(code[pc + 5].b);
    double d1 = sdf_minbox(K + u0, un0, P);
    double s = 1.0;
    F3 Q = P;
    for (int it = 0; it < iters; ++it) {
        Q = sdf_xrep(K + xr, xf_point(K + xm, Q));
        s = s * (1.0 * (1.0 * K[xs]));
        const double d = sdf_minbox(K + u1, un1, Q);
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
