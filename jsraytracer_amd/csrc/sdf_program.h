// sdf_program.h — SDF trees (sdf.js:53-477) compiled to a small stack program.
//
// The reference evaluates SDFs by recursive virtual calls (SDF.distance / SDFTransformer.transform).
// On the GPU every lane of a wave marches the same SDF, so the tree is compiled once at scene load
// into a linear program whose instruction stream is wave-uniform; per-lane state is the current
// point P (f32 xyz, w == 1 everywhere on this path), a float64 distance stack and a float64 scale
// stack that reproduces the reference's nesting of `s = s * st` products exactly.
//
// Each SDF node compiles to a contiguous range [start, end) that pushes exactly one distance and
// leaves P unchanged, so getMaterialData (sdf.js:87,103,120,...) can evaluate any child by range.
#pragma once
#include <stdint.h>

namespace jsrt {

enum SdfOp : int32_t {
    SOP_END = 0,
    SOP_BOX,        // a = const index of size (4 doubles: f32 size xyz, as double)   sdf.js:276-279
    SOP_SPHERE,     // a = const index of radius                                       sdf.js:232-234
    SOP_TETRA,      //                                                                 sdf.js:305-308
    SOP_MIN,        // a = n: pop n, push Math.min(...)                                sdf.js:83-85
    SOP_MAX,        // a = n: pop n, push Math.max(...)                                sdf.js:99-101
    SOP_NEG,        // d = -d
    SOP_SUBK,       // a = const: d = d - k                                            sdf.js:210-212
    SOP_SMIN,       // a = const k: pop b, pop a, push smoothMin(a, b, k)              sdf.js:128-131
    SOP_PUSHP,      // save P
    SOP_POPP,       // restore P
    SOP_TPUSH,      // push scale 1
    SOP_TPOP,       // drop scale
    SOP_TPOP_MUL,   // st = pop; top = top * st
    SOP_MULS,       // d = d * top-scale
    SOP_XMAT,       // a = const index of 12 doubles (inv rows 0..2), b = const of scale:
                    //   P = inv*P, top = top * scale                                   sdf.js:433-435
    SOP_XREF,       // a = const: normal xyz (f32 as double) + delta                    sdf.js:450-455
    SOP_XREP,       // a = const: sizes xyz, then 1/size (exact) or 0 per axis          sdf.js:471-473
    SOP_LOOP,       // a = iterations, b = index of the matching SOP_ENDLOOP
    SOP_ENDLOOP,    // a = index of the matching SOP_LOOP
    // fused forms (scene_load.cpp fuse_sdf: the same operations in the same order, one dispatch)
    SOP_MINBOX,     // BOX x b, MIN b: a = const of the first box (boxes 4 doubles apart)
    SOP_XMATS,      // TPUSH XMAT TPOP_MUL: P = inv*P, top = top * (1 * scale)
    SOP_XMATREP,    // TPUSH XMATS XREP TPOP_MUL: a = matrix, b = scale, pad = repetition const
    SOP_MULSMIN,    // MULS, MIN 2: d = pop * top-scale; push Math.min(pop, d)
    // a recognised program shape (scene_load.cpp match_sdf_forms): a = SFORM_*, the shape's fused
    // instructions follow and are run as straight-line code (sdf_forms.h)
    SOP_FORM,
};
enum SdfForm : int32_t {
    SFORM_RUNION_DIFF = 1,  // Difference(Box, RecursiveTransformUnion(Union(Box...), Sequence(Matrix, Repetition)))
    SFORM_RUNION = 2,       // RecursiveTransformUnion(Union(Box...), Sequence(Matrix, Repetition))
    SFORM_PAIR = 3,         // two Matrix-transformed primitives combined (Union / Intersection / Difference / Smooth*)
    SFORM_TXREC = 4,        // Transform(primitive, Recursive(Sequence(Matrix, Reflection...)))  (SDF_Sierpinski)
    SFORM_PRIM = 5,         // a bare primitive (SDF_Simple)
    SFORM_TX1 = 6,          // Transform(primitive, Matrix | Repetition)  (SDF_SphereRepetition)
};
// SFORM_PAIR flags (the form instruction's b; its pad = the second operand's offset after the marker)
enum : int32_t { SPAIR_NEG_A = 1, SPAIR_NEG_B = 2, SPAIR_NEG_OUT = 4, SPAIR_MAX = 8, SPAIR_SMIN = 16 };

struct SdfInsn {
    int32_t op, a, b, pad;
};

// Stack limits sized to the reference scenes (deepest: SDF_Menger d=5, Sierpinski s=3, one loop),
// small enough for the device VM to keep every stack in registers (the host rejects deeper trees).
constexpr int SDF_MAX_D = 6;    // distance stack depth
constexpr int SDF_MAX_P = 2;    // point stack depth
constexpr int SDF_MAX_S = 4;    // scale stack depth
constexpr int SDF_MAX_LOOP = 2; // nested loops

}  // namespace jsrt
