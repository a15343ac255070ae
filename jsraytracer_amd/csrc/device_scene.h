// device_scene.h — HBM layout of a loaded scene (built by scene_load.cpp from a JSRT blob).
//
// Everything the render kernel reads lives in ONE device allocation; DScene carries the device
// pointers by value as a kernel argument (scalar-cache loads).  Layout choices:
//   * top-level objects are walked in World.objects order by every lane together (wave-uniform
//     loop, world.js:7-15), so per-object records are read through the scalar path;
//   * BVH nodes are 32-byte records (center f32x3 | child/leaf word | half f32x3 | child/leaf word),
//     one 32-B sector per node visit, visited greater-child-first as aggregates.js:221-222;
//   * triangles are 96-byte records holding exactly the fields Triangle.intersect reads
//     (geometry.js:368-375: normal, delta, p0, v0, v1, d00/d01/d11/denom), shading-only data
//     (vertex normals, UVs) lives in a separate array touched once per hit.
#pragma once
#include <math.h>
#include <stdint.h>

#include <cmath>

#include "../../include/jsrt_scene.h"
#include "sdf_program.h"

namespace jsrt {

enum : int32_t { INST_PRIM = 1, INST_AGG = 2, INST_BVH = 3 };

// Kernel profiles: the render kernel is instantiated per feature set so that a scene without
// BVHs / aggregates / SDFs / triangles does not pay their register footprint.
enum : int32_t { PF_BVH = 1, PF_AGG = 2, PF_SDF = 4, PF_TRI = 8 };
enum : int32_t { PF_ANALYTIC = 0, PF_MESH = PF_BVH | PF_TRI, PF_SDF_ONLY = PF_SDF, PF_ALL = 15 };
#define PF_SDF_PROFILE PF_SDF

struct DPrim {           // world.js:104 Primitive
    double inv[12];      // inv_transform rows 0..2 (row 3 verified == 0,0,0,1 at load)
    int32_t gkind;       // JSRT_GEOM_*
    int32_t gindex;      // triangle / sdf-geometry index
    int32_t material;    // MATL index
    int32_t casts_shadow;
    float center[4];     // AABB geometry (geometry.js:77)
    float half[4];
};
static_assert(sizeof(DPrim) == 144, "DPrim");

struct DInst {           // one node of the object tree flattened per path (shared DAG nodes duplicated)
    int32_t kind;        // INST_*
    int32_t prim;        // INST_PRIM: DPrim index
    int32_t first;       // INST_AGG: first child in inst_child[]; INST_BVH: root node
    int32_t count;       // INST_AGG: child count; INST_BVH: 1 if every leaf object is an identity-
                         //           transform, shadow-casting triangle Primitive (fast leaf path)
    int32_t matrix;      // AGG/BVH: index of the object's inverse matrix in mats[] (12 doubles)
    int32_t ctx;         // AGG/BVH: shading context id of everything below it
    int32_t pad[2];
};

struct RootBound {       // conservative world-space bound of one top-level object (culling only)
    float lo[3];
    float k;             // margin per unit of |ray origin|_inf
    float hi[3];
    float e0;            // constant margin
    int32_t bounded;     // 0: unbounded (Plane, ...) -> never culled
    int32_t pad[3];
};
static_assert(sizeof(RootBound) == 48, "RootBound");

struct DRoot {           // one top-level object flattened for the world loop: every field the cull
    RootBound rb;        // and the test read sits in one record, read through independent scalar loads
    int32_t kind;        // INST_*
    int32_t inst;        // DInst index
    int32_t prim;        // INST_PRIM: DPrim index (p is its copy); else -1
    int32_t pad;
    DPrim p;             // INST_PRIM: the primitive; AGG/BVH: p.inv = the object's inverse matrix
};
static_assert(sizeof(DRoot) == 208, "DRoot");

// One shadow-casting top-level Primitive as the flat shadow loop reads it (render_levels.h shadow_cast_flat):
// every field the cull and the any-hit test read, in one 160-B record fetched by three scalar loads issued
// together (DRoot spreads them over a 208-B record whose fields the generic loop loads one dependent branch
// at a time).  The records are grouped by geometry class (SR_*), so the loop over a class runs one test
// with no kind dispatch.  A shadow cast only asks whether SOME object accepts a hit in (1e-4, 1)
// (materials.js:250-252, world.js:7-15), so any visiting order gives the same answer.
enum : int32_t { SR_BOX, SR_PLANE, SR_SQUARE, SR_CIRCLE, SR_SPHERE, SR_OTHER, SR_N };
struct SRoot {
    double inv[12];      // the primitive's inv_transform rows 0..2 (DPrim::inv)
    float lo[3], k;      // RootBound
    float hi[3], e0;
    float center[3];     // AABB geometry (DPrim::center / half)
    int32_t prim;        // DPrim index
    float half[3];
    int32_t bounded;     // RootBound::bounded
};
static_assert(sizeof(SRoot) == 160, "SRoot");

struct DBvhNode {        // aggregates.js:187-202 BVHAggregateNode
    float cx, cy, cz;
    int32_t a;           // internal: lesser child; leaf: first index into leaf_prims[]
    float hx, hy, hz;
    int32_t b;           // internal: greater child (>= 0); leaf: ~count (< 0)
};
static_assert(sizeof(DBvhNode) == 32, "DBvhNode");

struct DTri {            // geometry.js:334-354 Triangle (intersection fields)
    float n[3];          // this.normal (w = 0)
    float p0[3];         // ps[0] xyz (w = 1)
    float v0[3], v1[3];  // ps[1]-ps[0], ps[2]-ps[0] (to3)
    double delta, d00, d11, d01, denom;
    int32_t prim;        // owning DPrim (for shading / materials)
    int32_t shade;       // index into DTriShade or -1
};
static_assert(sizeof(DTri) == 96, "DTri");

struct DTriShade {       // Triangle.psdata (objloader.js:198-201): vertex normals / UVs
    float vn[3][4];
    float uv[3][4];
    int32_t has_normal, has_uv, uv_len, pad;
};

struct DLight {          // lights.js:27 / :56
    int32_t kind, color, gkind, samples;
    float pos[3];        // point light position (xyz)
    int32_t pos_len;
    float wn[4];         // area light over a plane-like surface: world normal, precomputed exactly
    int32_t needs_uv;    // colour depends on UV (a checkerboard in its MaterialColor chain)
    int32_t pad2[3];
    double T[16], Ti[16];
    double inv_n;        // 1 / (samples of an area light, 1 for a point light): colorFromLights' weight
    double pad3;
};

struct DCamera {         // cameras.js:18-53
    double T[16];
    double tan_fov, aspect, focus, sensor;
    int32_t kind, pad[3];
};

// material flags: MATF_UV colours depend on (u, v) (a checkerboard in some chain); MATF_DIFF_CONST /
// MATF_SPEC_CONST the diffuse / specular chain is a constant (mc_const); MATF_SPEC_ZERO the specular colour
// is the constant (+0, +0, +0) and the smoothness in [0, 1e5] (render_levels.h: no specular power)
enum { MATF_UV = 1, MATF_DIFF_CONST = 2, MATF_SPEC_CONST = 4, MATF_SPEC_ZERO = 8 };

struct DScene {
    const DPrim *prims;
    const DInst *insts;
    const int32_t *inst_child;
    const int32_t *roots;
    const RootBound *rbounds;   // parallel to roots
    const DRoot *rootrec;       // parallel to roots (world_cast)
    const double *mats;      // 12 doubles per AGG/BVH instance matrix
    const double *ctx;       // 16 doubles per shading context (ctx 0 = identity)
    const DBvhNode *bvh;
    const int32_t *leaf_prims;   // DPrim indices (generic leaves)
    const int32_t *leaf_tris;    // DTri indices (fast leaves), parallel to leaf_prims
    const DTri *tris;
    const DTriShade *trish;
    const jsrt_rec_material *mat;
    const int32_t *mat_flags;    // MATF_* per material
    const int32_t *prim_shade;   // per prim: -1 identity inv_transform, else its slot in shade0
    const double *shade0;        // 16 per slot: prim.inv x identity (the ctx-0 shading matrix)
    const double *shadeI;        // 16 per ctx: identity x ctx (shading matrix of identity prims)
    const jsrt_rec_mcolor *mc;
    const float *mc_const;       // 4 per mc record: xyz its colour when UV-independent (w = 1)
    const DLight *lights;
    const SdfInsn *sdf_insn;     // SDF programs (sdf_program.h)
    const double *sdf_const;
    const int32_t *sdf_range;    // [2*node]: code range of SDF node `node`
    const int32_t *sdf_child;    // child lists of SDF union/intersection nodes (blob CHLD)
    const jsrt_rec_sdfnode *sdf_nodes;
    const jsrt_rec_sdfgeom *sdfg;
    int32_t n_roots, n_lights, n_prims, n_insts;
    DCamera cam;
    float bg[4];
    int32_t all_roots_prims; // every root is an INST_PRIM (uniform fast path)
    int32_t profile;         // PF_* feature set the kernel is instantiated for
    const int32_t *sample_light;  // per light sample s of a node (lights in order): its light
    const int32_t *sample_call;   // ... and the RNG call index of its first draw
    int32_t light_draws;     // RNG draws of all light samples of a node (scatter draws follow)
    int32_t max_children;    // most children one ray-tree node can spawn (0..2)
    int32_t bvh_stack;       // LDS traversal-stack entries per lane (deepest BVH node + 2; 0: no BVH)
    const DTri *ltris;       // parallel to leaf_prims: the triangle of a fast leaf entry (leaf order)
    const int32_t *prim_lit; // per prim: 1 if its material takes light samples (not Solid / Transparent)
    int32_t sdf_all_forms;   // every SDF geometry root is a recognised program form (sdf_forms.h)
    int32_t sphere_lights;   // an area light samples a Sphere (spherePick in k_shadow; its kernel variant)
    // Spatial buckets of the shadow hand-off (scene_load.cpp shadow_grid): hit points binned on a grid of
    // grid_cells <= 63 cells over the bounded top-level objects (bucket grid_cells: outside the grid), and
    // per bucket the top-level objects a shadow segment from that cell to any light can meet
    // (grid_mask[b] bit i: root i; the outside bucket holds every root).  grid_masked: n_roots <= 64.
    const uint64_t *grid_mask;   // grid_cells + 1 entries
    float grid_lo[3], grid_inv[3];
    int32_t grid_dim[3], grid_cells, grid_masked, pad_grid;
    // The per-hit tables of k_shade and k_shadow packed into one image of stab_words 16-B words (0: too big for
    // LDS), table k at byte offset stab_off[k] (STAB_*).  k_shade copies all of it into LDS and k_shadow the
    // prefix of its own tables (stab_words_shadow words), so a hit's dependent record chain (prim -> matrix /
    // material -> colour constants) is LDS round trips instead of L2 ones (render_levels.h k_shade, k_shadow).
    const void *stab;            // 16-B aligned
    int32_t stab_words, stab_words_shadow;
    int32_t stab_off[12];
    // The flat shadow loop (all roots Primitives, at most 64; n_sroot = 0: not built): the shadow-casting roots
    // as SRoot records grouped by class, class c at [sr_first[c], sr_first[c + 1]); grid_smask[b] = grid_mask[b]
    // over these records (bit j: record j).
    const SRoot *sroot;
    const uint64_t *grid_smask;  // grid_cells + 1 entries
    int32_t n_sroot, pad_sroot;
    int32_t sr_first[SR_N + 1 + 1];
};
enum {  // DScene::stab tables, in image order: k_shadow's first (mat .. sample_light), then k_shade's
    STAB_MAT, STAB_MAT_FLAGS, STAB_MC, STAB_MC_CONST, STAB_SAMPLE_CALL, STAB_SAMPLE_LIGHT,
    STAB_PRIMS, STAB_PRIM_SHADE, STAB_SHADE0, STAB_SHADEI, STAB_PRIM_LIT, STAB_N
};
constexpr int STAB_MAX_WORDS = 1024;  // 16 KB of LDS at most

// Dynamic LDS of a casting kernel over a scene with BVHs: per lane a traversal stack of bvh_stack
// 4-byte entries (device_common.h bvh_cast).
inline size_t bvh_lds_bytes(const DScene &S, int block) { return (size_t)S.bvh_stack * block * 4; }

}  // namespace jsrt
