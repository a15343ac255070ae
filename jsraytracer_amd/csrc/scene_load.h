// scene_load.h — host side: JSRT blob -> validated, flattened HostScene (then uploaded to HBM).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "device_scene.h"

namespace jsrt {

struct HostScene {
    std::vector<DPrim> prims;
    std::vector<int32_t> prim_obj;     // per DPrim: its OBJS index in the blob (jsrt_cast)
    std::vector<int32_t> prim_lit;     // per DPrim: its material takes light samples (DScene::prim_lit)
    std::vector<DInst> insts;
    std::vector<int32_t> inst_child, roots;
    std::vector<RootBound> rbounds;
    std::vector<DRoot> rootrec;
    std::vector<double> mats, ctx;
    std::vector<DBvhNode> bvh;
    std::vector<int32_t> leaf_prims, leaf_tris;
    std::vector<DTri> tris;
    std::vector<DTri> ltris;       // parallel to leaf_prims: tris[leaf_tris[i]] (zero record if none)
    std::vector<DTriShade> trish;
    std::vector<jsrt_rec_material> mat;
    std::vector<int32_t> mat_flags;    // MATF_* per material
    std::vector<int32_t> prim_shade;   // -1: identity inv_transform; else slot in shade0
    std::vector<double> shade0, shadeI;  // 16 per slot / per ctx: precomputed shading matrices
    std::vector<jsrt_rec_mcolor> mc;
    std::vector<float> mc_const;        // 4 per mc record: its colour when UV-independent (w = 1), else w = 0
    std::vector<DLight> lights;
    std::vector<int32_t> sample_light, sample_call;  // per light sample of a node
    int32_t light_draws = 0;
    std::vector<SdfInsn> sdf_insn;
    int32_t sdf_all_forms = 0;         // every SDF geometry root's program is a recognised form
    std::vector<double> sdf_const;
    std::vector<int32_t> sdf_range;
    std::vector<int32_t> sdf_child;
    std::vector<jsrt_rec_sdfnode> sdf_nodes;
    std::vector<jsrt_rec_sdfgeom> sdfg;
    DCamera cam;
    float bg[4];
    int32_t kind, spp, max_depth, width, height;
    int32_t all_roots_prims;
    int32_t max_children = 2;  // most children a ray-tree node can spawn (0..2)
    int32_t features = 0, profile = PF_ALL;  // PF_* bits used / kernel instantiation chosen
    // workload facts used for algorithmic-byte accounting
    int64_t n_bvh_nodes = 0, n_triangles = 0;
    int32_t bvh_max_depth = 0;  // deepest BVH node (root = 0): sizes the LDS traversal stack
    // shadow hand-off grid (DScene::grid_*): cells, their root masks (+ the outside bucket's)
    std::vector<uint64_t> grid_mask;
    float grid_lo[3] = {0, 0, 0}, grid_inv[3] = {0, 0, 0};
    int32_t grid_dim[3] = {0, 0, 0}, grid_cells = 0;
    // the flat shadow loop's records (DScene::sroot, empty: not built) and the grid masks over them
    std::vector<SRoot> sroot;
    std::vector<uint64_t> grid_smask;
    int32_t sr_first[SR_N + 2] = {};
};

// Returns 0 on success; otherwise fills err.
int load_scene(const void *blob, size_t nbytes, HostScene &out, std::string &err);

}  // namespace jsrt
