// scene_load.cpp — parse + validate a JSRT blob (include/jsrt_scene.h) into the HBM layout of
// device_scene.h.  Host-only; compiled with -ffp-contract=off so the few float64 values computed
// here (shading contexts, area-light normals) round exactly as the reference's JS does.
#include "scene_load.h"

#include <float.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <set>
#include <unordered_map>

namespace jsrt {
namespace {

struct Blob {
    const jsrt_rec_renderer *rndr = nullptr;
    const jsrt_rec_camera *cam = nullptr;
    const jsrt_rec_mcolor *mc = nullptr;
    const jsrt_rec_material *mat = nullptr;
    const jsrt_rec_geometry *geom = nullptr;
    const jsrt_rec_object *obj = nullptr;
    const jsrt_rec_matrix *mats = nullptr;
    const int32_t *root = nullptr, *chld = nullptr;
    const jsrt_rec_bvhnode *bvh = nullptr;
    const jsrt_rec_triangle *tri = nullptr;
    const jsrt_rec_light *lite = nullptr;
    const jsrt_rec_sdfnode *sdf = nullptr;
    const jsrt_rec_sdfgeom *sdfg = nullptr;
    uint32_t n_mc = 0, n_mat = 0, n_geom = 0, n_obj = 0, n_mats = 0, n_root = 0, n_chld = 0, n_bvh = 0, n_tri = 0,
             n_lite = 0, n_sdf = 0, n_sdfg = 0;
};

struct LoadError {
    std::string msg;
};
[[noreturn]] void fail(const std::string &m) { throw LoadError{m}; }

template <class T>
void bind(const jsrt_section &s, const uint8_t *base, const T *&ptr, uint32_t &n, const char *name) {
    if (s.bytes != (uint64_t)s.count * sizeof(T)) fail(std::string("bad section size: ") + name);
    ptr = reinterpret_cast<const T *>(base + s.offset);
    n = s.count;
}

Blob parse(const void *data, size_t nbytes) {
    Blob B;
    const uint8_t *b = static_cast<const uint8_t *>(data);
    if (!b || nbytes < sizeof(jsrt_blob_header)) fail("scene blob too small");
    const auto *h = reinterpret_cast<const jsrt_blob_header *>(b);
    if (h->magic != JSRT_MAGIC) fail("not a JSRT scene blob");
    if (h->version != JSRT_VERSION) fail("unsupported JSRT blob version");
    if (sizeof(*h) + (uint64_t)h->n_sections * sizeof(jsrt_section) > nbytes) fail("truncated section table");
    const auto *sec = reinterpret_cast<const jsrt_section *>(b + sizeof(*h));
    for (uint32_t i = 0; i < h->n_sections; ++i) {
        const jsrt_section &s = sec[i];
        if (s.offset > nbytes || s.bytes > nbytes - s.offset) fail("section out of range");
        if (s.offset % 8) fail("misaligned section");
        uint32_t one = 0;
        switch (s.tag) {
        case JSRT_SEC_RENDERER: bind(s, b, B.rndr, one, "RNDR"); if (one != 1) fail("need one renderer"); break;
        case JSRT_SEC_CAMERA: bind(s, b, B.cam, one, "CAMR"); if (one != 1) fail("need one camera"); break;
        case JSRT_SEC_MCOLOR: bind(s, b, B.mc, B.n_mc, "MCOL"); break;
        case JSRT_SEC_MATERIAL: bind(s, b, B.mat, B.n_mat, "MATL"); break;
        case JSRT_SEC_GEOMETRY: bind(s, b, B.geom, B.n_geom, "GEOM"); break;
        case JSRT_SEC_OBJECT: bind(s, b, B.obj, B.n_obj, "OBJS"); break;
        case JSRT_SEC_MATRIX: bind(s, b, B.mats, B.n_mats, "MATS"); break;
        case JSRT_SEC_ROOT: bind(s, b, B.root, B.n_root, "ROOT"); break;
        case JSRT_SEC_CHILD: bind(s, b, B.chld, B.n_chld, "CHLD"); break;
        case JSRT_SEC_BVHNODE: bind(s, b, B.bvh, B.n_bvh, "BVHN"); break;
        case JSRT_SEC_TRIANGLE: bind(s, b, B.tri, B.n_tri, "TRIS"); break;
        case JSRT_SEC_LIGHT: bind(s, b, B.lite, B.n_lite, "LITE"); break;
        case JSRT_SEC_SDFNODE: bind(s, b, B.sdf, B.n_sdf, "SDFN"); break;
        case JSRT_SEC_SDFGEOM: bind(s, b, B.sdfg, B.n_sdfg, "SDFG"); break;
        default: break;  // unknown sections are ignored (forward compatible)
        }
    }
    if (!B.rndr || !B.cam) fail("scene blob lacks renderer/camera");
    return B;
}

// Row 3 must map w exactly as (0,0,0,1) does after the f32 store: the kernels carry w implicitly
// (1 for points, 0 for directions).  Mat4.inverse can leave m33 = 0.9999999999999998, whose f32
// rounding is exactly 1 (tests/AMultipleBVH), so compare in f32 for m33.
bool is_affine(const double *m) {
    for (int i = 0; i < 12; ++i)  // a NaN in rows 0..2 makes every transformed ray NaN: no hit,
        if (m[i] != m[i]) return true;  // whatever row 3 holds (tests/SDF_RecursiveUnionTest: Math.pi)
    return m[12] == 0 && m[13] == 0 && m[14] == 0 && (float)m[15] == 1.0f;
}
bool is_identity(const double *m) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            if (m[4 * r + c] != (r == c ? 1.0 : 0.0)) return false;
    return true;
}

// The shading matrix prim.inv x ctx exactly as render.hip's shade_node computes it (prim row 3
// taken as 0,0,0,1; sums from 0, left to right, float64) — precomputed for the common cases.
void shade_matrix(const double *pinv12, const double *C, double *out) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            const double a0 = r < 3 ? pinv12[4 * r + 0] : 0.0, a1 = r < 3 ? pinv12[4 * r + 1] : 0.0,
                         a2 = r < 3 ? pinv12[4 * r + 2] : 0.0, a3 = r < 3 ? pinv12[4 * r + 3] : 1.0;
            double s = 0;
            s += a0 * C[c];
            s += a1 * C[4 + c];
            s += a2 * C[8 + c];
            s += a3 * C[12 + c];
            out[4 * r + c] = s;
        }
}

// Mat*Mat exactly as math.js:399-409 (sum from 0, left to right, float64)
void mat_mul(const double *A, const double *B, double *R) {
    double t[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += A[4 * r + k] * B[4 * k + c];
            t[4 * r + c] = s;
        }
    memcpy(R, t, sizeof t);
}

// ---- conservative world bounds for culling (never change results: DESIGN.md §3.4) ----
struct LBox {
    double lo[3], hi[3];
    bool bounded;
};

// General 4x4 inverse (Gauss-Jordan, partial pivoting, long double): maps local -> world.
bool invert4(const double *m, long double *out) {
    long double a[4][8];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c) a[r][c] = c < 4 ? (long double)m[4 * r + c] : (c - 4 == r ? 1.0L : 0.0L);
    for (int c = 0; c < 4; ++c) {
        int piv = c;
        for (int r = c + 1; r < 4; ++r)
            if (fabsl(a[r][c]) > fabsl(a[piv][c])) piv = r;
        if (!(fabsl(a[piv][c]) > 0) || !isfinite((double)a[piv][c])) return false;
        if (piv != c)
            for (int k = 0; k < 8; ++k) { long double t = a[c][k]; a[c][k] = a[piv][k]; a[piv][k] = t; }
        const long double d = a[c][c];
        for (int k = 0; k < 8; ++k) a[c][k] /= d;
        for (int r = 0; r < 4; ++r)
            if (r != c) {
                const long double f = a[r][c];
                for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k];
            }
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out[4 * r + c] = a[r][4 + c];
    return true;
}

double frob3(const long double *m) {  // Frobenius norm of the linear 3x3 part
    long double s = 0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) s += m[4 * r + c] * m[4 * r + c];
    return (double)sqrtl(s);
}

// Box in the parent space of an object whose world->local matrix is `inv`; kappa accumulates the
// condition number of the linear part (error amplification).
LBox to_parent(const LBox &b, const double *inv, double &kappa) {
    LBox r;
    r.bounded = false;
    if (!b.bounded) return r;
    long double T[16], M[16];
    if (!invert4(inv, T)) return r;
    for (int i = 0; i < 16; ++i) M[i] = inv[i];
    kappa *= frob3(M) * frob3(T);
    for (int k = 0; k < 3; ++k) { r.lo[k] = INFINITY; r.hi[k] = -INFINITY; }
    for (int c = 0; c < 8; ++c) {
        const long double p[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
        for (int k = 0; k < 3; ++k) {
            const long double v = T[4 * k] * p[0] + T[4 * k + 1] * p[1] + T[4 * k + 2] * p[2] + T[4 * k + 3];
            r.lo[k] = fmin(r.lo[k], (double)v);
            r.hi[k] = fmax(r.hi[k], (double)v);
        }
    }
    r.bounded = true;
    for (int k = 0; k < 3; ++k) r.bounded &= isfinite(r.lo[k]) && isfinite(r.hi[k]);
    return r;
}

struct Loader {
    const Blob &B;
    HostScene &S;
    std::unordered_map<int32_t, int32_t> prim_of_obj;   // OBJS idx -> DPrim idx
    std::unordered_map<int32_t, int32_t> tri_of_blob;   // TRIS idx -> DTri idx
    std::unordered_map<int32_t, int32_t> bvh_of_root;   // BVHN root -> DBvhNode root
    std::unordered_map<int32_t, int32_t> bvh_fast;      // BVHN root -> fast flag
    std::unordered_map<int32_t, int32_t> sdfg_of_blob;
    std::unordered_map<int32_t, std::pair<int32_t, int32_t>> sdf_code_of;
    std::vector<LBox> prim_box;                          // local bound per DPrim
    double cur_leaf_kappa = 1;
    std::unordered_map<int32_t, double> bvh_leaf_kappa;  // BVHN root -> max leaf condition number

    Loader(const Blob &b, HostScene &s) : B(b), S(s) {}

    const jsrt_rec_matrix &matrix(int32_t i) {
        if (i < 0 || (uint32_t)i >= B.n_mats) fail("matrix index out of range");
        return B.mats[i];
    }

    void check_mc(int32_t i, int depth = 0) {
        if (i < 0) return;
        if ((uint32_t)i >= B.n_mc) fail("material colour index out of range");
        if (depth > 8) fail("material colour nesting too deep");
        const jsrt_rec_mcolor &m = B.mc[i];
        switch (m.kind) {
        case JSRT_MC_SOLID:
            if (m.len != 3) fail("colours must be 3-vectors (Vec.of(r,g,b))");
            break;
        case JSRT_MC_SCALED_SCALAR: check_mc(m.a, depth + 1); break;
        case JSRT_MC_SCALED_VEC:
            if (m.len < 3) fail("vector colour scale shorter than 3");
            check_mc(m.a, depth + 1);
            break;
        case JSRT_MC_CHECKER: check_mc(m.a, depth + 1); check_mc(m.b, depth + 1); break;
        default: fail("unsupported material colour kind");
        }
    }

    bool mc_uses_uv(int32_t i, int depth = 0) {
        if (i < 0 || (uint32_t)i >= B.n_mc || depth > 8) return false;
        const jsrt_rec_mcolor &m = B.mc[i];
        if (m.kind == JSRT_MC_CHECKER) return true;
        if (m.kind == JSRT_MC_SCALED_SCALAR || m.kind == JSRT_MC_SCALED_VEC) return mc_uses_uv(m.a, depth + 1);
        return false;
    }

    void shading_matrices() {
        static const double I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        S.prim_shade.assign(S.prims.size(), -1);
        for (size_t p = 0; p < S.prims.size(); ++p) {
            if (memcmp(S.prims[p].inv, I, sizeof I) == 0) continue;  // bitwise identity (no -0)
            double m[16];
            shade_matrix(S.prims[p].inv, S.ctx.data(), m);
            S.prim_shade[p] = (int32_t)(S.shade0.size() / 16);
            S.shade0.insert(S.shade0.end(), m, m + 16);
        }
        for (size_t c = 0; c < S.ctx.size() / 16; ++c) {
            double m[16];
            shade_matrix(I, S.ctx.data() + 16 * c, m);
            S.shadeI.insert(S.shadeI.end(), m, m + 16);
        }
    }

    int32_t tri_index(int32_t t) {
        auto it = tri_of_blob.find(t);
        if (it != tri_of_blob.end()) return it->second;
        if (t < 0 || (uint32_t)t >= B.n_tri) fail("triangle index out of range");
        const jsrt_rec_triangle &R = B.tri[t];
        DTri d;
        memset(&d, 0, sizeof d);
        for (int k = 0; k < 3; ++k) {
            d.n[k] = R.normal[k];
            d.p0[k] = R.p[0][k];
            d.v0[k] = R.v0[k];
            d.v1[k] = R.v1[k];
        }
        if (R.normal[3] != 0.0f) fail("triangle normal must have w = 0");
        d.delta = R.delta;
        d.d00 = R.d00;
        d.d11 = R.d11;
        d.d01 = R.d01;
        d.denom = R.denom;
        d.prim = -1;
        d.shade = -1;
        if (R.has_normal || R.has_uv) {
            DTriShade s;
            memset(&s, 0, sizeof s);
            memcpy(s.vn, R.vn, sizeof s.vn);
            memcpy(s.uv, R.uv, sizeof s.uv);
            s.has_normal = R.has_normal;
            s.has_uv = R.has_uv;
            s.uv_len = R.uv_len;
            if (R.has_uv && (R.uv_len < 2 || R.uv_len > 4)) fail("bad triangle UV length");
            d.shade = (int32_t)S.trish.size();
            S.trish.push_back(s);
        }
        int32_t idx = (int32_t)S.tris.size();
        S.tris.push_back(d);
        tri_of_blob[t] = idx;
        S.n_triangles++;
        return idx;
    }

    int32_t prim_index(int32_t o) {
        auto it = prim_of_obj.find(o);
        if (it != prim_of_obj.end()) return it->second;
        const jsrt_rec_object &O = B.obj[o];
        if (O.geometry < 0 || (uint32_t)O.geometry >= B.n_geom) fail("geometry index out of range");
        if (O.material < 0 || (uint32_t)O.material >= B.n_mat) fail("primitive without material");
        const jsrt_rec_matrix &M = matrix(O.matrix);
        if (!is_affine(M.inv)) fail("non-affine primitive transforms are not supported");
        const jsrt_rec_geometry &G = B.geom[O.geometry];
        DPrim p;
        memset(&p, 0, sizeof p);
        memcpy(p.inv, M.inv, sizeof p.inv);
        p.gkind = (int32_t)G.kind;
        p.gindex = -1;
        p.material = O.material;
        p.casts_shadow = O.casts_shadow ? 1 : 0;
        switch (G.kind) {
        case JSRT_GEOM_PLANE:
        case JSRT_GEOM_SQUARE:
        case JSRT_GEOM_CIRCLE:
        case JSRT_GEOM_SPHERE:
        case JSRT_GEOM_CYLINDER: break;
        case JSRT_GEOM_AABB: memcpy(p.center, G.center, 16); memcpy(p.half, G.half, 16); break;
        case JSRT_GEOM_TRIANGLE: p.gindex = tri_index(G.index); break;
        case JSRT_GEOM_SDF: p.gindex = sdfg_index(G.index); break;
        default: fail("unsupported geometry kind");
        }
        int32_t idx = (int32_t)S.prims.size();
        S.prims.push_back(p);
        S.prim_obj.push_back(o);
        prim_of_obj[o] = idx;
        LBox lb;
        lb.bounded = true;
        auto set = [&](double x0, double y0, double z0, double x1, double y1, double z1) {
            lb.lo[0] = x0; lb.lo[1] = y0; lb.lo[2] = z0; lb.hi[0] = x1; lb.hi[1] = y1; lb.hi[2] = z1;
        };
        switch (G.kind) {
        case JSRT_GEOM_SQUARE: set(-0.5, -0.5, 0, 0.5, 0.5, 0); break;
        case JSRT_GEOM_CIRCLE: set(-1, -1, 0, 1, 1, 0); break;
        case JSRT_GEOM_SPHERE:
        case JSRT_GEOM_CYLINDER: set(-1, -1, -1, 1, 1, 1); break;
        case JSRT_GEOM_AABB:
            set((double)G.center[0] - G.half[0], (double)G.center[1] - G.half[1], (double)G.center[2] - G.half[2],
                (double)G.center[0] + G.half[0], (double)G.center[1] + G.half[1], (double)G.center[2] + G.half[2]);
            break;
        case JSRT_GEOM_TRIANGLE: {
            const jsrt_rec_triangle &T = B.tri[G.index];
            set(INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY);
            for (int v = 0; v < 3; ++v)
                for (int k = 0; k < 3; ++k) {
                    lb.lo[k] = fmin(lb.lo[k], (double)T.p[v][k]);
                    lb.hi[k] = fmax(lb.hi[k], (double)T.p[v][k]);
                }
            break;
        }
        case JSRT_GEOM_SDF: {
            const jsrt_rec_sdfgeom &SG = B.sdfg[G.index];
            set((double)SG.center[0] - SG.half[0], (double)SG.center[1] - SG.half[1], (double)SG.center[2] - SG.half[2],
                (double)SG.center[0] + SG.half[0], (double)SG.center[1] + SG.half[1], (double)SG.center[2] + SG.half[2]);
            break;
        }
        default: lb.bounded = false; break;  // SimplePlane / Plane: unbounded
        }
        for (int k = 0; k < 3; ++k) lb.bounded &= isfinite(lb.lo[k]) && isfinite(lb.hi[k]);
        prim_box.push_back(lb);
        return idx;
    }

    // ---- BVH (aggregates.js:187-225) ----
    int32_t bvh_node(int32_t n, int depth, bool &fast) {
        if (n < 0 || (uint32_t)n >= B.n_bvh) fail("BVH node index out of range");
        if (depth > 60) fail("BVH too deep");
        const jsrt_rec_bvhnode &R = B.bvh[n];
        int32_t idx = (int32_t)S.bvh.size();
        S.bvh.push_back(DBvhNode{});
        S.n_bvh_nodes++;
        S.bvh_max_depth = std::max(S.bvh_max_depth, depth);
        DBvhNode d;
        d.cx = R.center[0]; d.cy = R.center[1]; d.cz = R.center[2];
        d.hx = R.half[0]; d.hy = R.half[1]; d.hz = R.half[2];
        if (R.is_leaf) {
            d.a = (int32_t)S.leaf_prims.size();
            d.b = ~R.n_obj;
            for (int32_t i = 0; i < R.n_obj; ++i) {
                const int32_t o = B.chld[R.first_obj + i];
                if (o < 0 || (uint32_t)o >= B.n_obj) fail("BVH leaf object out of range");
                if (B.obj[o].kind != JSRT_OBJ_PRIMITIVE) fail("BVH leaves must hold Primitives");
                const int32_t p = prim_index(o);
                S.leaf_prims.push_back(p);
                const DPrim &P = S.prims[p];
                const bool tri = P.gkind == JSRT_GEOM_TRIANGLE;
                S.leaf_tris.push_back(tri ? P.gindex : -1);
                const jsrt_rec_matrix &M = matrix(B.obj[o].matrix);
                if (!(tri && is_identity(M.inv) && P.casts_shadow)) fast = false;
                if (!is_identity(M.inv)) {
                    double kk = 1;
                    LBox lb = to_parent(prim_box[p], M.inv, kk);
                    cur_leaf_kappa = fmax(cur_leaf_kappa, lb.bounded ? kk : INFINITY);
                }
            }
        } else {
            d.a = bvh_node(R.lesser, depth + 1, fast);
            d.b = bvh_node(R.greater, depth + 1, fast);
        }
        S.bvh[idx] = d;
        return idx;
    }

    // ---- leaf-ordered triangles ----
    // Copies each fast leaf's triangle into leaf order (ltris, parallel to leaf_prims), so a leaf test
    // loads its record without first loading its index (one dependent load less per leaf visit).
    // (Renumbering the nodes greater-first for locality was measured too: no effect, r02_s6.)
    void leaf_triangles() {
        S.ltris.assign(S.leaf_tris.size(), DTri{});
        for (size_t i = 0; i < S.leaf_tris.size(); ++i)
            if (S.leaf_tris[i] >= 0) S.ltris[i] = S.tris[S.leaf_tris[i]];
    }

    // ---- SDF (sdf.js) -> program (sdf_program.h) ----
    int32_t kconst(std::initializer_list<double> v) {
        int32_t i = (int32_t)S.sdf_const.size();
        for (double x : v) S.sdf_const.push_back(x);
        return i;
    }
    void emit(int32_t op, int32_t a = 0, int32_t b = 0) { S.sdf_insn.push_back(SdfInsn{op, a, b, 0}); }
    const jsrt_rec_sdfnode &sdfnode(int32_t n) {
        if (n < 0 || (uint32_t)n >= B.n_sdf) fail("SDF node index out of range");
        return B.sdf[n];
    }

    // transformer: multiplies the top of the scale stack by its st (sdf.js:382-477)
    void compile_transformer(int32_t n, int depth) {
        if (depth > 32) fail("SDF transformer nesting too deep");
        const jsrt_rec_sdfnode &N = sdfnode(n);
        switch (N.kind) {
        case JSRT_SDFT_SEQUENCE:
            for (int32_t i = 0; i < N.count; ++i) {
                emit(SOP_TPUSH);
                compile_transformer(B.chld[N.first + i], depth + 1);
                emit(SOP_TPOP_MUL);
            }
            break;
        case JSRT_SDFT_RECURSIVE: {
            const int32_t loop = (int32_t)S.sdf_insn.size();
            emit(SOP_LOOP, N.iterations, 0);
            emit(SOP_TPUSH);
            compile_transformer(N.a, depth + 1);
            emit(SOP_TPOP_MUL);
            S.sdf_insn[loop].b = (int32_t)S.sdf_insn.size();
            emit(SOP_ENDLOOP, loop);
            break;
        }
        case JSRT_SDFT_MATRIX: {
            if (!is_affine(N.minv)) fail("non-affine SDF matrix transformer");
            int32_t c = kconst({N.minv[0], N.minv[1], N.minv[2], N.minv[3], N.minv[4], N.minv[5], N.minv[6],
                                N.minv[7], N.minv[8], N.minv[9], N.minv[10], N.minv[11]});
            emit(SOP_XMAT, c, kconst({N.k}));
            break;
        }
        case JSRT_SDFT_REFLECTION:
            if (N.vec[3] != 0.0f) fail("reflection normal must have w = 0");
            emit(SOP_XREF, kconst({N.vec[0], N.vec[1], N.vec[2], N.k}));
            break;
        case JSRT_SDFT_REPETITION: {  // + the exact reciprocal of a power-of-two size (x / s == x * (1 / s))
            auto rcp2 = [](double v) {
                int e;
                const double m = frexp(v, &e);
                return (isfinite(v) && fabs(m) == 0.5) ? 1.0 / v : 0.0;
            };
            emit(SOP_XREP, kconst({N.vec[0], N.vec[1], N.vec[2], rcp2(N.vec[0]), rcp2(N.vec[1]), rcp2(N.vec[2])}));
            break;
        }
        default: fail("unsupported SDF transformer");
        }
    }

    void compile_sdf(int32_t n, int depth) {
        if (depth > 32) fail("SDF nesting too deep");
        const jsrt_rec_sdfnode &N = sdfnode(n);
        const int32_t start = (int32_t)S.sdf_insn.size();
        switch (N.kind) {
        case JSRT_SDF_UNION:
        case JSRT_SDF_INTERSECTION:
            if (N.count < 1) fail("empty SDF union/intersection");
            for (int32_t i = 0; i < N.count; ++i) compile_sdf(B.chld[N.first + i], depth + 1);
            emit(N.kind == JSRT_SDF_UNION ? SOP_MIN : SOP_MAX, N.count);
            break;
        case JSRT_SDF_DIFFERENCE:
            compile_sdf(N.a, depth + 1);
            compile_sdf(N.b, depth + 1);
            emit(SOP_NEG);
            emit(SOP_MAX, 2);
            break;
        case JSRT_SDF_SMOOTH_UNION:
            compile_sdf(N.a, depth + 1);
            compile_sdf(N.b, depth + 1);
            emit(SOP_SMIN, kconst({N.k}));
            break;
        case JSRT_SDF_SMOOTH_INTERSECTION:
            compile_sdf(N.a, depth + 1);
            emit(SOP_NEG);
            compile_sdf(N.b, depth + 1);
            emit(SOP_NEG);
            emit(SOP_SMIN, kconst({N.k}));
            emit(SOP_NEG);
            break;
        case JSRT_SDF_SMOOTH_DIFFERENCE:
            compile_sdf(N.a, depth + 1);
            emit(SOP_NEG);
            compile_sdf(N.b, depth + 1);
            emit(SOP_SMIN, kconst({N.k}));
            emit(SOP_NEG);
            break;
        case JSRT_SDF_ROUND:
            compile_sdf(N.a, depth + 1);
            emit(SOP_SUBK, kconst({N.k}));
            break;
        case JSRT_SDF_SPHERE: emit(SOP_SPHERE, kconst({N.k})); break;
        case JSRT_SDF_BOX: emit(SOP_BOX, kconst({N.vec[0], N.vec[1], N.vec[2], N.vec[3]})); break;
        case JSRT_SDF_TETRAHEDRON: emit(SOP_TETRA); break;
        case JSRT_SDF_TRANSFORM: /* sdf.js:330-333 */
            emit(SOP_PUSHP);
            emit(SOP_TPUSH);
            compile_transformer(N.b, depth + 1);
            compile_sdf(N.a, depth + 1);
            emit(SOP_MULS);
            emit(SOP_TPOP);
            emit(SOP_POPP);
            break;
        case JSRT_SDF_RECURSIVE_UNION: { /* sdf.js:349-357 */
            emit(SOP_PUSHP);
            compile_sdf(N.a, depth + 1);
            emit(SOP_TPUSH);
            const int32_t loop = (int32_t)S.sdf_insn.size();
            emit(SOP_LOOP, N.iterations, 0);
            emit(SOP_TPUSH);
            compile_transformer(N.b, depth + 1);
            emit(SOP_TPOP_MUL);
            compile_sdf(N.a, depth + 1);
            emit(SOP_MULS);
            emit(SOP_MIN, 2);
            S.sdf_insn[loop].b = (int32_t)S.sdf_insn.size();
            emit(SOP_ENDLOOP, loop);
            emit(SOP_TPOP);
            emit(SOP_POPP);
            break;
        }
        default: fail("unsupported SDF node");
        }
        if (N.kind == JSRT_SDF_SPHERE || N.kind == JSRT_SDF_BOX || N.kind == JSRT_SDF_TETRAHEDRON)
            if (N.basecolor_len != 3) fail("SDF basecolor must be a 3-vector");
        if (!sdf_code_of.count(n)) sdf_code_of[n] = {start, (int32_t)S.sdf_insn.size()};
    }

    // Static stack-depth check of one compiled program (loops have zero net effect).
    void check_sdf_stacks(size_t begin, size_t end) {
        int d = 0, p = 0, sc = 0, l = 0, md = 0, mp = 0, ms = 0, ml = 0;
        for (size_t i = begin; i < end; ++i) {
            const SdfInsn &I = S.sdf_insn[i];
            switch (I.op) {
            case SOP_BOX: case SOP_SPHERE: case SOP_TETRA: ++d; break;
            case SOP_MIN: case SOP_MAX: d -= I.a - 1; break;
            case SOP_SMIN: --d; break;
            case SOP_PUSHP: ++p; break;
            case SOP_POPP: --p; break;
            case SOP_TPUSH: ++sc; break;
            case SOP_TPOP: case SOP_TPOP_MUL: --sc; break;
            case SOP_LOOP: ++l; break;
            case SOP_ENDLOOP: --l; break;
            default: break;
            }
            md = d > md ? d : md; mp = p > mp ? p : mp; ms = sc > ms ? sc : ms; ml = l > ml ? l : ml;
            if (d < 0 || p < 0 || sc < 0 || l < 0) fail("SDF program stack underflow");
        }
        if (md > SDF_MAX_D || mp > SDF_MAX_P || ms > SDF_MAX_S || ml > SDF_MAX_LOOP)
            fail("SDF tree too deep/wide for the GPU program stacks");
    }

    // A union of n boxes at sdf_const[a] (4 doubles apart) that is the Menger sponge's cross (device_common.h
    // sdf_cross): three boxes, box i infinite along axis i, its other half sizes and those of the other boxes the
    // same finite, non-negative f32 h.  JSRT_SDF_CROSS=0 leaves every union to sdf_minbox (A/B).
    bool is_cross(int32_t a, size_t n) const {
        const char *knob = getenv("JSRT_SDF_CROSS");
        if (n != 3 || (knob && knob[0] == '0')) return false;
        const float h = (float)S.sdf_const.at(a + 1);
        if (!(h >= 0.0f && h <= FLT_MAX)) return false;
        for (int b = 0; b < 3; ++b)
            for (int i = 0; i < 3; ++i) {
                const double v = S.sdf_const.at(a + 4 * b + i);
                if (i == b ? !(v == INFINITY) : (float)v != h) return false;
            }
        return true;
    }

    // Peephole fusion of a compiled range into one-dispatch forms (sdf_program.h); returns the fused
    // range appended to the program.  Every fused op performs the same IEEE operations in the same
    // order as the sequence it replaces; only scale multiplies by an exact 1.0 (a transformer that
    // does not scale) are dropped.  LOOP / ENDLOOP targets are remapped.
    std::pair<int32_t, int32_t> fuse_sdf(int32_t begin, int32_t end) {
        std::vector<SdfInsn> in(S.sdf_insn.begin() + begin, S.sdf_insn.begin() + end);
        std::vector<int32_t> origin(in.size());  // original index of each instruction (loops)
        for (size_t i = 0; i < in.size(); ++i) origin[i] = begin + (int32_t)i;
        for (bool changed = true; changed;) {
            changed = false;
            std::vector<SdfInsn> out;
            std::vector<int32_t> og;
            for (size_t i = 0; i < in.size();) {
                auto op = [&](size_t k) { return k < in.size() ? in[k].op : -1; };
                if (op(i) == SOP_TPUSH && (op(i + 1) == SOP_XREP || op(i + 1) == SOP_XREF) && op(i + 2) == SOP_TPOP_MUL) {
                    out.push_back(in[i + 1]), og.push_back(-1), i += 3, changed = true;  // top * 1.0: exact
                    continue;
                }
                if (op(i) == SOP_TPUSH && op(i + 1) == SOP_XMAT && op(i + 2) == SOP_TPOP_MUL) {
                    out.push_back(SdfInsn{SOP_XMATS, in[i + 1].a, in[i + 1].b, 0}), og.push_back(-1), i += 3, changed = true;
                    continue;
                }
                if (op(i) == SOP_TPUSH && op(i + 1) == SOP_XMATS && op(i + 2) == SOP_XREP && op(i + 3) == SOP_TPOP_MUL) {
                    out.push_back(SdfInsn{SOP_XMATREP, in[i + 1].a, in[i + 1].b, in[i + 2].a}), og.push_back(-1);
                    i += 4, changed = true;
                    continue;
                }
                if (op(i) == SOP_MULS && op(i + 1) == SOP_MIN && in[i + 1].a == 2) {
                    out.push_back(SdfInsn{SOP_MULSMIN, 0, 0, 0}), og.push_back(-1), i += 2, changed = true;
                    continue;
                }
                if (op(i) == SOP_BOX) {
                    size_t n = 1;
                    while (op(i + n) == SOP_BOX && in[i + n].a == in[i].a + 4 * (int32_t)n) ++n;
                    if (n >= 2 && op(i + n) == SOP_MIN && in[i + n].a == (int32_t)n) {
                        out.push_back(SdfInsn{SOP_MINBOX, in[i].a, (int32_t)n, is_cross(in[i].a, n) ? 1 : 0}), og.push_back(-1);
                        i += n + 1, changed = true;
                        continue;
                    }
                }
                out.push_back(in[i]), og.push_back(origin[i]), ++i;
            }
            in.swap(out);
            origin.swap(og);
        }
        const int32_t fb = (int32_t)S.sdf_insn.size();
        std::unordered_map<int32_t, int32_t> at;  // original index -> fused index (loop markers)
        for (size_t i = 0; i < in.size(); ++i)
            if (origin[i] >= 0) at[origin[i]] = fb + (int32_t)i;
        for (SdfInsn &I : in) {
            if (I.op == SOP_LOOP) I.b = at.at(I.b);
            if (I.op == SOP_ENDLOOP) I.a = at.at(I.a);
        }
        S.sdf_insn.insert(S.sdf_insn.end(), in.begin(), in.end());
        return {fb, (int32_t)S.sdf_insn.size()};
    }

    // An SFORM_RUNION_DIFF's flags (the marker's b; sdf_forms.h sdf_form_normal4): 1 when the loop's matrix
    // (XMATREP a, 3 rows of 4) is diagonal -- every off-diagonal entry a zero of either sign, the translations +0
    // (their bits), the diagonal below 1e30 in magnitude -- so each coordinate's chain through the loop depends on
    // that coordinate alone.  JSRT_SDF_N4=0 clears it (A/B).
    int32_t runion_flags(const SdfInsn *R) const {
        const char *knob = getenv("JSRT_SDF_N4");
        if (knob && knob[0] == '0') return 0;
        if (R[4].a < 0 || R[4].a + 12 > (int32_t)S.sdf_const.size()) return 0;
        const double *m = S.sdf_const.data() + R[4].a;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) {
                const double v = m[4 * r + c];
                if (c == 3 ? !(v == 0.0 && !signbit(v)) : c == r ? !(fabs(v) < 1e30) : v != 0.0) return 0;
            }
        return 1;
    }

    // Program shapes with straight-line device code (sdf_forms.h): a recognised fused range gets a copy
    // prefixed by an SOP_FORM marker (the form reads its constants from the copied instructions).
    std::pair<int32_t, int32_t> match_sdf_forms(int32_t begin, int32_t end) {
        const SdfInsn *I = S.sdf_insn.data() + begin;
        const int32_t n = end - begin;
        static const int32_t runion[] = {SOP_PUSHP, SOP_MINBOX, SOP_TPUSH, SOP_LOOP, SOP_XMATREP, SOP_MINBOX,
                                         SOP_MULSMIN, SOP_ENDLOOP, SOP_TPOP, SOP_POPP};
        auto is_runion = [&](int32_t at) {  // the RecursiveTransformUnion shape at [at, at + 10)
            bool ok = at + 10 <= n;
            for (int32_t i = 0; ok && i < 10; ++i) ok = I[at + i].op == runion[i];
            return ok && I[at + 3].b == begin + at + 7 && I[at + 7].a == begin + at + 3;  // LOOP brackets [4, 6]
        };
        auto is_prim = [&](int32_t at) {
            return at < n && (I[at].op == SOP_BOX || I[at].op == SOP_SPHERE || I[at].op == SOP_TETRA);
        };
        // TransformSDF(primitive, Matrix) at [at, at + 7): PUSHP TPUSH XMAT PRIM MULS TPOP POPP
        auto is_tprim = [&](int32_t at) {
            return at + 7 <= n && I[at].op == SOP_PUSHP && I[at + 1].op == SOP_TPUSH && I[at + 2].op == SOP_XMAT &&
                   is_prim(at + 3) && I[at + 4].op == SOP_MULS && I[at + 5].op == SOP_TPOP && I[at + 6].op == SOP_POPP;
        };
        int32_t form = 0, fflags = 0, fpad = 0;
        if (n == 1 && is_prim(0)) form = SFORM_PRIM;
        else if (n == 7 && I[0].op == SOP_PUSHP && I[1].op == SOP_TPUSH && (I[2].op == SOP_XMAT || I[2].op == SOP_XREP) &&
                 is_prim(3) && I[4].op == SOP_MULS && I[5].op == SOP_TPOP && I[6].op == SOP_POPP)
            form = SFORM_TX1;
        else if (n == 10 && is_runion(0)) form = SFORM_RUNION;
        else if (n == 13 && I[0].op == SOP_BOX && is_runion(1) && I[11].op == SOP_NEG && I[12].op == SOP_MAX && I[12].a == 2)
            form = SFORM_RUNION_DIFF;
        else if (is_tprim(0)) {  // SFORM_PAIR: tprim [NEG] tprim [NEG] (MIN 2 | MAX 2 | SMIN) [NEG]
            int32_t j = 7, fl = 0;
            if (j < n && I[j].op == SOP_NEG) { fl |= SPAIR_NEG_A; ++j; }
            const int32_t ob = j;
            if (is_tprim(j)) {
                j += 7;
                if (j < n && I[j].op == SOP_NEG) { fl |= SPAIR_NEG_B; ++j; }
                bool comb = true;
                if (j < n && I[j].op == SOP_MIN && I[j].a == 2) {
                } else if (j < n && I[j].op == SOP_MAX && I[j].a == 2) {
                    fl |= SPAIR_MAX;
                } else if (j < n && I[j].op == SOP_SMIN) {
                    fl |= SPAIR_SMIN;
                } else {
                    comb = false;
                }
                if (comb) {
                    ++j;
                    if (j < n && I[j].op == SOP_NEG) { fl |= SPAIR_NEG_OUT; ++j; }
                    if (j == n) { form = SFORM_PAIR; fflags = fl; fpad = ob; }
                }
            }
        } else if (n >= 11 && I[0].op == SOP_PUSHP && I[1].op == SOP_TPUSH && I[2].op == SOP_LOOP &&
                   I[3].op == SOP_TPUSH && I[4].op == SOP_XMATS) {  // SFORM_TXREC
            int32_t m = 0;
            while (5 + m < n && I[5 + m].op == SOP_XREF) ++m;
            const int32_t e = 6 + m;  // ENDLOOP
            if (n == 11 + m && I[5 + m].op == SOP_TPOP_MUL && I[e].op == SOP_ENDLOOP && I[2].b == begin + e &&
                I[e].a == begin + 2 && is_prim(7 + m) && I[8 + m].op == SOP_MULS && I[9 + m].op == SOP_TPOP &&
                I[10 + m].op == SOP_POPP) {
                form = SFORM_TXREC;
                fflags = m;
            }
        }
        if (!form) return {begin, end};
        if (form == SFORM_RUNION_DIFF) fflags = runion_flags(I + 1);
        const int32_t fb = (int32_t)S.sdf_insn.size();
        S.sdf_insn.push_back(SdfInsn{SOP_FORM, form, fflags, fpad});
        for (int32_t i = 0; i < n; ++i) {
            SdfInsn c = S.sdf_insn[begin + i];
            if (c.op == SOP_LOOP) c.b += fb + 1 - begin;
            if (c.op == SOP_ENDLOOP) c.a += fb + 1 - begin;
            S.sdf_insn.push_back(c);
        }
        return {fb, (int32_t)S.sdf_insn.size()};
    }

    int32_t sdfg_index(int32_t g) {
        auto it = sdfg_of_blob.find(g);
        if (it != sdfg_of_blob.end()) return it->second;
        if (g < 0 || (uint32_t)g >= B.n_sdfg) fail("SDF geometry index out of range");
        jsrt_rec_sdfgeom G = B.sdfg[g];
        const size_t first = S.sdf_insn.size();
        compile_sdf(G.root, 0);
        emit(SOP_END);
        check_sdf_stacks(first, S.sdf_insn.size());
        int32_t idx = (int32_t)S.sdfg.size();
        S.sdfg.push_back(G);
        sdfg_of_blob[g] = idx;
        return idx;
    }

    // ---- object graph -> instance tree ----
    int32_t inst(int32_t o, const double *ctx_mat, int depth) {
        if (o < 0 || (uint32_t)o >= B.n_obj) fail("object index out of range");
        if (depth > 8) fail("aggregate nesting deeper than 8 levels");
        const jsrt_rec_object &O = B.obj[o];
        DInst d;
        memset(&d, 0, sizeof d);
        d.kind = 0;
        switch (O.kind) {
        case JSRT_OBJ_PRIMITIVE:
            d.kind = INST_PRIM;
            d.prim = prim_index(o);
            break;
        case JSRT_OBJ_AGGREGATE:
        case JSRT_OBJ_BVH: {
            const jsrt_rec_matrix &M = matrix(O.matrix);
            if (!is_affine(M.inv)) fail("non-affine aggregate transforms are not supported");
            d.matrix = (int32_t)(S.mats.size() / 12);
            for (int k = 0; k < 12; ++k) S.mats.push_back(M.inv[k]);
            double child_ctx[16];
            mat_mul(M.inv, ctx_mat, child_ctx);  // world.js:37-39
            d.ctx = (int32_t)(S.ctx.size() / 16);
            for (int k = 0; k < 16; ++k) S.ctx.push_back(child_ctx[k]);
            if (O.kind == JSRT_OBJ_BVH) {
                d.kind = INST_BVH;
                auto it = bvh_of_root.find(O.bvh_root);
                if (it == bvh_of_root.end()) {
                    bool fast = true;
                    cur_leaf_kappa = 1;
                    const int32_t r = bvh_node(O.bvh_root, 0, fast);
                    bvh_leaf_kappa[O.bvh_root] = cur_leaf_kappa;
                    bvh_of_root[O.bvh_root] = r;
                    bvh_fast[O.bvh_root] = fast ? 1 : 0;
                    it = bvh_of_root.find(O.bvh_root);
                }
                d.first = it->second;
                d.count = bvh_fast[O.bvh_root];
            } else {
                d.kind = INST_AGG;
                std::vector<int32_t> kids;
                for (int32_t i = 0; i < O.n_children; ++i) kids.push_back(inst(B.chld[O.first_child + i], child_ctx, depth + 1));
                d.first = (int32_t)S.inst_child.size();
                d.count = (int32_t)kids.size();
                for (int32_t k : kids) S.inst_child.push_back(k);
            }
            break;
        }
        default: fail("unsupported world object (TransformedWorldObject is not renderable in the reference either)");
        }
        int32_t idx = (int32_t)S.insts.size();
        S.insts.push_back(d);
        return idx;
    }

    // Bound of instance `i` in its parent's space; kappa = error amplification below the parent.
    LBox inst_bound(int32_t i, double &kappa) {
        const DInst &I = S.insts[i];
        if (I.kind == INST_PRIM) {
            double m[16];
            for (int k = 0; k < 12; ++k) m[k] = S.prims[I.prim].inv[k];
            m[12] = m[13] = m[14] = 0; m[15] = 1;
            return to_parent(prim_box[I.prim], m, kappa);
        }
        LBox local;
        local.bounded = true;
        double kin = 1;
        if (I.kind == INST_BVH) {
            const DBvhNode &R = S.bvh[I.first];
            local.lo[0] = (double)R.cx - R.hx; local.lo[1] = (double)R.cy - R.hy; local.lo[2] = (double)R.cz - R.hz;
            local.hi[0] = (double)R.cx + R.hx; local.hi[1] = (double)R.cy + R.hy; local.hi[2] = (double)R.cz + R.hz;
            for (auto &kv : bvh_of_root)
                if (kv.second == I.first) kin = bvh_leaf_kappa[kv.first];
        } else {
            for (int k = 0; k < 3; ++k) { local.lo[k] = INFINITY; local.hi[k] = -INFINITY; }
            for (int32_t c = 0; c < I.count; ++c) {
                double kc = 1;
                const LBox cb = inst_bound(S.inst_child[I.first + c], kc);
                if (!cb.bounded) { local.bounded = false; break; }
                kin = fmax(kin, kc);
                for (int k = 0; k < 3; ++k) { local.lo[k] = fmin(local.lo[k], cb.lo[k]); local.hi[k] = fmax(local.hi[k], cb.hi[k]); }
            }
        }
        for (int k = 0; k < 3; ++k) local.bounded &= isfinite(local.lo[k]) && isfinite(local.hi[k]);
        double m[16];
        for (int k = 0; k < 12; ++k) m[k] = S.mats[12 * I.matrix + k];
        m[12] = m[13] = m[14] = 0; m[15] = 1;
        kappa *= kin;
        return to_parent(local, m, kappa);
    }

    void root_bounds() {
        for (int32_t r : S.roots) {
            RootBound rb;
            memset(&rb, 0, sizeof rb);
            double kappa = 1;
            const LBox b = inst_bound(r, kappa);
            rb.bounded = b.bounded && isfinite(kappa) && kappa < 1e6;
            if (rb.bounded) {
                double c2 = 0, r2 = 0;
                for (int k = 0; k < 3; ++k) {
                    const double c = 0.5 * (b.lo[k] + b.hi[k]), h = 0.5 * (b.hi[k] - b.lo[k]);
                    c2 += c * c;
                    r2 += h * h;
                }
                // margin >= 1e3 x the f32 rounding bound 4u*kappa*(|o| + |c| + R) of an accepted hit point
                const double k = 1e-4 * kappa * sqrt(3.0);
                const double e0 = 1e-4 * kappa * (sqrt(c2) + sqrt(r2)) + 1e-6 * (1 + sqrt(r2));
                rb.k = (float)(k * 1.001);
                rb.e0 = (float)(e0 * 1.001);
                for (int i = 0; i < 3; ++i) {
                    rb.lo[i] = nextafterf((float)b.lo[i], -INFINITY);
                    rb.hi[i] = nextafterf((float)b.hi[i], INFINITY);
                }
            }
            S.rbounds.push_back(rb);
        }
    }

    // MaterialColor.color(data) of every colour chain that does not read (u, v) (no checkerboard):
    // mc_eval's arithmetic (device_common.h) done once here -- the solid colour, then the Scaled
    // wrappers innermost first, f32(x * s) in f64 for a scalar, f32 products for a vector -- so the
    // kernels read one record instead of walking the chain with dependent loads.
    void mc_constants() {
        S.mc_const.assign(4 * S.mc.size(), 0.0f);
        for (size_t x = 0; x < S.mc.size(); ++x) {
            if (mc_uses_uv((int32_t)x)) continue;
            std::vector<int32_t> wrap;  // Scaled wrappers from the top down
            int32_t y = (int32_t)x;
            bool ok = true;
            for (int g = 0; g < 16 && ok && S.mc[y].kind != JSRT_MC_SOLID; ++g) {
                const uint32_t k = S.mc[y].kind;
                ok = (k == JSRT_MC_SCALED_SCALAR || k == JSRT_MC_SCALED_VEC) && S.mc[y].a >= 0 &&
                     (size_t)S.mc[y].a < S.mc.size();
                wrap.push_back(y);
                if (ok) y = S.mc[y].a;
            }
            if (!ok || S.mc[y].kind != JSRT_MC_SOLID) continue;
            float c[3] = {S.mc[y].vec[0], S.mc[y].vec[1], S.mc[y].vec[2]};
            for (size_t i = wrap.size(); i-- > 0;) {
                const jsrt_rec_mcolor &M = S.mc[wrap[i]];
                for (int k = 0; k < 3; ++k)
                    c[k] = M.kind == JSRT_MC_SCALED_SCALAR ? (float)((double)c[k] * M.scalar) : c[k] * M.vec[k];
            }
            memcpy(&S.mc_const[4 * x], c, sizeof c);
            S.mc_const[4 * x + 3] = 1.0f;
        }
    }

    // Area light world normal: inv_transform.transposed().times(n).to4(0).normalized() (lights.js:90)
    void area_normal(const double *Ti, float *out) {
        const double n[4] = {0, 0, 1, 0};
        float r[4];
        for (int i = 0; i < 4; ++i) {  // transposed row i = column i of Ti; dot over the 4-vector n
            double s = n[0] * Ti[0 * 4 + i] + n[1] * Ti[1 * 4 + i] + n[2] * Ti[2 * 4 + i] + n[3] * Ti[3 * 4 + i];
            r[i] = (float)s;
        }
        auto or0 = [](float x) { return (x != x || x == 0.0f) ? 0.0f : x; };
        float v[4] = {r[0], or0(r[1]), or0(r[2]), 0.0f};
        double nn = sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2] + (double)v[3] * v[3]);
        if (nn > 0.00001) {
            const double s = 1 / nn;
            for (int i = 0; i < 4; ++i) v[i] = (float)((double)v[i] * s);
        }
        memcpy(out, v, sizeof v);
    }

    void run() {
        const jsrt_rec_renderer &R = *B.rndr;
        S.kind = (int32_t)R.kind;
        S.spp = (int32_t)R.spp;
        S.max_depth = (int32_t)R.max_depth;
        S.width = (int32_t)R.width;
        S.height = (int32_t)R.height;
        if (R.bg_len != 3) fail("World.bg_color must be a 3-vector");
        memcpy(S.bg, R.bg, sizeof S.bg);
        const jsrt_rec_camera &C = *B.cam;
        if (!is_affine(C.transform)) fail("non-affine camera transform");
        memcpy(S.cam.T, C.transform, sizeof S.cam.T);
        S.cam.tan_fov = C.tan_fov;
        S.cam.aspect = C.aspect;
        S.cam.focus = C.focus_distance;
        S.cam.sensor = C.sensor_size;
        S.cam.kind = (int32_t)C.kind;

        // the shadow hand-off packs the material index into 20 bits beside the grid mask and its plane flags
        // (render_levels.h store_hand: mat << 8 | mask | HAND_*)
        if (B.n_mat >= (1u << 20)) fail("more than 2^20 materials");
        for (uint32_t i = 0; i < B.n_mat; ++i) {
            const jsrt_rec_material &M = B.mat[i];
            if (M.kind < JSRT_MAT_PHONG || M.kind > JSRT_MAT_TRANSPARENT) fail("unsupported material kind");
            if (M.kind == JSRT_MAT_SOLID || M.kind == JSRT_MAT_TRANSPARENT) check_mc(M.color);
            else {
                check_mc(M.ambient); check_mc(M.diffuse); check_mc(M.specular); check_mc(M.reflect); check_mc(M.transmit);
                if (M.ambient < 0 || M.diffuse < 0 || M.specular < 0 || M.reflect < 0 || M.transmit < 0)
                    fail("Phong material lacks a colour");
                if (M.kind == JSRT_MAT_PATH && !isfinite(M.smoothness))
                    fail("infinite-smoothness path-tracing scatter is broken in the reference (materials.js:430)");
            }
            S.mat.push_back(M);
            int32_t fl = 0;
            for (int32_t root : {M.color, M.ambient, M.diffuse, M.specular, M.reflect, M.transmit})
                if (mc_uses_uv(root)) fl |= MATF_UV;
            S.mat_flags.push_back(fl);
        }
        for (uint32_t i = 0; i < B.n_mc; ++i) S.mc.push_back(B.mc[i]);
        mc_constants();
        // constant diffuse / specular colours (k_shadow reads them from mc_const, not the hand-off)
        for (size_t i = 0; i < S.mat.size(); ++i) {
            const jsrt_rec_material &M = S.mat[i];
            if (M.kind == JSRT_MAT_SOLID || M.kind == JSRT_MAT_TRANSPARENT) continue;
            const float *d = &S.mc_const[4 * (size_t)M.diffuse], *sp = &S.mc_const[4 * (size_t)M.specular];
            if (d[3] != 0.0f) S.mat_flags[i] |= MATF_DIFF_CONST;
            if (sp[3] != 0.0f) {
                S.mat_flags[i] |= MATF_SPEC_CONST;
                uint32_t b[3];
                memcpy(b, sp, sizeof b);
                if (b[0] == 0u && b[1] == 0u && b[2] == 0u && M.smoothness >= 0.0 && M.smoothness <= 1e5)
                    S.mat_flags[i] |= MATF_SPEC_ZERO;
            }
        }

        const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        for (int k = 0; k < 16; ++k) S.ctx.push_back(I[k]);  // ctx 0: World.color's Mat4.identity()
        S.all_roots_prims = 1;
        for (uint32_t i = 0; i < B.n_root; ++i) {
            const int32_t ix = inst(B.root[i], I, 0);
            S.roots.push_back(ix);
            if (S.insts[ix].kind != INST_PRIM) S.all_roots_prims = 0;
        }
        root_bounds();
        for (size_t i = 0; i < S.roots.size(); ++i) {
            DRoot r;
            memset(&r, 0, sizeof r);
            const DInst &in = S.insts[S.roots[i]];
            r.rb = S.rbounds[i];
            r.kind = in.kind;
            r.inst = S.roots[i];
            r.prim = in.kind == INST_PRIM ? in.prim : -1;
            if (in.kind == INST_PRIM) r.p = S.prims[in.prim];
            else memcpy(r.p.inv, &S.mats[12 * (size_t)in.matrix], sizeof r.p.inv);
            S.rootrec.push_back(r);
        }
        for (uint32_t i = 0; i < B.n_lite; ++i) {
            const jsrt_rec_light &L = B.lite[i];
            DLight d;
            memset(&d, 0, sizeof d);
            d.kind = (int32_t)L.kind;
            d.color = L.color;
            check_mc(L.color);
            for (int32_t m = L.color, g = 0; m >= 0 && g < 16; ++g) {  // checkerboard anywhere in the chain?
                const jsrt_rec_mcolor &mc = B.mc[m];
                if (mc.kind == JSRT_MC_CHECKER) { d.needs_uv = 1; break; }
                m = (mc.kind == JSRT_MC_SCALED_SCALAR || mc.kind == JSRT_MC_SCALED_VEC) ? mc.a : -1;
            }
            d.gkind = (int32_t)L.geometry_kind;
            d.samples = (int32_t)L.samples;
            d.pos_len = (int32_t)L.pos_len;
            memcpy(d.pos, L.position, sizeof d.pos);
            memcpy(d.T, L.transform, sizeof d.T);
            memcpy(d.Ti, L.inv, sizeof d.Ti);
            if (L.kind == JSRT_LIGHT_POINT) {
                if (L.pos_len < 3 || L.pos_len > 4) fail("point light position must be a 3- or 4-vector");
                if (L.pos_len == 4 && L.position[3] != 1.0f) fail("point light position must have w = 1");
            } else if (L.kind == JSRT_LIGHT_AREA) {
                if (!is_affine(L.transform) || !is_affine(L.inv)) fail("non-affine area light transform");
                if (L.geometry_kind != JSRT_GEOM_SQUARE && L.geometry_kind != JSRT_GEOM_CIRCLE &&
                    L.geometry_kind != JSRT_GEOM_SPHERE)
                    fail("unsupported area light surface");
                area_normal(L.inv, d.wn);
            } else fail("unsupported light kind");
            // colorFromLights order: the light's samples in turn; each area sample draws twice
            const int32_t ns = L.kind == JSRT_LIGHT_POINT ? 1 : (int32_t)L.samples;
            d.inv_n = ns > 0 ? 1.0 / ns : 0.0;  // colorFromLights: light_color.times(1 / samples)
            if (ns < 0 || S.sample_light.size() + (size_t)ns > 4096) fail("too many light samples per shading point");
            for (int32_t k = 0; k < ns; ++k) {
                S.sample_light.push_back((int32_t)S.lights.size());
                S.sample_call.push_back(S.light_draws);
                if (L.kind == JSRT_LIGHT_AREA) S.light_draws += 2;
            }
            S.lights.push_back(d);
        }
        int32_t f = 0;
        for (const DInst &in : S.insts) {
            if (in.kind == INST_BVH) f |= PF_BVH | PF_TRI;
            if (in.kind == INST_AGG) f |= PF_AGG;
        }
        for (const DPrim &pr : S.prims) {
            if (pr.gkind == JSRT_GEOM_SDF) f |= PF_SDF;
            if (pr.gkind == JSRT_GEOM_TRIANGLE) f |= PF_TRI;
        }
        S.features = f;
        // most children one ray-tree node can spawn (materials.js:277-330), conservatively: the
        // wavefront pool is sized by it and a scene with <= 1 needs no per-batch overflow check
        auto maybe_nonzero = [&](int32_t m) {  // could this colour chain evaluate to a non-zero vector?
            std::vector<int32_t> todo{m};
            for (int g = 0; g < 64 && !todo.empty(); ++g) {
                const int32_t x = todo.back();
                todo.pop_back();
                if (x < 0) continue;
                const jsrt_rec_mcolor &c = B.mc[x];
                if (c.kind == JSRT_MC_SOLID) {
                    for (uint32_t k = 0; k < c.len && k < 4; ++k)
                        if (!(c.vec[k] == 0.0f)) return true;
                } else if (c.kind == JSRT_MC_CHECKER) {
                    todo.push_back(c.a);
                    todo.push_back(c.b);
                } else todo.push_back(c.a);
            }
            return !todo.empty();
        };
        S.max_children = 0;
        for (const jsrt_rec_material &M : S.mat) {
            int n = 0;
            if (M.kind == JSRT_MAT_TRANSPARENT) n = 1;
            else if (M.kind == JSRT_MAT_PHONG) n = (int)maybe_nonzero(M.reflect) + (int)maybe_nonzero(M.transmit);
            else if (M.kind != JSRT_MAT_SOLID) n = isinf(M.ratio) ? 1 : 2;  // infinite ratio: kr = 1
            S.max_children = std::max(S.max_children, n);
        }
        shading_matrices();
        leaf_triangles();
        for (const DPrim &pr : S.prims) {  // shade_node: every material but Solid / Transparent takes light samples
            const uint32_t k = S.mat[pr.material].kind;
            S.prim_lit.push_back(k != JSRT_MAT_SOLID && k != JSRT_MAT_TRANSPARENT ? 1 : 0);
        }
        S.profile = f == 0 ? PF_ANALYTIC : (f & ~PF_MESH) == 0 ? PF_MESH : (f & ~PF_SDF) == 0 ? PF_SDF : PF_ALL;
        for (uint32_t i = 0; i < B.n_sdf; ++i) S.sdf_nodes.push_back(B.sdf[i]);
        if (B.n_sdf) S.sdf_child.assign(B.chld, B.chld + B.n_chld);
        S.sdf_range.assign(2 * (size_t)B.n_sdf, -1);
        for (auto &kv : sdf_code_of) {
            S.sdf_range[2 * kv.first] = kv.second.first;
            S.sdf_range[2 * kv.first + 1] = kv.second.second;
        }
        // every node's distance (a geometry's root on each march step and for the normal, the children
        // getMaterialData compares) runs a fused copy of its range (JSRT_SDF_NOFUSE=1: A/B)
        const char *nf = getenv("JSRT_SDF_NOFUSE");
        if (!(nf && nf[0] == '1'))
            for (uint32_t n = 0; n < B.n_sdf; ++n) {
                if (S.sdf_range[2 * n] < 0) continue;
                auto fr = fuse_sdf(S.sdf_range[2 * n], S.sdf_range[2 * n + 1]);
                const char *nform = getenv("JSRT_SDF_NOFORMS");  // A/B: the VM for every shape
                if (!(nform && nform[0] == '1')) fr = match_sdf_forms(fr.first, fr.second);
                S.sdf_range[2 * n] = fr.first;
                S.sdf_range[2 * n + 1] = fr.second;
            }
        S.sdf_all_forms = S.sdfg.empty() ? 0 : 1;
        for (const jsrt_rec_sdfgeom &G : S.sdfg) {
            const int32_t pc = S.sdf_range[2 * (size_t)G.root];
            if (pc < 0 || S.sdf_insn[pc].op != SOP_FORM) S.sdf_all_forms = 0;
        }
        shadow_grid();
        shadow_roots();
    }

    // Spatial buckets of the shadow hand-off and their shadow-root masks (DScene::grid_*).
    //
    // The grid spans the bounded top-level objects' cull boxes with at most 63 cells (as cubic as the
    // extents allow); a hit point outside it goes to bucket grid_cells.  A shadow ray of a lit node in
    // cell c starts at the hit point P (in c, up to the rounding of the cell index, covered by growing
    // the cell by 1e-4 of the grid) and ends at delta = Q - P, Q a light sample point (in the light's
    // world box, grown for the f32 rounding of Q and of the subtraction): the segment lies in the box
    // hull(cell, light boxes).  A root whose cull box (RootBound: lo/hi grown by k |P|_inf + e0, with
    // the largest |P|_inf of the cell) misses that hull cannot produce an accepted shadow hit from any
    // point of the cell -- world_cast's own cull (root_needed) would reject it on every such ray -- so
    // the cell's mask leaves it out.  Unbounded roots are in every mask; the outside bucket's mask holds
    // every root.
    void shadow_grid() {
        const size_t nr = S.roots.size();
        const uint64_t all = nr >= 64 ? ~0ull : ((1ull << nr) - 1);
        S.grid_cells = 0;
        S.grid_mask.assign(1, all);
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool any = false;
        for (const RootBound &rb : S.rbounds)
            if (rb.bounded) {
                any = true;
                for (int k = 0; k < 3; ++k) { lo[k] = fmin(lo[k], rb.lo[k]); hi[k] = fmax(hi[k], rb.hi[k]); }
            }
        if (!any) return;
        double ext[3];
        for (int k = 0; k < 3; ++k) ext[k] = fmax(hi[k] - lo[k], 1e-6 * fmax(1.0, fmax(fabs(lo[k]), fabs(hi[k]))));
        int dim[3] = {1, 1, 1};
        double best = INFINITY;
        const char *gm = getenv("JSRT_GRID_MAX");  // A/B: fewer, larger cells
        const int cmax = gm ? std::max(1, std::min(63, atoi(gm))) : 63;
        for (int x = 1; x <= cmax; ++x)
            for (int y = 1; x * y <= cmax; ++y)
                for (int z = 1; x * y * z <= cmax; ++z) {
                    const double w = fmax(ext[0] / x, fmax(ext[1] / y, ext[2] / z));
                    if (w < best * (1 - 1e-9) || (w <= best * (1 + 1e-9) && x * y * z > dim[0] * dim[1] * dim[2])) {
                        best = w;
                        dim[0] = x; dim[1] = y; dim[2] = z;
                    }
                }
        // light sample points: a point light's position; an area light's surface through its transform
        // (Square / Circle sample [-0.5, 0.5]^2 x {0}, a Sphere the unit sphere, lights.js:80-92)
        double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const DLight &L : S.lights) {
            double c[3], h[3];
            if (L.kind == JSRT_LIGHT_POINT) {
                for (int k = 0; k < 3; ++k) { c[k] = L.pos[k]; h[k] = 0; }
            } else {
                const double lh[3] = {L.gkind == JSRT_GEOM_SPHERE ? 1.0 : 0.5, L.gkind == JSRT_GEOM_SPHERE ? 1.0 : 0.5,
                                      L.gkind == JSRT_GEOM_SPHERE ? 1.0 : 0.0};
                for (int k = 0; k < 3; ++k) {
                    c[k] = L.T[4 * k + 3];
                    h[k] = fabs(L.T[4 * k]) * lh[0] + fabs(L.T[4 * k + 1]) * lh[1] + fabs(L.T[4 * k + 2]) * lh[2];
                }
            }
            for (int k = 0; k < 3; ++k) {
                const double g = 1e-5 * (fabs(c[k]) + h[k] + 1.0);
                llo[k] = fmin(llo[k], c[k] - h[k] - g);
                lhi[k] = fmax(lhi[k], c[k] + h[k] + g);
            }
        }
        for (int k = 0; k < 3; ++k)
            if (!isfinite(llo[k]) || !isfinite(lhi[k])) return;  // no lights, or one that is not bounded
        const int cells = dim[0] * dim[1] * dim[2];
        S.grid_mask.assign(cells + 1, all);
        const double grow = 1e-4 * fmax(ext[0], fmax(ext[1], ext[2])) + 1e-6;
        for (int c = 0; c < cells; ++c) {
            const int ci[3] = {c % dim[0], (c / dim[0]) % dim[1], c / (dim[0] * dim[1])};
            double a[3], b[3], oabs = 0;
            for (int k = 0; k < 3; ++k) {
                const double w = ext[k] / dim[k];
                a[k] = lo[k] + ci[k] * w - grow;
                b[k] = lo[k] + (ci[k] + 1) * w + grow;
                oabs = fmax(oabs, fmax(fabs(a[k]), fabs(b[k])));
            }
            uint64_t m = 0;
            for (size_t r = 0; r < nr && r < 64; ++r) {
                const RootBound &rb = S.rbounds[r];
                bool need = !rb.bounded;
                if (!need) {
                    need = true;
                    for (int k = 0; k < 3 && need; ++k) {
                        const double hlo = fmin(a[k], llo[k]), hhi = fmax(b[k], lhi[k]);
                        const double g = 1e-5 * (fabs(hlo) + fabs(hhi) + 1.0);
                        const double e = 1.01 * ((double)rb.k * oabs + (double)rb.e0) + 1e-5 * (fabs(rb.lo[k]) + fabs(rb.hi[k]) + 1.0);
                        need = (double)rb.lo[k] - e <= hhi + g && (double)rb.hi[k] + e >= hlo - g;
                    }
                }
                if (need) m |= 1ull << r;
            }
            S.grid_mask[c] = nr <= 64 ? m : all;
        }
        S.grid_cells = cells;
        for (int k = 0; k < 3; ++k) {
            S.grid_dim[k] = dim[k];
            S.grid_lo[k] = (float)lo[k];
            S.grid_inv[k] = (float)(dim[k] / ext[k]);
        }
    }

    // The flat shadow loop's records (DScene::sroot): for a scene whose top level is at most 64 Primitives, the
    // shadow-casting ones (a shadow cast is not transparent: Primitive.intersect gives Infinity for the others,
    // world.js:104-113, which is never accepted) grouped by geometry class, and the grid masks remapped onto
    // them.  Called after shadow_grid.
    void shadow_roots() {
        S.sroot.clear();
        S.grid_smask.clear();
        for (int c = 0; c < SR_N + 2; ++c) S.sr_first[c] = 0;
        const size_t nr = S.roots.size();
        if (!S.all_roots_prims || nr == 0 || nr > 64) return;
        auto cls = [](int32_t g) {
            switch (g) {
            case JSRT_GEOM_AABB: return (int)SR_BOX;
            case JSRT_GEOM_PLANE: return (int)SR_PLANE;
            case JSRT_GEOM_SQUARE: return (int)SR_SQUARE;
            case JSRT_GEOM_CIRCLE: return (int)SR_CIRCLE;
            case JSRT_GEOM_SPHERE: return (int)SR_SPHERE;
            default: return (int)SR_OTHER;
            }
        };
        std::vector<int> perm;  // record j -> root index
        for (int c = 0; c < SR_N; ++c) {
            S.sr_first[c] = (int32_t)perm.size();
            for (size_t r = 0; r < nr; ++r) {
                const DPrim &P = S.prims[S.insts[S.roots[r]].prim];
                if (P.casts_shadow && cls(P.gkind) == c) perm.push_back((int)r);
            }
        }
        S.sr_first[SR_N] = S.sr_first[SR_N + 1] = (int32_t)perm.size();
        for (int r : perm) {
            const int32_t pi = S.insts[S.roots[r]].prim;
            const DPrim &P = S.prims[pi];
            const RootBound &rb = S.rbounds[r];
            SRoot s;
            memset(&s, 0, sizeof s);
            memcpy(s.inv, P.inv, sizeof s.inv);
            for (int k = 0; k < 3; ++k) {
                s.lo[k] = rb.lo[k];
                s.hi[k] = rb.hi[k];
                s.center[k] = P.center[k];
                s.half[k] = P.half[k];
            }
            s.k = rb.k;
            s.e0 = rb.e0;
            s.prim = pi;
            s.bounded = rb.bounded;
            S.sroot.push_back(s);
        }
        S.grid_smask.resize(S.grid_mask.size());
        for (size_t b = 0; b < S.grid_mask.size(); ++b) {
            uint64_t m = 0;
            for (size_t j = 0; j < perm.size(); ++j)
                if ((S.grid_mask[b] >> perm[j]) & 1ull) m |= 1ull << j;
            S.grid_smask[b] = m;
        }
    }
};

}  // namespace

int load_scene(const void *blob, size_t nbytes, HostScene &out, std::string &err) {
    try {
        Blob B = parse(blob, nbytes);
        out = HostScene();
        Loader L(B, out);
        L.run();
        return 0;
    } catch (const LoadError &e) {
        err = e.msg;
        return -1;
    } catch (const std::exception &e) {
        err = std::string("scene load: ") + e.what();
        return -1;
    }
}

}  // namespace jsrt
