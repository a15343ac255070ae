// mesh_build.cpp — native OBJ ingest + BVH build, spliced into a JSRT scene blob (include/jsrt_mesh.h).
//
// The reference builds its meshes in JS on every worker: loadObjFile/parseObjFile
// (src/objloader.js:144-238) turns OBJ text into Triangle primitives, BVHAggregate.build
// (src/aggregates.js:33-41) and BVHAggregateNode.build/split_objects (:65-185) bin them into a
// binary SAH tree.  For the dragon (99,968 triangles) that is ~25 s of JS; here it is plain C++ on the
// host, and it must reproduce the reference's tree BIT FOR BIT: the device traverses greater-first
// exactly as aggregates.js:221-222, so only an identical topology gives identical closest-hit
// tie-breaks.  Every value below is therefore computed with the reference's numeric model
// (SURVEY.md §8.0): Vec components are f32, scalars f64, Mat x Vec per-row f64 dot then an f32 store.
//
// Host code only: nothing here touches the GPU.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <map>
#include <string>
#include <vector>

#include "../../include/jsrt_mesh.h"
#include "../../include/jsrt_scene.h"
#include "obj_parse.h"

namespace jsrt {
int record_error(int code, const std::string &m);  // capi.cpp (jsrt_last_error)
}

namespace {
using namespace jsrt::objp;

// ---------------------------------------------------------------- JS number parsing / Vec helpers
inline bool js_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// Number.parseFloat (ECMA-262 §19.2.4): longest prefix that is a StrDecimalLiteral, else NaN.
// strtod accepts more (hex, "inf", "nan"), so those prefixes are screened first.
double js_parse_float(const std::string &t) {
    size_t i = 0;
    while (i < t.size() && js_space(t[i])) ++i;
    const char *s = t.c_str() + i;
    const char *p = s;
    if (*p == '+' || *p == '-') ++p;
    if (strncmp(p, "Infinity", 8) == 0) return (*s == '-') ? -INFINITY : INFINITY;
    if (!((*p >= '0' && *p <= '9') || (*p == '.' && p[1] >= '0' && p[1] <= '9'))) return NAN;
    // the decimal literal: digits [. digits] [(e|E) [+-] digits]
    const char *q = p;
    while (*q >= '0' && *q <= '9') ++q;
    if (*q == '.') {
        ++q;
        while (*q >= '0' && *q <= '9') ++q;
    }
    if (*q == 'e' || *q == 'E') {
        const char *e = q + 1;
        if (*e == '+' || *e == '-') ++e;
        if (*e >= '0' && *e <= '9') {
            while (*e >= '0' && *e <= '9') ++e;
            q = e;
        }
    }
    std::string lit(s, q);
    return strtod(lit.c_str(), nullptr);  // correctly rounded, like V8
}

// Number.parseInt(x) - 1 on a regex group; a missing or empty group is NaN (objloader.js:139-141).
double js_index(const std::string *g) {
    if (!g || g->empty()) return NAN;
    return strtod(g->c_str(), nullptr) - 1.0;
}

inline float f32(double x) { return (float)x; }
inline float or0(float x) { return (x != x || x == 0.0f) ? 0.0f : x; }  // `x || 0` (math.js:272,275)

struct V4 {
    float v[4];
    int n;  // Vec length
};

// ---------------------------------------------------------------- OBJ text -> triangles
}  // namespace

namespace jsrt {
namespace objp {
void triangle_ctor(Tri &t) {
    float a[3], b[3];
    for (int i = 0; i < 3; ++i) {  // ps[k].minus(ps[0]) is an f32 op per component, then to3()
        a[i] = or0(t.ps[1][i] - t.ps[0][i]);
        b[i] = or0(t.ps[2][i] - t.ps[0][i]);
    }
    // cross (math.js:277-279): f64 products and difference, f32 store
    const float h[3] = {f32((double)a[1] * b[2] - (double)a[2] * b[1]), f32((double)a[2] * b[0] - (double)a[0] * b[2]),
                        f32((double)a[0] * b[1] - (double)a[1] * b[0])};
    const double hn = sqrt((double)h[0] * h[0] + (double)h[1] * h[1] + (double)h[2] * h[2]);
    t.area = hn / 2.0;
    float n[3];
    if (hn > 0.00001) {  // normalized(): times(1 / norm) (math.js:242-245)
        const double s = 1 / hn;
        for (int i = 0; i < 3; ++i) n[i] = f32((double)h[i] * s);
    } else {
        for (int i = 0; i < 3; ++i) n[i] = h[i];
    }
    t.normal[0] = n[0];  // to4(0)
    t.normal[1] = or0(n[1]);
    t.normal[2] = or0(n[2]);
    t.normal[3] = 0.0f;
    for (int i = 0; i < 3; ++i) {
        t.v0[i] = a[i];
        t.v1[i] = b[i];
    }
    t.v0[3] = t.v1[3] = 0.0f;
    t.delta = (double)t.normal[0] * t.ps[0][0] + (double)t.normal[1] * t.ps[0][1] + (double)t.normal[2] * t.ps[0][2] +
              (double)t.normal[3] * t.ps[0][3];
    t.d00 = (double)a[0] * a[0] + (double)a[1] * a[1] + (double)a[2] * a[2];
    t.d11 = (double)b[0] * b[0] + (double)b[1] * b[1] + (double)b[2] * b[2];
    t.d01 = (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2];
    t.denom = t.d00 * t.d11 - t.d01 * t.d01;
}
}  // namespace objp
}  // namespace jsrt

namespace {

// AABB.fromMinMax centre (math.js:233-235 mix(b, 0.5)) for finite boxes
inline float mid(float lo, float hi) { return f32((1 - 0.5) * lo + 0.5 * (double)hi); }
inline float halfw(float lo, float hi) { return f32((double)(hi - lo) * 0.5); }

// Triangle.getBoundingBox(transform) = AABB.fromPoints(ps.map(p => transform.times(p)))
void triangle_bounds(Tri &t, const double *M) {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 3; ++k) {
        float q[3];
        for (int r = 0; r < 3; ++r)  // Mat x Vec: per-row p.dot(row), 4 terms, f32 store (math.js:392-397)
            q[r] = f32((double)t.ps[k][0] * M[4 * r] + (double)t.ps[k][1] * M[4 * r + 1] +
                       (double)t.ps[k][2] * M[4 * r + 2] + (double)t.ps[k][3] * M[4 * r + 3]);
        for (int i = 0; i < 3; ++i) {
            if (q[i] < mn[i]) mn[i] = q[i];
            if (q[i] > mx[i]) mx[i] = q[i];
        }
    }
    for (int i = 0; i < 3; ++i) {
        if (!isfinite(mn[i]) || !isfinite(mx[i])) fail("Infinite objects not allowed in");  // aggregates.js:38-39
        t.bmin[i] = mn[i];
        t.bmax[i] = mx[i];
        t.bcenter[i] = mid(mn[i], mx[i]);
    }
}

// Tokens of one line: l.match(/\S+/g)
void tokenize(const char *b, const char *e, std::vector<std::string> &out) {
    out.clear();
    const char *p = b;
    while (p < e) {
        while (p < e && js_space(*p)) ++p;
        const char *s = p;
        while (p < e && !js_space(*p)) ++p;
        if (p > s) out.emplace_back(s, p);
    }
}

// parseIndices (objloader.js:139-142): t.match(/(\d+)(?:\/(\d*)(?:\/(\d+))?)?/) per face token.
struct Idx {
    double v, t, n;  // parseInt - 1 (NaN when absent)
};
Idx parse_index(const std::string &tok) {
    size_t i = 0;
    while (i < tok.size() && !(tok[i] >= '0' && tok[i] <= '9')) ++i;
    if (i == tok.size()) fail("Error while attempting to parse obj face token \"" + tok + "\"");
    size_t j = i;
    while (j < tok.size() && tok[j] >= '0' && tok[j] <= '9') ++j;
    std::string g1 = tok.substr(i, j - i), g2, g3;
    bool has2 = false, has3 = false;
    if (j < tok.size() && tok[j] == '/') {
        has2 = true;
        size_t k = j + 1;
        while (k < tok.size() && tok[k] >= '0' && tok[k] <= '9') ++k;
        g2 = tok.substr(j + 1, k - j - 1);
        if (k < tok.size() && tok[k] == '/' && k + 1 < tok.size() && tok[k + 1] >= '0' && tok[k + 1] <= '9') {
            size_t m = k + 1;
            while (m < tok.size() && tok[m] >= '0' && tok[m] <= '9') ++m;
            g3 = tok.substr(k + 1, m - k - 1);
            has3 = true;
        }
    }
    return Idx{js_index(&g1), has2 ? js_index(&g2) : NAN, has3 ? js_index(&g3) : NAN};
}

template <class T>
const T &at_index(const std::vector<T> &v, double i, const char *what) {
    if (!(i >= 0) || i >= (double)v.size()) fail(std::string("obj face references a missing ") + what);
    return v[(size_t)i];
}

// ---------------------------------------------------------------- MTL (objloader.js:58-123)
// What makeMaterial (objloader.js:9-20) reads from a newmtl block.  Textures (map_*) are browser-only
// in the reference (createImageBitmap, :33-40) and rejected here.

}  // namespace

namespace jsrt {
namespace objp {
// parseMtlFile (objloader.js:58-123) over the text of every mtllib, in order (loadMtlFiles merges them
// with Object.assign).
void parse_mtl(const char *text, size_t n, MtlLib &lib) {
    std::vector<std::string> t;
    const char *p = text, *end = text + n;
    bool have = false;
    std::string name;
    MtlMat cur;
    auto commit = [&]() {
        if (!have) return;
        auto it = lib.by_name.find(name);
        if (it != lib.by_name.end()) lib.mats[it->second] = cur;
        else {
            lib.by_name[name] = (int32_t)lib.mats.size();
            lib.mats.push_back(cur);
        }
    };
    while (p <= end) {
        const char *e = (const char *)memchr(p, '\n', end - p);
        if (!e) e = end;
        tokenize(p, e, t);
        p = e + 1;
        if (t.empty() || t[0][0] == '#') continue;  // /^\s*($|#)/
        const std::string &k = t[0];
        if (k == "newmtl") {
            commit();
            name = t.size() > 1 ? t[1] : "undefined";
            cur = MtlMat{};
            have = true;
            continue;
        }
        if (!have) fail("material parameter " + k + " before any newmtl");  // curr is null in the reference
        auto num = [&](size_t i) { return i < t.size() ? js_parse_float(t[i]) : NAN; };
        if (k == "Ka" || k == "Kd" || k == "Ks") {  // Vec.of(t[1], t[2], t[3])
            float *dst = k == "Ka" ? cur.Ka : k == "Kd" ? cur.Kd : cur.Ks;
            for (int i = 0; i < 3; ++i) dst[i] = f32(num(1 + i));
            (k == "Ka" ? cur.ka : k == "Kd" ? cur.kd : cur.ks) = true;
        } else if (k == "Ke" || k == "Tf") {
            // stored, never read by makeMaterial
        } else if (k == "Ns" || k == "Ni" || k == "illum" || k == "d" || k == "Tr") {
            // Ni, illum, d and Tr only reach the discarded Fresnel material (objloader.js:16-18) or nothing
            if (k == "Ns") {
                if (t.size() < 2) cur.Ns = NAN;  // curr.Ns = undefined -> smoothness 0
                else {
                    cur.Ns = js_parse_float(t[1]);
                    if (cur.Ns != cur.Ns) fail("non-numeric Ns is not supported: " + t[1]);  // a string smoothness
                }
            }
        } else if (k == "map_Ka" || k == "map_Kd" || k == "map_Ks") {
            fail("MTL textures (" + k + ") are browser-only in the reference and not supported");
        } else {
            fail("Unsupported material parameter: " + k);
        }
    }
    commit();
}

// parseObjFile (objloader.js:144-221) with loadObjFile's minArea filter (:224-231).
void parse_obj(const char *text, size_t n, double min_area, const double *prim_transform, const MtlLib &mtl,
               std::vector<Tri> &tris) {
    int32_t cur_mtl = -1;  // currentMaterial = defaultMaterial
    std::vector<V4> pos, tex, nrm;
    std::vector<std::string> t;
    const char *p = text, *end = text + n;
    while (p <= end) {
        const char *e = (const char *)memchr(p, '\n', end - p);
        if (!e) e = end;
        tokenize(p, e, t);
        const char *line = p;
        p = e + 1;
        if (t.empty() || t[0][0] == '#') continue;  // /^\s*($|#)/
        const std::string &k = t[0];
        if (k == "mtllib") continue;  // the caller passes the mtllib texts (loadMtlFiles)
        if (k == "usemtl") {
            const std::string nm = t.size() > 1 ? t[1] : "undefined";
            auto it = mtl.by_name.find(nm);
            if (it == mtl.by_name.end()) fail("No material defined with name: " + nm);
            cur_mtl = it->second;
            continue;
        }
        if (k == "f") {
            std::vector<Idx> ix;
            for (size_t i = 1; i < t.size(); ++i) ix.push_back(parse_index(t[i]));
            for (size_t i = 2; i < ix.size(); ++i) {
                const Idx abc[3] = {ix[0], ix[i - 1], ix[i]};
                Tri tr;
                for (int c = 0; c < 3; ++c) {
                    const V4 &v = at_index(pos, abc[c].v, "vertex");
                    for (int d = 0; d < 4; ++d) tr.ps[c][d] = v.v[d];
                }
                bool uv = true, nn = true;
                for (int c = 0; c < 3; ++c) {
                    uv = uv && !isnan(abc[c].t);
                    nn = nn && !isnan(abc[c].n);
                }
                if (uv) {
                    tr.has_uv = 1;
                    for (int c = 0; c < 3; ++c) {
                        const V4 &v = at_index(tex, abc[c].t, "texture coordinate");
                        tr.uv_len = v.n;
                        for (int d = 0; d < 4; ++d) tr.uv[c][d] = v.v[d];
                    }
                }
                if (nn) {
                    tr.has_normal = 1;
                    for (int c = 0; c < 3; ++c) {
                        const V4 &v = at_index(nrm, abc[c].n, "normal");
                        for (int d = 0; d < 4; ++d) tr.vn[c][d] = v.v[d];
                    }
                }
                tr.mtl = cur_mtl;
                triangle_ctor(tr);
                if (tr.area >= min_area) {
                    triangle_bounds(tr, prim_transform);
                    tris.push_back(tr);
                }
            }
            continue;
        }
        std::vector<double> f(t.size(), NAN);
        for (size_t i = 1; i < t.size(); ++i) f[i] = js_parse_float(t[i]);
        auto arg = [&](size_t i) { return i < f.size() ? f[i] : NAN; };  // t[i] undefined -> NaN
        auto orz = [](double x) { return (x != x || x == 0) ? 0.0 : x; };
        if (k == "v")
            pos.push_back(V4{{f32(arg(1)), f32(arg(2)), f32(arg(3)), f32(t.size() < 5 ? 1.0 : arg(4))}, 4});
        else if (k == "vt")
            tex.push_back(V4{{f32(arg(1)), f32(orz(arg(2))), f32(orz(arg(3))), 0.0f}, 3});
        else if (k == "vn")
            nrm.push_back(V4{{f32(arg(1)), f32(arg(2)), f32(arg(3)), 0.0f}, 4});
        else if (k == "s" || k == "o" || k == "g" || k == "vp")
            continue;
        else
            fail("Error while attempting to parse obj file on line \"" + std::string(line, e) + "\"");
    }
}
}  // namespace objp
}  // namespace jsrt

namespace {

// ---------------------------------------------------------------- BVH build (aggregates.js:65-185)
struct Box {  // only min/max are state; centre/half are derived as AABB.fromMinMax does
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool empty = true;  // AABB.empty(): half_size (0,0,0) by construction (geometry.js:91-93)
    void add(const float *bmn, const float *bmx) {  // AABB.hull([this, b]): strict compares
        for (int i = 0; i < 3; ++i) {
            if (bmn[i] < mn[i]) mn[i] = bmn[i];
            if (bmx[i] > mx[i]) mx[i] = bmx[i];
        }
        empty = false;
    }
    float half(int i) const { return empty ? 0.0f : halfw(mn[i], mx[i]); }
    float center(int i) const { return empty ? 0.0f : mid(mn[i], mx[i]); }
    // surfaceArea (geometry.js:160-164); AABB.empty() has half_size (0,0,0)
    double area() const {
        const double h0 = half(0), h1 = half(1), h2 = half(2);
        return 4 * (h0 * h1 + h0 * h2 + h1 * h2);
    }
};

// quickSelectStep / median (math.js:95-157), JS `undefined` modelled as NaN (it compares and adds alike).
int js_cmp(double a, double b) { return a < b ? -1 : a > b ? 1 : 0; }
void qs_step(std::vector<double> &arr, long k, long left, long right) {
    auto sw = [&](long i, long j) { std::swap(arr[i], arr[j]); };
    while (right > left) {
        if (right - left > 600) {
            const double n = right - left + 1, m = k - left + 1, z = log(n), s = 0.5 * exp(2 * z / 3);
            const double sd = 0.5 * sqrt(z * s * (n - s) / n) * (m - n / 2 < 0 ? -1 : 1);
            const long nl = std::max(left, (long)floor(k - m * s / n + sd));
            const long nr = std::min(right, (long)floor(k + (n - m) * s / n + sd));
            qs_step(arr, k, nl, nr);
        }
        const double t = arr[k];
        long i = left, j = right;
        sw(left, k);
        if (js_cmp(arr[right], t) > 0) sw(left, right);
        while (i < j) {
            sw(i, j);
            ++i;
            --j;
            while (js_cmp(arr[i], t) < 0) ++i;
            while (js_cmp(arr[j], t) > 0) --j;
        }
        if (js_cmp(arr[left], t) == 0)
            sw(left, j);
        else {
            ++j;
            sw(j, right);
        }
        if (j <= k) left = j + 1;
        if (k <= j) right = j - 1;
    }
}
double quick_select(std::vector<double> &arr, long k) {
    const long right = (long)arr.size() - 1;
    if ((long)arr.size() <= k) arr.resize(k + 1, NAN);  // reads/writes past the end, as a JS array allows
    qs_step(arr, k, 0, right);
    return arr[k];
}
double js_median(std::vector<double> arr) {
    if (arr.empty()) return NAN;
    const long len2 = (long)arr.size() / 2;
    if (arr.size() % 2 == 1) return quick_select(arr, len2);
    const double a = quick_select(arr, len2);
    return (a + quick_select(arr, len2 + 1)) / 2;
}

struct Node {
    Box box;
    int depth;
    bool leaf;
    int lesser = -1, greater = -1;
    std::vector<int32_t> objs;  // leaf members (triangle indices)
};

struct Builder {
    const std::vector<Tri> &T;
    std::vector<Node> nodes;  // pre-order, lesser subtree before greater (the exporter's order)
    explicit Builder(const std::vector<Tri> &t) : T(t) {}

    Box hull(const std::vector<int32_t> &o) const {
        Box b;
        for (int32_t i : o) b.add(T[i].bmin, T[i].bmax);
        return b;
    }

    // split_objects (aggregates.js:89-185); false when objects.length < 2
    bool split(const std::vector<int32_t> &objs, Box &bounds, std::vector<int32_t> &lo, std::vector<int32_t> &hi) {
        if (objs.size() < 2) return false;
        const int B = 8;
        bounds = hull(objs);
        int best_axis = -1;
        double best_sep = INFINITY, best_cost = INFINITY;
        const double sa = bounds.area();
        for (int axis = 0; axis < 3; ++axis) {
            const float h = bounds.half(axis);
            if (h < 0.000001) continue;
            Box bins[B];
            int count[B] = {0};
            for (int32_t o : objs) {
                double bi = floor(B * (((double)T[o].bcenter[axis] - bounds.mn[axis]) / (2 * (double)h)));
                if (bi == B) bi = B - 1;
                if (!(bi >= 0 && bi < B)) fail("BVH bin index out of range");  // JS would throw on bins[bi]
                const int b = (int)bi;
                count[b]++;
                bins[b].add(T[o].bmin, T[o].bmax);
            }
            for (int i = 0; i < B - 1; ++i) {
                Box b0, b1;
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= i; ++j)
                    if (count[j] > 0) {
                        b0.add(bins[j].mn, bins[j].mx);
                        c0 += count[j];
                    }
                for (int j = i + 1; j < B; ++j)
                    if (count[j] > 0) {
                        b1.add(bins[j].mn, bins[j].mx);
                        c1 += count[j];
                    }
                const double cost = .125 + (c0 * b0.area() + c1 * b1.area()) / sa;
                if (cost < best_cost && c0 > 0 && c1 > 0) {
                    best_axis = axis;
                    best_sep = (double)bounds.mn[axis] + ((double)(i + 1) / B) * (2 * (double)h);
                    best_cost = cost;
                }
            }
        }
        if (best_axis < 0) {  // median fallback (aggregates.js:142-162)
            for (int axis = 0; axis < 3; ++axis) {
                std::vector<double> c(objs.size());
                for (size_t i = 0; i < objs.size(); ++i) c[i] = T[objs[i]].bcenter[axis];
                const double med = js_median(c);
                std::vector<int32_t> a0, a1;
                for (int32_t o : objs) (T[o].bcenter[axis] < med ? a0 : a1).push_back(o);
                if (a0.empty() || a1.empty()) continue;  // the cost test needs both sides non-empty
                const double cost = .125 + ((double)a0.size() * hull(a0).area() + (double)a1.size() * hull(a1).area()) / sa;
                if (cost < best_cost) {
                    best_axis = axis;
                    best_sep = med;
                    best_cost = cost;
                }
            }
            if (best_axis < 0) {  // arbitrary middle split (aggregates.js:164-176)
                const size_t m = objs.size() / 2;
                lo.assign(objs.begin(), objs.begin() + m);
                hi.assign(objs.begin() + m, objs.end());
                return true;
            }
        }
        for (int32_t o : objs) ((double)T[o].bcenter[best_axis] < best_sep ? lo : hi).push_back(o);
        return true;
    }

    // BVHAggregateNode.build (aggregates.js:65-87) with maxDepth = Infinity, minNodeSize = 1
    int build(std::vector<int32_t> objs, int depth) {
        const int id = (int)nodes.size();
        nodes.emplace_back();
        nodes[id].depth = depth;
        Box bounds;
        std::vector<int32_t> lo, hi;
        if (objs.size() > 1 && split(objs, bounds, lo, hi)) {
            nodes[id].leaf = false;
            nodes[id].box = bounds;
            objs.clear();
            objs.shrink_to_fit();
            const int l = build(std::move(lo), depth + 1);
            const int g = build(std::move(hi), depth + 1);
            nodes[id].lesser = l;
            nodes[id].greater = g;
        } else {
            nodes[id].leaf = true;
            nodes[id].box = hull(objs);
            nodes[id].objs = std::move(objs);
        }
        return id;
    }
};

// ---------------------------------------------------------------- blob splice
struct Sections {
    std::vector<uint32_t> tags;
    std::vector<std::vector<uint8_t>> data;
    std::vector<uint32_t> counts;
    int find(uint32_t tag) const {
        for (size_t i = 0; i < tags.size(); ++i)
            if (tags[i] == tag) return (int)i;
        return -1;
    }
};

Sections read_blob(const void *blob, size_t n) {
    if (!blob || n < sizeof(jsrt_blob_header)) fail("blob too small", -1);
    const uint8_t *b = (const uint8_t *)blob;
    jsrt_blob_header h;
    memcpy(&h, b, sizeof h);
    if (h.magic != JSRT_MAGIC || h.version != JSRT_VERSION) fail("not a JSRT v1 blob", -1);
    if (sizeof h + (uint64_t)h.n_sections * sizeof(jsrt_section) > n) fail("truncated section table", -1);
    Sections S;
    for (uint32_t i = 0; i < h.n_sections; ++i) {
        jsrt_section s;
        memcpy(&s, b + sizeof h + i * sizeof s, sizeof s);
        if (s.offset > n || s.bytes > n - s.offset) fail("section out of range", -1);
        S.tags.push_back(s.tag);
        S.counts.push_back(s.count);
        S.data.emplace_back(b + s.offset, b + s.offset + s.bytes);
    }
    return S;
}

template <class R>
R *recs(Sections &S, uint32_t tag, uint32_t &count) {
    int i = S.find(tag);
    if (i < 0) {
        S.tags.push_back(tag);
        S.counts.push_back(0);
        S.data.emplace_back();
        i = (int)S.tags.size() - 1;
    }
    if (S.data[i].size() != (size_t)S.counts[i] * sizeof(R)) fail("section size mismatch", -1);
    count = S.counts[i];
    return (R *)S.data[i].data();
}

template <class R>
int32_t append(Sections &S, uint32_t tag, const R &r) {
    const int i = S.find(tag);
    const size_t o = S.data[i].size();
    S.data[i].resize(o + sizeof(R));
    memcpy(S.data[i].data() + o, &r, sizeof(R));
    return (int32_t)S.counts[i]++;
}

std::vector<uint8_t> write_blob(const Sections &S) {
    const size_t hdr = sizeof(jsrt_blob_header) + S.tags.size() * sizeof(jsrt_section);
    size_t off = (hdr + 7) & ~(size_t)7, total = off;
    for (const auto &d : S.data) total += (d.size() + 7) & ~(size_t)7;
    std::vector<uint8_t> out(total, 0);
    jsrt_blob_header h{JSRT_MAGIC, JSRT_VERSION, (uint32_t)S.tags.size(), 0};
    memcpy(out.data(), &h, sizeof h);
    for (size_t i = 0; i < S.tags.size(); ++i) {
        jsrt_section s{S.tags[i], S.counts[i], off, S.data[i].size()};
        memcpy(out.data() + sizeof h + i * sizeof s, &s, sizeof s);
        if (!S.data[i].empty()) memcpy(out.data() + off, S.data[i].data(), S.data[i].size());
        off += (S.data[i].size() + 7) & ~(size_t)7;
    }
    return out;
}

void put4(float *dst, const float *src) { memcpy(dst, src, 16); }

// makeMaterial(data) (objloader.js:9-20) as blob records: the Fresnel / path-tracing material it
// builds for a finite Ni is never returned (missing `return`), so every MTL material is
// PhongMaterial(Vec.of(1,1,1), ambient, diffuse, specular, Ns || 0) with ambient / diffuse / specular
// = Solid(K? given ? K? : Vec.of(0,0,0)) and reflectivity = transmissivity = Scaled(White, 0)
// (PhongMaterial defaults, materials.js:196-205).  Encoded as jsraytracer_amd/js/scene_blob.js does.
int32_t mtl_material(Sections &S, const MtlMat &m, int32_t &white) {
    auto solid = [&](const float *v) {
        jsrt_rec_mcolor r;
        memset(&r, 0, sizeof r);
        r.kind = JSRT_MC_SOLID;
        r.a = r.b = -1;
        r.len = 3;
        for (int i = 0; i < 3; ++i) r.vec[i] = v[i];
        return append(S, JSRT_SEC_MCOLOR, r);
    };
    static const float one[3] = {1, 1, 1}, zero[3] = {0, 0, 0};
    if (white < 0) white = solid(one);  // SolidMaterialColor.White (shared)
    auto scaled0 = [&]() {
        jsrt_rec_mcolor r;
        memset(&r, 0, sizeof r);
        r.kind = JSRT_MC_SCALED_SCALAR;
        r.a = white;
        r.b = -1;
        r.scalar = 0.0;
        return append(S, JSRT_SEC_MCOLOR, r);
    };
    jsrt_rec_material M;
    memset(&M, 0, sizeof M);
    M.kind = JSRT_MAT_PHONG;
    M.base = solid(one);
    M.ambient = solid(m.ka ? m.Ka : zero);
    M.diffuse = solid(m.kd ? m.Kd : zero);
    M.specular = solid(m.ks ? m.Ks : zero);
    M.reflect = scaled0();
    M.transmit = scaled0();
    M.color = -1;
    M.smoothness = (m.Ns != m.Ns || m.Ns == 0) ? 0.0 : m.Ns;  // data.Ns || 0
    M.ratio = 1;
    M.mirror_prob = 0;
    M.opacity = 0;
    return append(S, JSRT_SEC_MATERIAL, M);
}

void splice(const void *blob, size_t n, const jsrt_mesh_options *opt, const char *obj, size_t obj_len,
            const char *mtl_text, size_t mtl_len, std::vector<uint8_t> &out, jsrt_mesh_info *info) {
    Sections S = read_blob(blob, n);
    MtlLib mtl;
    for (size_t a = 0; a < mtl_len;) {  // one parseMtlFile per NUL-separated file, merged like Object.assign
        const char *z = (const char *)memchr(mtl_text + a, 0, mtl_len - a);
        const size_t b = z ? (size_t)(z - mtl_text) : mtl_len;
        parse_mtl(mtl_text + a, b - a, mtl);
        a = b + 1;
    }
    uint32_t n_obj, n_bvh, n_chld, n_geom, n_tri, n_mats;
    for (uint32_t tag : {JSRT_SEC_GEOMETRY, JSRT_SEC_OBJECT, JSRT_SEC_CHILD, JSRT_SEC_BVHNODE, JSRT_SEC_TRIANGLE,
                         JSRT_SEC_MATRIX, JSRT_SEC_MCOLOR, JSRT_SEC_MATERIAL})
        if (S.find(tag) < 0) (void)recs<uint8_t>(S, tag, n_obj);  // create missing (empty) sections
    const jsrt_rec_object *O = recs<jsrt_rec_object>(S, JSRT_SEC_OBJECT, n_obj);
    const jsrt_rec_bvhnode *N = recs<jsrt_rec_bvhnode>(S, JSRT_SEC_BVHNODE, n_bvh);
    const int32_t *C = recs<int32_t>(S, JSRT_SEC_CHILD, n_chld);
    const jsrt_rec_geometry *G = recs<jsrt_rec_geometry>(S, JSRT_SEC_GEOMETRY, n_geom);
    (void)recs<jsrt_rec_triangle>(S, JSRT_SEC_TRIANGLE, n_tri);
    const jsrt_rec_matrix *M = recs<jsrt_rec_matrix>(S, JSRT_SEC_MATRIX, n_mats);

    // the target BVHAggregate and its template primitive (one leaf, one Primitive over a Triangle)
    int32_t bo = opt ? opt->bvh_object : -1;
    if (bo < 0)
        for (uint32_t i = 0; i < n_obj && bo < 0; ++i)
            if (O[i].kind == JSRT_OBJ_BVH) bo = (int32_t)i;
    if (bo < 0 || (uint32_t)bo >= n_obj || O[bo].kind != JSRT_OBJ_BVH) fail("no BVHAggregate object to attach to", -1);
    const int32_t r = O[bo].bvh_root;
    if (r < 0 || (uint32_t)r >= n_bvh || !N[r].is_leaf || N[r].n_obj != 1 || N[r].first_obj < 0 ||
        (uint32_t)N[r].first_obj >= n_chld)
        fail("the BVHAggregate must hold exactly one template primitive (one leaf, one object)", -1);
    const int32_t tp = C[N[r].first_obj];
    if (tp < 0 || (uint32_t)tp >= n_obj || O[tp].kind != JSRT_OBJ_PRIMITIVE || O[tp].geometry < 0 ||
        (uint32_t)O[tp].geometry >= n_geom || G[O[tp].geometry].kind != JSRT_GEOM_TRIANGLE)
        fail("the template object must be a Primitive over a Triangle", -1);
    if (O[tp].matrix < 0 || (uint32_t)O[tp].matrix >= n_mats) fail("template primitive has no matrix", -1);
    const jsrt_rec_object tmpl = O[tp];
    double pm[16];
    memcpy(pm, M[tmpl.matrix].m, sizeof pm);

    std::vector<Tri> tris;
    const double min_area = opt ? opt->min_area : 0.00001;
    parse_obj(obj, obj_len, min_area, pm, mtl, tris);
    if (tris.empty()) fail("the OBJ text holds no triangle of at least min_area", -1);

    Builder B(tris);
    std::vector<int32_t> all(tris.size());
    for (size_t i = 0; i < tris.size(); ++i) all[i] = (int32_t)i;
    B.build(std::move(all), 0);

    // records: geometry + triangle + primitive per triangle, nodes in pre-order
    std::vector<int32_t> prim_of(tris.size()), mat_of(mtl.mats.size(), -1);
    int32_t white = -1;
    for (size_t i = 0; i < tris.size(); ++i) {
        const Tri &t = tris[i];
        jsrt_rec_triangle tr;
        memset(&tr, 0, sizeof tr);
        for (int k = 0; k < 3; ++k) put4(tr.p[k], t.ps[k]);
        put4(tr.v0, t.v0);
        put4(tr.v1, t.v1);
        put4(tr.normal, t.normal);
        tr.delta = t.delta;
        tr.d00 = t.d00;
        tr.d11 = t.d11;
        tr.d01 = t.d01;
        tr.denom = t.denom;
        tr.area = t.area;
        tr.has_normal = (uint32_t)t.has_normal;
        tr.has_uv = (uint32_t)t.has_uv;
        tr.uv_len = t.has_uv ? (uint32_t)t.uv_len : 0;
        for (int k = 0; k < 3; ++k) {
            put4(tr.vn[k], t.vn[k]);
            put4(tr.uv[k], t.uv[k]);
        }
        jsrt_rec_geometry g;
        memset(&g, 0, sizeof g);
        g.kind = JSRT_GEOM_TRIANGLE;
        g.index = append(S, JSRT_SEC_TRIANGLE, tr);
        jsrt_rec_object o = tmpl;
        o.geometry = append(S, JSRT_SEC_GEOMETRY, g);
        if (t.mtl >= 0) {  // usemtl: the MTL material (one record per material used)
            if (mat_of[t.mtl] < 0) mat_of[t.mtl] = mtl_material(S, mtl.mats[t.mtl], white);
            o.material = mat_of[t.mtl];
        }
        prim_of[i] = append(S, JSRT_SEC_OBJECT, o);
    }
    uint32_t base;
    (void)recs<jsrt_rec_bvhnode>(S, JSRT_SEC_BVHNODE, base);
    int max_depth = 0;
    for (const Node &nd : B.nodes) {
        jsrt_rec_bvhnode rec;
        memset(&rec, 0, sizeof rec);
        for (int i = 0; i < 3; ++i) {
            rec.center[i] = nd.box.center(i);
            rec.half[i] = nd.box.half(i);
        }
        rec.center[3] = 1.0f;  // mix of the w = 1 corners; half w = 0
        rec.half[3] = 0.0f;
        rec.is_leaf = nd.leaf ? 1u : 0u;
        rec.lesser = nd.leaf ? -1 : (int32_t)base + nd.lesser;
        rec.greater = nd.leaf ? -1 : (int32_t)base + nd.greater;
        rec.depth = nd.depth;
        max_depth = std::max(max_depth, nd.depth);
        if (nd.leaf) {
            uint32_t nc;
            (void)recs<int32_t>(S, JSRT_SEC_CHILD, nc);
            rec.first_obj = (int32_t)nc;
            rec.n_obj = (int32_t)nd.objs.size();
            for (int32_t o : nd.objs) append(S, JSRT_SEC_CHILD, prim_of[o]);
        } else {
            rec.first_obj = 0;
            rec.n_obj = 0;
        }
        append(S, JSRT_SEC_BVHNODE, rec);
    }
    // every BVHAggregate over the template tree gets the new one: `new BVHAggregate(objs, tie1.kdtree, T)`
    // instances share a tree (tests/starwars/test.mjs); the old template tree is now unreferenced
    jsrt_rec_object *Ow = recs<jsrt_rec_object>(S, JSRT_SEC_OBJECT, n_obj);
    for (uint32_t i = 0; i < n_obj; ++i)
        if (Ow[i].kind == JSRT_OBJ_BVH && Ow[i].bvh_root == r) Ow[i].bvh_root = (int32_t)base;
    out = write_blob(S);
    if (info) {
        memset(info, 0, sizeof *info);
        info->triangles = (int64_t)tris.size();
        info->nodes = (int64_t)B.nodes.size();
        info->max_depth = max_depth;
        info->bvh_object = bo;
    }
}

}  // namespace

extern "C" {

int jsrt_blob_attach_obj(const void *blob, size_t n, const char *obj_text, size_t obj_len,
                         const jsrt_mesh_options *options, void **out_blob, size_t *out_n, jsrt_mesh_info *info) {
    return jsrt_blob_attach_obj_mtl(blob, n, obj_text, obj_len, nullptr, 0, options, out_blob, out_n, info);
}

int jsrt_blob_attach_obj_mtl(const void *blob, size_t n, const char *obj_text, size_t obj_len, const char *mtl_text,
                             size_t mtl_len, const jsrt_mesh_options *options, void **out_blob, size_t *out_n,
                             jsrt_mesh_info *info) {
    if (!out_blob || !out_n) return jsrt::record_error(-1, "out_blob / out_n is NULL");
    *out_blob = nullptr;
    *out_n = 0;
    if (!obj_text && obj_len) return jsrt::record_error(-1, "obj_text is NULL");
    try {
        std::vector<uint8_t> out;
        if (!mtl_text && mtl_len) return jsrt::record_error(-1, "mtl_text is NULL");
        splice(blob, n, options, obj_text ? obj_text : "", obj_len, mtl_text, mtl_len, out, info);
        void *p = malloc(out.size());
        if (!p) return jsrt::record_error(-4, "out of host memory");
        memcpy(p, out.data(), out.size());
        *out_blob = p;
        *out_n = out.size();
        return 0;
    } catch (const Fail &f) {
        return jsrt::record_error(f.code, f.msg);
    } catch (const std::bad_alloc &) {
        return jsrt::record_error(-4, "out of host memory");
    }
}

void jsrt_blob_free(void *p) { free(p); }

}  // extern "C"
