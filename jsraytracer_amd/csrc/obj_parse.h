// Host-side OBJ / MTL parsing and the Triangle constructor shared by the native mesh ingest
// (mesh_build.cpp, include/jsrt_mesh.h) and the Serializer-JSON reader (json_scene.cpp,
// include/jsrt_json.h).  Internal to libjsrt: no C-ABI.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace jsrt {
namespace objp {

struct Fail {  // thrown by the parsers; the C-ABI entry points turn it into jsrt_last_error
    int code;
    std::string msg;
};
[[noreturn]] inline void fail(const std::string &m, int code = -2) { throw Fail{code, m}; }

// One Triangle as loadObjFile makes it (objloader.js:195-212) plus its constructor results.
struct Tri {
    int32_t mtl = -1;  // MTL material (index into the parsed list) or -1: loadObjFile's defaultMaterial
    float ps[3][4];
    int has_normal = 0, has_uv = 0, uv_len = 0;
    float vn[3][4] = {}, uv[3][4] = {};
    // Triangle constructor results (geometry.js:335-354)
    float v0[4], v1[4], normal[4];
    double delta, d00, d11, d01, denom, area;
    // Primitive.getBoundingBox (world.js:138-140 -> geometry.js:378-380 -> AABB.fromPoints)
    float bmin[4], bmax[4], bcenter[4];
};

// What makeMaterial (objloader.js:9-20) reads from a newmtl block.
struct MtlMat {
    bool ka = false, kd = false, ks = false;
    float Ka[3] = {0, 0, 0}, Kd[3] = {0, 0, 0}, Ks[3] = {0, 0, 0};
    double Ns = 0.0 / 0.0;  // NaN: absent (`data.Ns || 0`)
};
struct MtlLib {
    std::vector<MtlMat> mats;
    std::map<std::string, int32_t> by_name;  // ret[name] = ...: a later definition replaces an earlier one
};

// Triangle constructor (geometry.js:335-354) in the reference's numeric model.
void triangle_ctor(Tri &t);
// parseMtlFile (objloader.js:58-123), merged into `lib`.
void parse_mtl(const char *text, size_t n, MtlLib &lib);
// parseObjFile (objloader.js:144-221) with loadObjFile's minArea filter (:224-231); prim_transform
// (16 doubles, row-major) is the per-triangle Primitive transform the bounds are taken under, or null.
void parse_obj(const char *text, size_t n, double min_area, const double *prim_transform, const MtlLib &mtl,
               std::vector<Tri> &tris);

}  // namespace objp
}  // namespace jsrt
