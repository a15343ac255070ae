/*
 * jsrt_mesh.h — native mesh ingest for libjsrt: OBJ text -> Triangle primitives -> BVHAggregate,
 * spliced into a JSRT scene blob (include/jsrt_scene.h).  Host-only (never touches the GPU).
 *
 * Reference interfaces replaced (alitteneker/jsraytracer):
 *   jsrt_blob_attach_obj <- loadObjFile(filename, defaultMaterial, callback, transform, minArea)
 *                           (src/objloader.js:224-231) -> parseObjFile (:144-221: v / vt / vn / f,
 *                           fan triangulation, Triangle ctor geometry.js:335-354, `area >= minArea`
 *                           filter, each triangle wrapped in Primitive(tri, material, transform))
 *                           followed by BVHAggregate.build(triangles, transform) (src/aggregates.js:33-41)
 *                           -> BVHAggregateNode.build / split_objects (:65-185: 8-bin SAH per axis,
 *                           median fallback, middle split), maxDepth = Infinity, minNodeSize = 1.
 *                           The tree is bit-identical to the reference's (same node boxes, same
 *                           lesser/greater children, same leaf order) so closest-hit ties break alike.
 *   jsrt_blob_free        <- (memory returned by jsrt_blob_attach_obj)
 *
 * The blob names the target: a BVHAggregate object (OBJS kind JSRT_OBJ_BVH; options->bvh_object, or
 * the first one when < 0) whose tree is ONE leaf holding ONE template Primitive over a Triangle.  The
 * template supplies what loadObjFile's caller passes: the material, the per-triangle Primitive
 * transform (and inverse) and does_cast_shadow.  The BVHAggregate's own transform is kept.  Every
 * triangle of the OBJ becomes a copy of the template with its own Triangle geometry; the template's
 * old one-leaf tree stays in the blob, unreferenced.
 *
 * Errors: negative return, message in jsrt_last_error of jsrt.h (the reference throws strings, e.g.
 * objloader.js:217 "Error while attempting to parse obj file on line ...", aggregates.js:39).
 *
 * jsrt_blob_attach_obj_mtl <- the same with the OBJ's mtllib files (loadMtlFiles / parseMtlFile,
 *                           objloader.js:58-137; the text of each file in mtllib order,
 *                           separated by NUL bytes): `usemtl`
 *                           switches the current material to makeMaterial(newmtl block)
 *                           (objloader.js:9-20, always a PhongMaterial: the Fresnel / path-tracing one
 *                           is built and dropped), faces before any usemtl take the template's material
 *                           (loadObjFile's defaultMaterial).  Without MTL text, usemtl throws "No
 *                           material defined with name: ..." as the reference does for a missing one.
 *                           Every BVHAggregate sharing the template tree receives the built tree.
 */
#ifndef JSRT_MESH_H
#define JSRT_MESH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t bvh_object; /* OBJS index of the target BVHAggregate; < 0: the first BVHAggregate */
    int32_t pad;
    double min_area;    /* loadObjFile minArea (objloader.js:224 default 0.00001) */
} jsrt_mesh_options;

typedef struct {
    int64_t triangles; /* triangles kept (area >= min_area) */
    int64_t nodes;     /* BVH nodes (BVHAggregate.nodeCount(), aggregates.js:230) */
    int32_t max_depth; /* BVHAggregate.maxDepth() (aggregates.js:227) */
    int32_t bvh_object;
} jsrt_mesh_info;

/* Returns 0 and a malloc'd blob in *out_blob / *out_n (free with jsrt_blob_free), or negative.
 * options and info may be NULL (defaults: first BVHAggregate, min_area 0.00001). */
int jsrt_blob_attach_obj(const void *blob, size_t n, const char *obj_text, size_t obj_len,
                         const jsrt_mesh_options *options, void **out_blob, size_t *out_n, jsrt_mesh_info *info);
int jsrt_blob_attach_obj_mtl(const void *blob, size_t n, const char *obj_text, size_t obj_len, const char *mtl_text,
                             size_t mtl_len, const jsrt_mesh_options *options, void **out_blob, size_t *out_n,
                             jsrt_mesh_info *info);
void jsrt_blob_free(void *blob);

#ifdef __cplusplus
}
#endif
#endif
