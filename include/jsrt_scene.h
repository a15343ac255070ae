/*
 * jsrt_scene.h — binary scene blob ("JSRT" v1): the wire format that crosses the drop-in
 * boundary between the JS host (the reference's live scene graph) and libjsrt.
 *
 * It carries exactly what the reference's render path reads from the scene graph:
 *   renderer   src/renderers.js:1-118     (kind, samplesPerPixel, maxRecursionDepth) + PixelBuffer W,H
 *   camera     src/cameras.js:18-53        (transform, tan_fov, aspect, DOF focus/sensor)
 *   world      src/world.js:1-141          (objects, lights, bg_color; Primitive/TransformedWorldObject)
 *   aggregates src/aggregates.js:1-232     (Aggregate, BVHAggregate + BVHAggregateNode topology)
 *   geometry   src/geometry.js:77-488      (AABB/UnitBox, SimplePlane/Plane, Square, Circle, Triangle,
 *                                           Sphere, Cylinder)
 *   sdf        src/sdf.js:1-477            (SDFGeometry + SDF tree + transformers)
 *   materials  src/materials.js:1-476      (MaterialColor trees, Phong/Fresnel/PathTracing/...)
 *   lights     src/lights.js:27-94         (SimplePointLight, RandomSampleAreaLight)
 *
 * The reference's own wire format (src/serializer.js JSON) is lossy on this path (drops triangle
 * vertex normals, geometry.js:355-357; rebuilds PhongPathTracingMaterial as Fresnel,
 * materials.js:394-396; Infinity -> null), so the host exporter (jsraytracer_amd/js/scene_blob.js)
 * walks the live objects instead and writes this blob.  Every float field is the exact bit
 * pattern the reference holds (Vec = Float32Array, Mat rows = float64).
 *
 * Layout: header, then n_sections section descriptors, then section payloads (8-byte aligned).
 * All integers little-endian.  Records are fixed-size C structs (static_asserted below).
 */
#ifndef JSRT_SCENE_H
#define JSRT_SCENE_H
#include <stdint.h>

#define JSRT_MAGIC 0x5452534Au /* "JSRT" */
#define JSRT_VERSION 1u

#define JSRT_FOURCC(a, b, c, d) \
    ((uint32_t)(a) | ((uint32_t)(b) << 8) | ((uint32_t)(c) << 16) | ((uint32_t)(d) << 24))
#define JSRT_SEC_RENDERER JSRT_FOURCC('R', 'N', 'D', 'R')
#define JSRT_SEC_CAMERA JSRT_FOURCC('C', 'A', 'M', 'R')
#define JSRT_SEC_MCOLOR JSRT_FOURCC('M', 'C', 'O', 'L')
#define JSRT_SEC_MATERIAL JSRT_FOURCC('M', 'A', 'T', 'L')
#define JSRT_SEC_GEOMETRY JSRT_FOURCC('G', 'E', 'O', 'M')
#define JSRT_SEC_OBJECT JSRT_FOURCC('O', 'B', 'J', 'S')
#define JSRT_SEC_MATRIX JSRT_FOURCC('M', 'A', 'T', 'S')
#define JSRT_SEC_ROOT JSRT_FOURCC('R', 'O', 'O', 'T')
#define JSRT_SEC_CHILD JSRT_FOURCC('C', 'H', 'L', 'D')
#define JSRT_SEC_BVHNODE JSRT_FOURCC('B', 'V', 'H', 'N')
#define JSRT_SEC_TRIANGLE JSRT_FOURCC('T', 'R', 'I', 'S')
#define JSRT_SEC_LIGHT JSRT_FOURCC('L', 'I', 'T', 'E')
#define JSRT_SEC_SDFNODE JSRT_FOURCC('S', 'D', 'F', 'N')
#define JSRT_SEC_SDFGEOM JSRT_FOURCC('S', 'D', 'F', 'G')

/* renderer kinds: renderers.js:1 SimpleRenderer, :65 IncrementalMultisamplingRenderer,
 * :47 RandomMultisamplingRenderer */
enum { JSRT_RENDERER_SIMPLE = 0, JSRT_RENDERER_INCREMENTAL = 1, JSRT_RENDERER_RANDOM = 2 };
/* camera kinds: cameras.js:18 PerspectiveCamera, :40 DepthOfFieldPerspectiveCamera */
enum { JSRT_CAMERA_PERSPECTIVE = 0, JSRT_CAMERA_DOF = 1 };
/* material colours: materials.js:27 Solid, :43 Scaled (number or Vec scale), :63 Checkerboard */
enum { JSRT_MC_SOLID = 1, JSRT_MC_SCALED_SCALAR = 2, JSRT_MC_SCALED_VEC = 3, JSRT_MC_CHECKER = 4 };
/* materials: materials.js:195 Phong, :294 FresnelPhong, :389 PhongPathTracing, :145 SolidColor,
 * :160 Transparent */
enum {
    JSRT_MAT_PHONG = 1,
    JSRT_MAT_FRESNEL = 2,
    JSRT_MAT_PATH = 3,
    JSRT_MAT_SOLID = 4,
    JSRT_MAT_TRANSPARENT = 5
};
/* geometry: geometry.js:239 SimplePlane (and :257 Plane), :280 Square, :303 Circle, :412 Sphere,
 * :458 Cylinder, :77 AABB (:230 UnitBox), :334 Triangle, sdf.js:1 SDFGeometry */
enum {
    JSRT_GEOM_PLANE = 1,
    JSRT_GEOM_SQUARE = 2,
    JSRT_GEOM_CIRCLE = 3,
    JSRT_GEOM_SPHERE = 4,
    JSRT_GEOM_CYLINDER = 5,
    JSRT_GEOM_AABB = 6,
    JSRT_GEOM_TRIANGLE = 7,
    JSRT_GEOM_SDF = 8
};
/* world objects: world.js:104 Primitive, aggregates.js:1 Aggregate, :26 BVHAggregate,
 * world.js:82 TransformedWorldObject */
enum { JSRT_OBJ_PRIMITIVE = 1, JSRT_OBJ_AGGREGATE = 2, JSRT_OBJ_BVH = 3, JSRT_OBJ_TRANSFORMED = 4 };
/* lights: lights.js:27 SimplePointLight, :56 RandomSampleAreaLight */
enum { JSRT_LIGHT_POINT = 1, JSRT_LIGHT_AREA = 2 };
/* SDF nodes (sdf.js) and SDF transformers (sdf.js:370-477) share one table */
enum {
    JSRT_SDF_UNION = 1,              /* :78  children list */
    JSRT_SDF_INTERSECTION = 2,       /* :94  children list */
    JSRT_SDF_DIFFERENCE = 3,         /* :110 a=positive b=negative */
    JSRT_SDF_SMOOTH_UNION = 4,       /* :139 a b k */
    JSRT_SDF_SMOOTH_INTERSECTION = 5,/* :160 a b k */
    JSRT_SDF_SMOOTH_DIFFERENCE = 6,  /* :181 a b k */
    JSRT_SDF_ROUND = 7,              /* :204 a k=rounding */
    JSRT_SDF_SPHERE = 8,             /* :226 k=radius basecolor */
    JSRT_SDF_BOX = 9,                /* :266 vec=size(to4(0)) basecolor */
    JSRT_SDF_TETRAHEDRON = 10,       /* :295 basecolor */
    JSRT_SDF_TRANSFORM = 11,         /* :324 a=child b=transformer */
    JSRT_SDF_RECURSIVE_UNION = 12,   /* :342 a=sdf b=transformer iterations */
    JSRT_SDFT_SEQUENCE = 20,         /* :382 children list of transformers */
    JSRT_SDFT_RECURSIVE = 21,        /* :402 a=transformer iterations */
    JSRT_SDFT_MATRIX = 22,           /* :423 m=transform minv=inverse k=scale */
    JSRT_SDFT_REFLECTION = 23,       /* :441 vec=normal k=delta */
    JSRT_SDFT_REPETITION = 24        /* :466 vec=sizes */
};

typedef struct {
    uint32_t magic, version, n_sections, reserved;
} jsrt_blob_header;

typedef struct {
    uint32_t tag, count;
    uint64_t offset, bytes; /* offset from blob start; bytes = count * record size */
} jsrt_section;

typedef struct { /* RNDR: exactly one */
    uint32_t kind, spp, max_depth, width, height;
    uint32_t bg_len; /* Vec length of World.bg_color (3 in every scene) */
    float bg[4];
    uint32_t pad[2];
} jsrt_rec_renderer;

typedef struct { /* CAMR: exactly one */
    uint32_t kind, pad;
    double transform[16]; /* Mat rows, row-major */
    double tan_fov, aspect, focus_distance, sensor_size;
} jsrt_rec_camera;

typedef struct { /* MCOL */
    uint32_t kind;
    int32_t a, b;
    uint32_t len; /* Vec length of vec[] */
    float vec[4];
    double scalar;
} jsrt_rec_mcolor;

typedef struct { /* MATL */
    uint32_t kind;
    int32_t base, ambient, diffuse, specular, reflect, transmit, color; /* MCOL idx or -1 */
    double smoothness, ratio, mirror_prob, opacity;
} jsrt_rec_material;

typedef struct { /* GEOM */
    uint32_t kind;
    int32_t index; /* TRIS idx (triangle) / SDFG idx (sdf) */
    uint32_t pad[2];
    float center[4], half[4]; /* AABB / UnitBox */
} jsrt_rec_geometry;

typedef struct { /* OBJS */
    uint32_t kind;
    int32_t geometry, material;
    uint32_t casts_shadow;
    int32_t first_child, n_children; /* CHLD range: aggregate members / transformed object */
    int32_t bvh_root;                /* BVHN idx */
    int32_t matrix;                  /* MATS idx: transform + inverse */
} jsrt_rec_object;

typedef struct { /* MATS */
    double m[16], inv[16];
} jsrt_rec_matrix;

typedef struct { /* BVHN */
    float center[4], half[4];
    uint32_t is_leaf;
    int32_t lesser, greater; /* BVHN idx */
    int32_t first_obj, n_obj; /* CHLD range of OBJS idx (leaf) */
    int32_t depth;
    uint32_t pad[2];
} jsrt_rec_bvhnode;

typedef struct { /* TRIS (geometry.js:334-354: ps, v0, v1, normal, delta, d00, d11, d01, denom) */
    float p[3][4];
    float v0[4], v1[4], normal[4];
    double delta, d00, d11, d01, denom, area;
    uint32_t has_normal, has_uv, uv_len, pad;
    float vn[3][4];
    float uv[3][4];
} jsrt_rec_triangle;

typedef struct { /* LITE */
    uint32_t kind;
    int32_t color; /* MCOL idx of light.color_mc */
    uint32_t geometry_kind, samples;
    float position[4];
    uint32_t pos_len, pad[3];
    double transform[16], inv[16];
} jsrt_rec_light;

typedef struct { /* SDFN */
    uint32_t kind;
    int32_t a, b, first, count, iterations;
    double k;
    float vec[4];
    float basecolor[4];
    uint32_t basecolor_len, pad[3];
    double m[16], minv[16];
} jsrt_rec_sdfnode;

typedef struct { /* SDFG (sdf.js:3-11) */
    int32_t root, max_samples;
    double eps, max_trace, normal_step;
    float center[4], half[4]; /* root_sdf.getBoundingBox(I, I) */
} jsrt_rec_sdfgeom;

#ifdef __cplusplus
#define JSRT_STATIC_ASSERT static_assert
#else
#define JSRT_STATIC_ASSERT _Static_assert
#endif
JSRT_STATIC_ASSERT(sizeof(jsrt_blob_header) == 16, "header");
JSRT_STATIC_ASSERT(sizeof(jsrt_section) == 24, "section");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_renderer) == 48, "renderer");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_camera) == 168, "camera");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_mcolor) == 40, "mcolor");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_material) == 64, "material");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_geometry) == 48, "geometry");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_object) == 32, "object");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_matrix) == 256, "matrix");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_bvhnode) == 64, "bvhnode");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_triangle) == 256, "triangle");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_light) == 304, "light");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_sdfnode) == 336, "sdfnode");
JSRT_STATIC_ASSERT(sizeof(jsrt_rec_sdfgeom) == 64, "sdfgeom");

#endif
