/*
 * jsrt.h — C-ABI of libjsrt, the MI355X (gfx950) renderer that drops in for the reference's CPU
 * web-worker render path.
 *
 * Reference interfaces replaced (alitteneker/jsraytracer):
 *   jsrt_scene_create   <- the worker building its scene graph (src/worker.js:23-24 import +
 *                          configureTest) and handing it to the renderer; the scene arrives as the
 *                          JSRT blob of include/jsrt_scene.h (host exporter:
 *                          jsraytracer_amd/js/scene_blob.js, in place of src/serializer.js:12-60)
 *   jsrt_render         <- SimpleRenderer.render / IncrementalMultisamplingRenderer.render
 *                          (src/renderers.js:10-41, 70-117): render(img, timelimit, callback,
 *                          x_offset, x_delt) writing PixelBuffer RGBA8 (src/pixelbuffer.js:39-49),
 *                          progress callback({pass, completion}) (renderers.js:35,110)
 *   jsrt_render_device  <- same, device-resident outputs on a caller stream (multi-GPU tile path)
 *   jsrt_cast           <- World.cast (src/world.js:28-30) for a batch of rays: closest-hit distance
 *                          and the hit Primitive (known-answer tests localise parity to one cast)
 *   jsrt_material_data  <- World.color(ray, 1) up to Material.color (world.js:31-41, 125-137):
 *                          Geometry.materialData + the world normal / position of each hit
 *   jsrt_sdf_distance   <- SDF.distance (src/sdf.js:53-74) of an SDFGeometry primitive's root
 *   jsrt_scene_destroy  <- worker teardown (src/raytrace_launcher.js:106-124 terminate)
 *   jsrt_last_error     <- the reference throws strings (e.g. src/aggregates.js:39); errors here are
 *                          negative return codes + this message, never C++ exceptions.
 *
 * Threading: renders of one scene are re-entrant; each call uses its own device buffers.
 * Ownership: the caller owns host output buffers; the library owns device memory and the scene.
 */
#ifndef JSRT_H
#define JSRT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JSRT_ABI_VERSION 4

typedef struct jsrt_scene jsrt_scene;

typedef struct {
    int32_t width, height;   /* <= 0: the blob's PixelBuffer size */
    int32_t spp;             /* <= 0: renderer.samplesPerPixel from the blob */
    int32_t max_depth;       /* <= 0: renderer.maxRecursionDepth from the blob */
    int32_t kind;            /* < 0: blob's renderer; 0 Simple, 1 Incremental, 2 RandomMultisampling */
    uint32_t seed;           /* keyed RNG seed (DESIGN.md "keyed RNG") */
    int32_t x_offset, x_delt;/* reference column partition (renderers.js:21,88); x_delt <= 0 -> 1 */
    int32_t device;          /* HIP device ordinal */
    int32_t samples_per_launch; /* progress granularity: samples per pixel between callbacks (<=0: all) */
    double timelimit_ms;     /* progress callback cadence (renderers.js:28-37); 0 = no callback */
    int32_t max_paths;       /* wavefront batch size in paths (<= 0: library default) */
    int32_t stage_events;    /* with stats: bitmask of the stages whose launches are bracketed by HIP
                                events (bit k -> stage_ms[k]); 0 = all.  Events cost launch gaps.
                                | JSRT_EVENTS_ONE_STREAM: run the render on one stream, so that a launch's
                                event interval is its own time (consecutive batches otherwise overlap on
                                two streams). */
    int32_t mode;            /* JSRT_MODE_STRICT (0): the reference's numeric model, f64 scalars and f32 vectors
                                (the only mode built; SURVEY §7's pure-f32 `fast` mode fails the 1e-5 bar on
                                0.35-2.6 % of pixels and is refused: -1) */
    uint32_t device_mask;    /* HIP devices that render this call's columns (bit d = device d; 0 = the scene's
                                device).  jsrt_render only: the owned columns are interleaved over the k devices
                                (device j takes x_offset + j * x_delt, step x_delt * k: the reference's own
                                worker partition, renderers.js:88), each rendering from its own copy of the
                                scene, and the host image is composited -- bit-identical to one device, as
                                pixels never split.  Progress callbacks need a single device.  The device entry
                                points accept only 0 or the scene's own device. */
    int32_t reserved[2];
} jsrt_params;

#define JSRT_MODE_STRICT 0
#define JSRT_MODE_FAST 1

#define JSRT_EVENTS_ONE_STREAM ((int32_t)0x40000000)
#define JSRT_STAGES 12
typedef struct {
    double kernel_ms;        /* sum of all render-kernel durations (HIP events on the render stream) */
    double total_ms;         /* host wall time of the call */
    uint64_t samples;        /* pixel-samples rendered */
    uint32_t launches;       /* render-kernel launches */
    uint32_t batches;        /* (pixels x samples) batches of the wavefront schedule */
    double stage_ms[JSRT_STAGES];        /* per kernel: gen, extend, shade, shadow, reduce, accum, final,
                                            resolve, 4 spare */
    uint32_t stage_launches[JSRT_STAGES];
    uint32_t attempts;       /* frame attempts: > 1 when a pool / launch bound was outgrown and the frame redone */
    uint32_t events_lost;    /* event pairs whose elapsed time HIP could not report (not in stage_ms) */
} jsrt_stats;

typedef void (*jsrt_progress_fn)(int32_t pass, double completion, void *user);

/* Parse + validate a JSRT blob and upload it to `device`. Returns 0 or negative. */
int jsrt_scene_create(const void *scene_blob, size_t n, int32_t device, jsrt_scene **out);
void jsrt_scene_destroy(jsrt_scene *scene);

/* Render into host buffers.  rgba8 (W*H*4 bytes) receives the PixelBuffer bytes of the rendered
 * columns only (other columns untouched, as each reference worker leaves them); colors_f32
 * (W*H*4, nullable) the final f32 colour handed to setColor (alpha 1).  progress may be NULL.
 * Incremental renderer with progress: before each callback for pass p, rgba8's owned columns hold
 * the running mean of samples 0..p (the img the reference's callback sees, renderers.js:93-112). */
int jsrt_render(jsrt_scene *scene, const jsrt_params *params, uint8_t *rgba8, float *colors_f32,
                jsrt_progress_fn progress, void *user, jsrt_stats *stats);

/* Render the owned columns into DEVICE buffers on `hip_stream` (a hipStream_t, 0 = null stream).
 * Owned columns: px >= x_offset, (px - x_offset) % x_delt == 0, packed in order: owned column c,
 * row py lives at [(c * H + py)] of d_rgba8 (u32 RGBA8) and d_colors (f32x4, nullable).
 * col_block > 1 assigns blocks of col_block columns round-robin (rank = (px / col_block) % x_delt
 * == x_offset) for coherent multi-GPU tiles.  Asynchronous w.r.t. the host. */
int jsrt_render_device(jsrt_scene *scene, const jsrt_params *params, int32_t col_block, uint32_t *d_rgba8,
                       float *d_colors, void *hip_stream, jsrt_stats *stats);

/* jsrt_render_device with progress (the multi-GPU tile path's preview cadence, renderers.js:103-112 /
 * worker.js:30-32): progress(pass, completion) is called at most every params->timelimit_ms (0 = never;
 * a tiny value = after every pass of params->samples_per_launch samples), from the calling thread, with
 * the stream idle.  With the Incremental renderer, d_rgba8 (and d_colors) then hold the running mean of
 * samples 0..pass of the owned columns -- the image the reference worker posts -- so a caller can gather
 * the ranks' tiles inside the callback.  Returns when the frame is done (synchronous). */
int jsrt_render_device_progress(jsrt_scene *scene, const jsrt_params *params, int32_t col_block, uint32_t *d_rgba8,
                                float *d_colors, void *hip_stream, jsrt_progress_fn progress, void *user,
                                jsrt_stats *stats);
/* (Every callback sees a clean preview: the progress check that finds a batch outgrew its device pool or
 * launch bound redoes the frame at once, before that pass is reported, and passes already reported are not
 * reported again -- each pass is reported once, from a clean frame.) */

/* The multi-rank form of jsrt_render_device_progress (jsraytracer_amd/tiles.py render_progressive): progress
 * is called for every pass the frame reports with clean = 1 when the device tile holds that pass's running
 * mean (always, as above; the flag is kept so a caller never has to assume it), so every rank calls back the
 * same passes and can keep its collectives in step (a rank that owns no column still reports each pass).  A
 * non-zero return aborts the frame: the call returns -4 ("render aborted by the progress callback") once the
 * device is idle. */
typedef int32_t (*jsrt_progress_ex_fn)(int32_t pass, double completion, int32_t clean, void *user);
int jsrt_render_device_progress_ex(jsrt_scene *scene, const jsrt_params *params, int32_t col_block, uint32_t *d_rgba8,
                                   float *d_colors, void *hip_stream, jsrt_progress_ex_fn progress, void *user,
                                   jsrt_stats *stats);

/* jsrt_render_device with the renderer's f32 accumulator as the output (the multi-GPU accumulator exchange,
 * jsraytracer_amd/tiles.py AccumGather): d_accum (ncols * H * 4 f32, laid out as d_rgba8 with 4 floats per pixel,
 * w = 0) receives each owned pixel's accumulator before setColor -- Incremental: the f32 sum of its samples in
 * order (renderers.js:93-97), RandomMultisampling: the sum of sample / spp (renderers.js:52-62), Simple: the
 * sample.  No RGBA8 is written.  Asynchronous w.r.t. the host. */
int jsrt_render_device_accum(jsrt_scene *scene, const jsrt_params *params, int32_t col_block, float *d_accum,
                             void *hip_stream, jsrt_stats *stats);

/* setColor of n accumulators (device f32 x 4 each, any pixel order, as jsrt_render_device_accum writes them):
 * the renderer's final colour (kind 1, Incremental: times(1 / passes), renderers.js:98; kinds 0 / 2: the
 * accumulator) and PixelBuffer.setColor's RGBA8 (pixelbuffer.js:39-49) into d_rgba8 (n u32) and d_colors
 * (n x 4 f32, nullable) -- the same k_final every render ends with, so a gathered composite's RGBA8 is the
 * single-GPU frame's bit for bit.  Asynchronous w.r.t. the host. */
int jsrt_finish_accum(const float *d_accum, int64_t n, int32_t kind, int32_t passes, uint32_t *d_rgba8,
                      float *d_colors, void *hip_stream);

/* World.cast(ray, min_dist, max_dist, intersect_transparent) (world.js:28-30) of n rays on the scene's
 * device: rays = n x 6 f32 host array (origin xyz with w = 1, direction xyz with w = 0, as
 * Camera.getRayForPixel and the materials make them).  out_dist (n f64): the closest hit's distance,
 * +Infinity for none; out_object (n i32): the hit Primitive as its OBJS index in the scene blob, -1
 * for none.  Synchronous. */
int jsrt_cast(jsrt_scene *scene, const float *rays, size_t n, double min_dist, double max_dist,
              int32_t intersect_transparent, double *out_dist, int32_t *out_object);

/* World.color(ray, 1) up to Material.color (world.js:31-41, 125-137) of n rays (as jsrt_cast): the
 * closest hit of World.cast(ray, 0) -- out_dist, out_object as jsrt_cast -- and the material_data the
 * hit Primitive hands to its material: normal (n x 4 f32: inv_transform.transposed().times(n).to4(0)
 * .normalized()), position (n x 4: ray.getPoint(distance)), uv (n x 3: UV, the third component always
 * NaN), bary (n x 3: a triangle's barycentric coordinates), basecolor (n x 3: an SDF's); NaN where a
 * field is absent (or no hit).  Synchronous. */
int jsrt_material_data(jsrt_scene *scene, const float *rays, size_t n, double *out_dist, int32_t *out_object,
                       float *normal, float *position, float *uv, float *bary, float *basecolor);

/* SDF.distance (sdf.js:53-74) of the root SDF of SDFGeometry primitive `object` (its OBJS index in the
 * blob) at n points (f32 x 4 in the primitive's local frame, w = 1).  Synchronous. */
int jsrt_sdf_distance(jsrt_scene *scene, int32_t object, const float *points, size_t n, double *out);

/* Number of owned columns for (W, x_offset, x_delt, col_block). */
int32_t jsrt_owned_columns(int32_t width, int32_t x_offset, int32_t x_delt, int32_t col_block);

const char *jsrt_last_error(void);
int32_t jsrt_abi_version(void);
/* Identity of this build: a hash of the sources, headers, compiler flags and defines it was compiled
 * from (jsraytracer_amd/build.py build_id).  Hosts compare it with the tree they run from. */
const char *jsrt_build_id(void);
/* Device count visible to HIP (0 without a GPU); never initialises a context it does not need. */
int32_t jsrt_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
