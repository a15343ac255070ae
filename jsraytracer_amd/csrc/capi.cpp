// capi.cpp — the C-ABI of include/jsrt.h: scene upload, render launches, host/device outputs.
//
// No C++ exception crosses the ABI; every entry point returns 0 / negative and records a message
// for jsrt_last_error() (the reference throws strings, e.g. src/aggregates.js:39).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

#include "../../include/jsrt.h"
#include "render_kernel.h"
#include "scene_load.h"

using namespace jsrt;

namespace {
thread_local std::string g_err;
int set_error(int code, const std::string &m) {
    g_err = m;
    return code;
}
}  // namespace

namespace jsrt {
// shared with mesh_build.cpp: the one jsrt_last_error() message per thread
int record_error(int code, const std::string &m) { return set_error(code, m); }
}  // namespace jsrt

namespace {
#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return set_error(-3, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct DeviceArena {  // one allocation holding every scene array (256-B aligned pieces)
    std::vector<uint8_t> host;
    size_t add(const void *p, size_t bytes) {
        size_t off = (host.size() + 255) & ~(size_t)255;
        host.resize(off + bytes);
        if (bytes) memcpy(host.data() + off, p, bytes);
        return off;
    }
    template <class T>
    size_t add(const std::vector<T> &v) { return add(v.data(), v.size() * sizeof(T)); }
};
}  // namespace

struct jsrt_scene {
    int device = 0;
    void *dmem = nullptr;
    DScene ds;
    HostScene hs;
    int ns = 0;            // light samples per lit node
    std::mutex wf_mutex;   // guards the cached wavefront buffers
    Wavefront wf;
    hipEvent_t wf_busy = nullptr;  // recorded after the last render that used wf (stream order for the next)
};

extern "C" {

int32_t jsrt_abi_version(void) { return JSRT_ABI_VERSION; }
const char *jsrt_last_error(void) { return g_err.c_str(); }

int32_t jsrt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int32_t jsrt_owned_columns(int32_t width, int32_t x_offset, int32_t x_delt, int32_t col_block) {
    if (width <= 0) return 0;
    if (x_delt <= 0) x_delt = 1;
    int32_t n = 0;
    if (col_block <= 1) {
        for (int32_t px = x_offset; px < width; px += x_delt) ++n;
        return n;
    }
    for (int32_t c = 0;; ++c) {
        if (owned_to_px(c, x_offset, x_delt, col_block) >= width) {
            // columns of a block are consecutive; stop at the first out-of-range one
            return n;
        }
        ++n;
    }
}

int jsrt_scene_create(const void *blob, size_t n, int32_t device, jsrt_scene **out) {
    if (!out) return set_error(-1, "out is NULL");
    *out = nullptr;
    std::unique_ptr<jsrt_scene> sc(new jsrt_scene());
    std::string err;
    if (load_scene(blob, n, sc->hs, err)) return set_error(-2, err);
    HostScene &H = sc->hs;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return set_error(-3, "no such HIP device");
    HIP_TRY(hipSetDevice(device));
    sc->device = device;
    DeviceArena A;
    const size_t o_prims = A.add(H.prims), o_insts = A.add(H.insts), o_ichild = A.add(H.inst_child),
                 o_roots = A.add(H.roots), o_rb = A.add(H.rbounds), o_rr = A.add(H.rootrec), o_mats = A.add(H.mats), o_ctx = A.add(H.ctx), o_bvh = A.add(H.bvh),
                 o_lp = A.add(H.leaf_prims), o_lt = A.add(H.leaf_tris), o_tris = A.add(H.tris),
                 o_trish = A.add(H.trish), o_mat = A.add(H.mat), o_matf = A.add(H.mat_flags), o_ps = A.add(H.prim_shade),
                 o_sh0 = A.add(H.shade0), o_shI = A.add(H.shadeI), o_mc = A.add(H.mc), o_mcc = A.add(H.mc_const), o_lights = A.add(H.lights),
                 o_sl = A.add(H.sample_light), o_sc = A.add(H.sample_call),
                 o_insn = A.add(H.sdf_insn), o_const = A.add(H.sdf_const), o_range = A.add(H.sdf_range),
                 o_schild = A.add(H.sdf_child), o_snodes = A.add(H.sdf_nodes), o_sdfg = A.add(H.sdfg), o_ltris = A.add(H.ltris), o_plit = A.add(H.prim_lit),
                 o_gmask = A.add(H.grid_mask);
    const size_t total = A.host.size() + 256;
    HIP_TRY(hipMalloc(&sc->dmem, total));
    HIP_TRY(hipMemcpy(sc->dmem, A.host.data(), A.host.size(), hipMemcpyHostToDevice));
    uint8_t *b = static_cast<uint8_t *>(sc->dmem);
    DScene &D = sc->ds;
    memset(&D, 0, sizeof D);
    D.prims = (const DPrim *)(b + o_prims);
    D.insts = (const DInst *)(b + o_insts);
    D.inst_child = (const int32_t *)(b + o_ichild);
    D.roots = (const int32_t *)(b + o_roots);
    D.rbounds = (const RootBound *)(b + o_rb);
    D.rootrec = (const DRoot *)(b + o_rr);
    D.mats = (const double *)(b + o_mats);
    D.ctx = (const double *)(b + o_ctx);
    D.bvh = (const DBvhNode *)(b + o_bvh);
    D.leaf_prims = (const int32_t *)(b + o_lp);
    D.leaf_tris = (const int32_t *)(b + o_lt);
    D.tris = (const DTri *)(b + o_tris);
    D.trish = (const DTriShade *)(b + o_trish);
    D.mat = (const jsrt_rec_material *)(b + o_mat);
    D.mat_flags = (const int32_t *)(b + o_matf);
    D.prim_shade = (const int32_t *)(b + o_ps);
    D.shade0 = (const double *)(b + o_sh0);
    D.shadeI = (const double *)(b + o_shI);
    D.mc = (const jsrt_rec_mcolor *)(b + o_mc);
    D.mc_const = (const float *)(b + o_mcc);
    D.lights = (const DLight *)(b + o_lights);
    D.sample_light = (const int32_t *)(b + o_sl);
    D.sample_call = (const int32_t *)(b + o_sc);
    D.light_draws = H.light_draws;
    D.max_children = H.max_children;
    D.bvh_stack = H.bvh.empty() ? 0 : H.bvh_max_depth + 2;
    D.ltris = (const DTri *)(b + o_ltris);
    D.prim_lit = (const int32_t *)(b + o_plit);
    D.grid_mask = (const uint64_t *)(b + o_gmask);
    for (int k = 0; k < 3; ++k) {
        D.grid_lo[k] = H.grid_lo[k];
        D.grid_inv[k] = H.grid_inv[k];
        D.grid_dim[k] = H.grid_dim[k];
    }
    D.grid_cells = H.grid_cells;
    D.grid_masked = H.roots.size() <= 64 ? 1 : 0;
    D.sdf_insn = (const SdfInsn *)(b + o_insn);
    D.sdf_const = (const double *)(b + o_const);
    D.sdf_range = (const int32_t *)(b + o_range);
    D.sdf_child = (const int32_t *)(b + o_schild);
    D.sdf_nodes = (const jsrt_rec_sdfnode *)(b + o_snodes);
    D.sdfg = (const jsrt_rec_sdfgeom *)(b + o_sdfg);
    D.n_roots = (int32_t)H.roots.size();
    D.n_lights = (int32_t)H.lights.size();
    D.n_prims = (int32_t)H.prims.size();
    D.n_insts = (int32_t)H.insts.size();
    D.cam = H.cam;
    memcpy(D.bg, H.bg, sizeof D.bg);
    D.all_roots_prims = H.all_roots_prims;
    const char *fo = getenv("JSRT_SDF_FO");  // A/B: 0 = the persistent marches keep the VM fallback
    D.sdf_all_forms = (fo && fo[0] == '0') ? 0 : H.sdf_all_forms;
    D.profile = H.profile;
    sc->ns = (int)H.sample_light.size();
    *out = sc.release();
    return 0;
}

void jsrt_scene_destroy(jsrt_scene *s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->wf_busy) {
        (void)hipEventSynchronize(s->wf_busy);
        (void)hipEventDestroy(s->wf_busy);
    }
    if (s->dmem) (void)hipFree(s->dmem);
    delete s;
}

}  // extern "C"

namespace {

struct Resolved {
    RenderArgs a;
    int32_t col_block;
};

int resolve(const jsrt_scene *s, const jsrt_params *p, int32_t col_block, Resolved &R) {
    if (!s) return set_error(-1, "scene is NULL");
    const HostScene &H = s->hs;
    RenderArgs &a = R.a;
    memset(&a, 0, sizeof a);
    a.W = p && p->width > 0 ? p->width : H.width;
    a.H = p && p->height > 0 ? p->height : H.height;
    a.spp = p && p->spp > 0 ? p->spp : H.spp;
    a.max_depth = p && p->max_depth > 0 ? p->max_depth : H.max_depth;
    a.kind = p && p->kind >= 0 ? p->kind : H.kind;
    a.seed = p ? p->seed : 1u;
    a.x_offset = p ? p->x_offset : 0;
    a.x_delt = p && p->x_delt > 0 ? p->x_delt : 1;
    if (a.W <= 0 || a.H <= 0) return set_error(-1, "image size must be positive");
    if (a.kind < 0 || a.kind > 2) return set_error(-1, "unknown renderer kind");
    if (a.kind == JSRT_RENDERER_SIMPLE) a.spp = 1;
    if (a.spp <= 0) return set_error(-1, "samplesPerPixel must be positive");
    if (a.max_depth < 0 || a.max_depth > MAX_TREE_DEPTH)
        return set_error(-1, "maxRecursionDepth above " + std::to_string(MAX_TREE_DEPTH) + " is not supported");
    if (a.x_offset < 0) return set_error(-1, "x_offset must be >= 0");
    if (col_block > 1 && a.x_offset >= a.x_delt) return set_error(-1, "block partition needs x_offset < x_delt");
    R.col_block = col_block > 1 ? col_block : 1;
    a.col_block = R.col_block;
    a.ncols = jsrt_owned_columns(a.W, a.x_offset, a.x_delt, R.col_block);
    a.patches_x = (a.ncols + 7) / 8;
    a.patches = a.patches_x * ((a.H + 7) / 8);
    return 0;
}

// Renders one frame (all spp) on `stream` through the wavefront schedule (render.hip); every
// kernel launch is bracketed by HIP events recorded on that same stream.
// Owned column c, row py -> image (px, py) of the host PixelBuffer; other columns untouched
// (worker.js semantics).
void scatter_columns(const RenderArgs &a, const uint32_t *h_rgba, const float *h_col, uint8_t *rgba8,
                     float *colors_f32) {
    for (int32_t c = 0; c < a.ncols; ++c) {
        const int32_t px = owned_to_px(c, a.x_offset, a.x_delt, 1);
        for (int32_t py = 0; py < a.H; ++py) {
            const size_t src = (size_t)c * a.H + py, dst = (size_t)py * a.W + px;
            memcpy(rgba8 + 4 * dst, &h_rgba[src], 4);
            if (colors_f32 && h_col) memcpy(colors_f32 + 4 * dst, &h_col[4 * src], 16);
        }
    }
}

// host_rgba (nullable): the caller's PixelBuffer.  With a progress callback and the Incremental
// renderer, the running mean of the passes done so far is written into its owned columns before each
// callback (renderers.js:93-112: setColor every pass, callback reads img), from clean passes only.
int run_launches(jsrt_scene *s, const jsrt_params *p, RenderArgs a, uint32_t *d_rgba, float *d_colors,
                 hipStream_t stream, jsrt_progress_fn progress, void *user, jsrt_stats *st,
                 uint8_t *host_rgba = nullptr) {
    const size_t nacc = (size_t)a.ncols * a.H * 4;
    float *accum = nullptr;
    HIP_TRY(hipMallocAsync((void **)&accum, nacc * sizeof(float) + 16, stream));
    a.rgba = d_rgba;
    a.colors = d_colors;
    a.accum = accum;
    a.final_pass = 1;
    std::unique_lock<std::mutex> lk(s->wf_mutex, std::try_to_lock);  // re-entrant: busy cache -> own buffers
    std::unique_ptr<Wavefront> own;
    Wavefront *wf = &s->wf;
    if (!lk.owns_lock()) {
        own.reset(new Wavefront());
        wf = own.get();
    }
    KernelTimes kt;
    if (p && (p->stage_events & ~JSRT_EVENTS_ONE_STREAM)) kt.mask = (uint32_t)(p->stage_events & ~JSRT_EVENTS_ONE_STREAM);
    kt.one_stream = p && (p->stage_events & JSRT_EVENTS_ONE_STREAM) != 0;
    auto t_last = std::chrono::steady_clock::now();
    const double tl = p ? p->timelimit_ms : 0;
    a.samples_per_batch = (p && p->samples_per_launch > 0) ? p->samples_per_launch : 0;
    const bool preview = host_rgba && a.kind == JSRT_RENDERER_INCREMENTAL;
    std::vector<uint32_t> h_prev;
    std::function<bool(int, double, bool)> prog;
    int prev_rc = 0;
    bool reported = false;  // a callback (or preview) has reached the caller: a retry would repeat passes
    if (progress && tl > 0)
        prog = [&](int pass, double completion, bool clean) {  // renderers.js:103-112 cadence, batch granularity
            if (completion >= 1.0) return true;
            auto now = std::chrono::steady_clock::now();
            if (std::chrono::duration<double, std::milli>(now - t_last).count() >= tl) {
                t_last = now;
                reported = true;
                if (preview && clean) {
                    const size_t npx = (size_t)a.ncols * a.H;
                    h_prev.resize(npx);
                    if (render_preview(a, pass + 1, stream) != hipSuccess ||
                        hipMemcpyAsync(h_prev.data(), d_rgba, npx * 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                        hipStreamSynchronize(stream) != hipSuccess) {
                        prev_rc = set_error(-3, "progress preview failed");
                        return false;
                    }
                    scatter_columns(a, h_prev.data(), nullptr, host_rgba, nullptr);
                }
                progress(pass, completion, user);
            }
            return true;
        };
    // default batch (A/B on MI355X, tools/ab_maxpaths.sh): 32 M paths (dragon +4 %, Menger +12 % over
    // 16 M; cornell, whose batches alternate between two pools and streams, +2.9 %: profiles/r03_s18_ab.txt)
    const size_t def_paths = (size_t)1 << 25;
    size_t max_paths = (p && p->max_paths > 0) ? (size_t)p->max_paths : def_paths;
    if (const char *e = getenv("JSRT_MAX_PATHS")) max_paths = (size_t)atoll(e);
    // The batch's state is cached per scene and sized by max_paths (render_kernel.h
    // wavefront_bytes_per_path: ~1.8 KB per path on the tree schedule, 60 GB at 32 M paths): the
    // default is capped at half the device memory free now, and a batch whose buffers cannot be
    // allocated is retried at half the size (the batch size never changes a bit of the image).
    // Simple / RandomMultisampling with a callback report per batch (renderers.js:28-37): at least 8
    if (prog && a.kind != JSRT_RENDERER_INCREMENTAL) {
        const size_t work = (size_t)a.patches * 64 * (size_t)a.spp;
        max_paths = std::min(max_paths, std::max<size_t>(64, (work + 7) / 8));
    }
    if (!(p && p->max_paths > 0)) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
            const size_t cap = free_b / 2 / std::max<size_t>(1, wavefront_bytes_per_path(s->ds, s->ns, a.max_depth));
            if (max_paths > cap) max_paths = std::max<size_t>((size_t)1 << 16, cap & ~(size_t)63);
        }
    }
    // a previous device-side render of this scene (jsrt_render_device returns before its kernels
    // finish) may still be using the cached buffers on another stream
    if (wf == &s->wf && s->wf_busy) (void)hipStreamWaitEvent(stream, s->wf_busy, 0);
    hipError_t e;
    for (;;) {
        e = render_frame(s->ds, a, s->ns, *wf, stream, st ? &kt : nullptr, max_paths, prog);
        // out of device memory: retry at half the batch, unless a callback already saw part of this
        // frame (its passes / completion would repeat or go backwards)
        if (e != hipErrorOutOfMemory || max_paths <= ((size_t)1 << 16) || reported) break;
        (void)hipGetLastError();
        max_paths /= 2;
        wf->release();
        if (st) kt.reset();
    }
    if (wf == &s->wf) {
        if (!s->wf_busy) (void)hipEventCreateWithFlags(&s->wf_busy, hipEventDisableTiming);
        if (s->wf_busy) (void)hipEventRecord(s->wf_busy, stream);
    }
    int rc = prev_rc;
    if (!rc && e != hipSuccess) rc = set_error(-3, std::string("render: ") + hipGetErrorString(e));
    if (!rc && st) {
        if (hipStreamSynchronize(stream) != hipSuccess) rc = set_error(-3, "render kernels failed");
        double ms = 0;
        uint32_t launches = 0;
        for (int k = 0; k < KT_N && k < JSRT_STAGES; ++k) {
            st->stage_ms[k] = kt.ev[k].total_ms(&st->events_lost);
            st->stage_launches[k] = (uint32_t)kt.ev[k].used;
            ms += st->stage_ms[k];
            launches += (uint32_t)kt.ev[k].used;
        }
        st->kernel_ms = ms;
        st->launches = launches;
        st->batches = kt.batches;
        st->attempts = kt.attempts;
        st->samples = (uint64_t)a.ncols * a.H * a.spp;
    }
    (void)hipFreeAsync(accum, stream);
    return rc;
}

}  // namespace

extern "C" {

int jsrt_cast(jsrt_scene *s, const float *rays, size_t n, double min_dist, double max_dist, int32_t intersect_transparent,
              double *out_dist, int32_t *out_object) {
    if (!s) return set_error(-1, "scene is NULL");
    if (n == 0) return 0;
    if (!rays || !out_dist || !out_object) return set_error(-1, "NULL buffer");
    if (n > (size_t)UINT32_MAX / 8) return set_error(-1, "too many rays");
    HIP_TRY(hipSetDevice(s->device));
    float *d_rays = nullptr;
    double *d_t = nullptr;
    int32_t *d_prim = nullptr;
    auto cleanup = [&] {
        if (d_rays) (void)hipFree(d_rays);
        if (d_t) (void)hipFree(d_t);
        if (d_prim) (void)hipFree(d_prim);
    };
    hipError_t e = hipMalloc(&d_rays, n * 6 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_t, n * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&d_prim, n * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, n * 6 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = cast_rays(s->ds, d_rays, (uint32_t)n, min_dist, max_dist, intersect_transparent != 0, d_t, d_prim, 0);
    if (e == hipSuccess) e = hipMemcpy(out_dist, d_t, n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_object, d_prim, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    cleanup();
    if (e != hipSuccess) return set_error(-3, std::string("jsrt_cast: ") + hipGetErrorString(e));
    const std::vector<int32_t> &po = s->hs.prim_obj;
    for (size_t i = 0; i < n; ++i) {
        const int32_t p = out_object[i];
        out_object[i] = (p >= 0 && (size_t)p < po.size()) ? po[p] : -1;
    }
    return 0;
}

int jsrt_material_data(jsrt_scene *s, const float *rays, size_t n, double *out_dist, int32_t *out_object, float *normal,
                       float *position, float *uv, float *bary, float *basecolor) {
    if (!s) return set_error(-1, "scene is NULL");
    if (n == 0) return 0;
    if (!rays || !out_dist || !out_object || !normal || !position || !uv || !bary || !basecolor)
        return set_error(-1, "NULL buffer");
    if (n > (size_t)UINT32_MAX / 16) return set_error(-1, "too many rays");
    HIP_TRY(hipSetDevice(s->device));
    // one device buffer: rays (6 f32), t (f64), prim (i32), normal + position (8 f32), uv + bary + basecolor (9 f32)
    const size_t o_t = (n * 6 * 4 + 7) & ~(size_t)7, o_p = o_t + n * 8, o_f = o_p + n * 4, total = o_f + n * 17 * 4;
    uint8_t *d = nullptr;
    hipError_t e = hipMalloc(&d, total);
    float *f = reinterpret_cast<float *>(d + o_f);
    if (e == hipSuccess) e = hipMemcpy(d, rays, n * 6 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = material_data_rays(s->ds, reinterpret_cast<const float *>(d), (uint32_t)n, reinterpret_cast<double *>(d + o_t),
                               reinterpret_cast<int32_t *>(d + o_p), f, f + 4 * n, f + 8 * n, f + 11 * n, f + 14 * n, 0);
    std::vector<float> h(n * 17);
    if (e == hipSuccess) e = hipMemcpy(out_dist, d + o_t, n * 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_object, d + o_p, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(h.data(), f, n * 17 * 4, hipMemcpyDeviceToHost);
    if (d) (void)hipFree(d);
    if (e != hipSuccess) return set_error(-3, std::string("jsrt_material_data: ") + hipGetErrorString(e));
    memcpy(normal, h.data(), n * 16);
    memcpy(position, h.data() + 4 * n, n * 16);
    memcpy(uv, h.data() + 8 * n, n * 12);
    memcpy(bary, h.data() + 11 * n, n * 12);
    memcpy(basecolor, h.data() + 14 * n, n * 12);
    const std::vector<int32_t> &po = s->hs.prim_obj;
    for (size_t i = 0; i < n; ++i) {
        const int32_t p = out_object[i];
        out_object[i] = (p >= 0 && (size_t)p < po.size()) ? po[p] : -1;
    }
    return 0;
}

int jsrt_sdf_distance(jsrt_scene *s, int32_t object, const float *points, size_t n, double *out) {
    if (!s) return set_error(-1, "scene is NULL");
    int32_t g = -1;
    for (size_t p = 0; p < s->hs.prims.size(); ++p)
        if (s->hs.prim_obj[p] == object && s->hs.prims[p].gkind == JSRT_GEOM_SDF) g = s->hs.prims[p].gindex;
    if (g < 0) return set_error(-1, "object " + std::to_string(object) + " is not an SDFGeometry primitive");
    if (n == 0) return 0;
    if (!points || !out) return set_error(-1, "NULL buffer");
    if (n > (size_t)UINT32_MAX / 16) return set_error(-1, "too many points");
    HIP_TRY(hipSetDevice(s->device));
    uint8_t *d = nullptr;
    hipError_t e = hipMalloc(&d, n * 16 + n * 8);
    if (e == hipSuccess) e = hipMemcpy(d, points, n * 16, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = sdf_distance_points(s->ds, g, reinterpret_cast<const float *>(d), (uint32_t)n, reinterpret_cast<double *>(d + n * 16), 0);
    if (e == hipSuccess) e = hipMemcpy(out, d + n * 16, n * 8, hipMemcpyDeviceToHost);
    if (d) (void)hipFree(d);
    if (e != hipSuccess) return set_error(-3, std::string("jsrt_sdf_distance: ") + hipGetErrorString(e));
    return 0;
}

int jsrt_render(jsrt_scene *s, const jsrt_params *p, uint8_t *rgba8, float *colors_f32, jsrt_progress_fn progress,
                void *user, jsrt_stats *stats) {
    const auto t0 = std::chrono::steady_clock::now();
    Resolved R;
    if (int rc = resolve(s, p, 1, R)) return rc;
    if (!rgba8) return set_error(-1, "rgba8 is NULL");
    RenderArgs &a = R.a;
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t stream;
    HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const size_t npx = (size_t)a.ncols * a.H;
    uint32_t *d_rgba = nullptr;
    float *d_col = nullptr;
    int rc = 0;
    jsrt_stats st;
    memset(&st, 0, sizeof st);
    if (hipMalloc(&d_rgba, npx * 4) != hipSuccess) rc = set_error(-3, "out of device memory");
    if (!rc && colors_f32 && hipMalloc(&d_col, npx * 16) != hipSuccess) rc = set_error(-3, "out of device memory");
    if (!rc) rc = run_launches(s, p, a, d_rgba, d_col, stream, progress, user, &st, rgba8);
    if (!rc && npx) {
        std::vector<uint32_t> h_rgba(npx);
        std::vector<float> h_col(colors_f32 ? npx * 4 : 0);
        if (hipMemcpyAsync(h_rgba.data(), d_rgba, npx * 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
            (colors_f32 && hipMemcpyAsync(h_col.data(), d_col, npx * 16, hipMemcpyDeviceToHost, stream) != hipSuccess) ||
            hipStreamSynchronize(stream) != hipSuccess)
            rc = set_error(-3, "device-to-host copy failed");
        if (!rc) scatter_columns(a, h_rgba.data(), colors_f32 ? h_col.data() : nullptr, rgba8, colors_f32);
    }
    if (d_rgba) (void)hipFree(d_rgba);
    if (d_col) (void)hipFree(d_col);
    (void)hipStreamDestroy(stream);
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = st;
    return rc;
}

int jsrt_render_device(jsrt_scene *s, const jsrt_params *p, int32_t col_block, uint32_t *d_rgba8, float *d_colors,
                       void *hip_stream, jsrt_stats *stats) {
    const auto t0 = std::chrono::steady_clock::now();
    Resolved R;
    if (int rc = resolve(s, p, col_block, R)) return rc;
    if (!d_rgba8) return set_error(-1, "d_rgba8 is NULL");
    HIP_TRY(hipSetDevice(s->device));
    jsrt_stats st;
    memset(&st, 0, sizeof st);
    const int rc = run_launches(s, p, R.a, d_rgba8, d_colors, (hipStream_t)hip_stream, nullptr, nullptr,
                                stats ? &st : nullptr);
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = st;
    return rc;
}

}  // extern "C"
