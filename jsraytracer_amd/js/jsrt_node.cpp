// jsrt_node.cpp — Node N-API addon over libjsrt's C-ABI (include/jsrt.h).
//
// This is the JS side of the drop-in boundary: the reference's worker
// (src/worker.js:17-40) builds a scene and calls renderer.render(img, timelimit, callback, x_offset,
// x_delt) (src/renderers.js:10,70).  hip_renderer.js keeps that contract and calls into this addon:
//
//   sceneCreate(blob: Uint8Array|Buffer, device: number) -> external scene handle
//   sceneDestroy(scene)
//   renderSync(scene, params, rgba: Uint8Array|Uint8ClampedArray (W*H*4), progress?: fn(pass, completion))
//       -> stats object.  Blocking, on the calling thread, exactly like the reference's synchronous
//       render(); progress is invoked on that same thread from inside the render.
//   render(scene, params, rgba, progress?) -> Promise<stats>.  Runs in napi_create_async_work;
//       progress arrives through a napi_threadsafe_function (N-API >= 4).
//   deviceCount(), abiVersion()
//
// Errors: a negative jsrt_* return code becomes a thrown JS Error carrying jsrt_last_error()
// (the reference throws strings, e.g. src/aggregates.js:39).  No C++ exception crosses N-API.
#define NAPI_VERSION 8
#include <node_api.h>
#include <string.h>

#include <string>

#include "../../include/jsrt.h"
#include "../../include/jsrt_json.h"
#include "../../include/jsrt_mesh.h"

namespace {

#define NAPI_OK(call)                                                                   \
    do {                                                                                \
        if ((call) != napi_ok) {                                                        \
            const napi_extended_error_info *ei = nullptr;                               \
            napi_get_last_error_info(env, &ei);                                         \
            napi_throw_error(env, "JSRT_NAPI", ei && ei->error_message ? ei->error_message : #call); \
            return nullptr;                                                             \
        }                                                                               \
    } while (0)

napi_value throw_jsrt(napi_env env, const char *what) {
    std::string m = std::string(what) + ": " + jsrt_last_error();
    napi_throw_error(env, "JSRT", m.c_str());
    return nullptr;
}

bool get_bytes(napi_env env, napi_value v, void **data, size_t *len) {
    bool is_buf = false, is_ta = false;
    napi_is_buffer(env, v, &is_buf);
    if (is_buf) return napi_get_buffer_info(env, v, data, len) == napi_ok;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return false;
    napi_typedarray_type t;
    size_t n = 0, off = 0;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &t, &n, data, &ab, &off) != napi_ok) return false;
    if (t != napi_uint8_array && t != napi_uint8_clamped_array && t != napi_int8_array) return false;
    *len = n;
    return true;
}

int32_t prop_i32(napi_env env, napi_value obj, const char *name, int32_t dflt) {
    bool has = false;
    napi_has_named_property(env, obj, name, &has);
    if (!has) return dflt;
    napi_value v;
    int32_t r = dflt;
    if (napi_get_named_property(env, obj, name, &v) == napi_ok) napi_get_value_int32(env, v, &r);
    return r;
}

double prop_f64(napi_env env, napi_value obj, const char *name, double dflt) {
    bool has = false;
    napi_has_named_property(env, obj, name, &has);
    if (!has) return dflt;
    napi_value v;
    double r = dflt;
    if (napi_get_named_property(env, obj, name, &v) == napi_ok) napi_get_value_double(env, v, &r);
    return r;
}

// params object -> jsrt_params (names follow the reference's renderer fields)
void read_params(napi_env env, napi_value o, jsrt_params *p) {
    memset(p, 0, sizeof *p);
    p->width = prop_i32(env, o, "width", 0);
    p->height = prop_i32(env, o, "height", 0);
    p->spp = prop_i32(env, o, "samplesPerPixel", 0);
    p->max_depth = prop_i32(env, o, "maxRecursionDepth", 0);
    p->kind = prop_i32(env, o, "kind", -1);
    p->seed = (uint32_t)prop_f64(env, o, "seed", 1);
    p->x_offset = prop_i32(env, o, "x_offset", 0);
    p->x_delt = prop_i32(env, o, "x_delt", 1);
    p->device = prop_i32(env, o, "device", 0);
    p->timelimit_ms = prop_f64(env, o, "timelimit", 0);
    p->max_paths = prop_i32(env, o, "maxPaths", 0);
    p->samples_per_launch = prop_i32(env, o, "samplesPerLaunch", 0);
    p->mode = prop_i32(env, o, "mode", JSRT_MODE_STRICT);
    p->device_mask = (uint32_t)prop_f64(env, o, "deviceMask", 0);
}

napi_value stats_object(napi_env env, const jsrt_stats &st) {
    napi_value o, v;
    napi_create_object(env, &o);
    napi_create_double(env, st.kernel_ms, &v);
    napi_set_named_property(env, o, "kernel_ms", v);
    napi_create_double(env, st.total_ms, &v);
    napi_set_named_property(env, o, "total_ms", v);
    napi_create_double(env, (double)st.samples, &v);
    napi_set_named_property(env, o, "samples", v);
    napi_create_uint32(env, st.launches, &v);
    napi_set_named_property(env, o, "launches", v);
    napi_create_uint32(env, st.batches, &v);
    napi_set_named_property(env, o, "batches", v);
    return o;
}

struct SceneBox {  // the external's payload: destroy is idempotent (explicit + GC finalizer)
    jsrt_scene *s = nullptr;
    int inflight = 0;              // async renders queued or running (all counted on the JS thread)
    bool destroy_pending = false;  // sceneDestroy while renders were in flight: destroyed by the last
};
void box_finalize(napi_env, void *data, void *) {
    SceneBox *b = static_cast<SceneBox *>(data);
    if (b->s) jsrt_scene_destroy(b->s);
    delete b;
}

SceneBox *get_scene(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) return nullptr;
    return static_cast<SceneBox *>(p);
}

napi_value SceneCreate(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    void *data = nullptr;
    size_t len = 0;
    if (argc < 1 || !get_bytes(env, argv[0], &data, &len)) {
        napi_throw_type_error(env, "JSRT", "sceneCreate(blob: Uint8Array, device?: number)");
        return nullptr;
    }
    int32_t device = 0;
    if (argc > 1) napi_get_value_int32(env, argv[1], &device);
    jsrt_scene *s = nullptr;
    if (jsrt_scene_create(data, len, device, &s) != 0) return throw_jsrt(env, "jsrt_scene_create");
    SceneBox *b = new SceneBox{s};
    napi_value ext;
    NAPI_OK(napi_create_external(env, b, box_finalize, nullptr, &ext));
    return ext;
}

napi_value SceneDestroy(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox *b = argc ? get_scene(env, argv[0]) : nullptr;
    if (b && b->s) {
        if (b->inflight > 0) {  // the scene is in use by queued / running async renders
            b->destroy_pending = true;
        } else {
            jsrt_scene_destroy(b->s);
            b->s = nullptr;
        }
    }
    return nullptr;
}

// ---- synchronous render: progress runs on the JS thread that called renderSync ----
struct SyncCtx {
    napi_env env;
    napi_value fn;
};
void sync_progress(int32_t pass, double completion, void *user) {
    SyncCtx *c = static_cast<SyncCtx *>(user);
    napi_value args[2], global, ret;
    napi_create_int32(c->env, pass, &args[0]);
    napi_create_double(c->env, completion, &args[1]);
    napi_get_global(c->env, &global);
    napi_call_function(c->env, global, c->fn, 2, args, &ret);  // a throw stays pending, reported after
}

napi_value RenderSync(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox *b = argc > 0 ? get_scene(env, argv[0]) : nullptr;
    if (!b || !b->s || b->destroy_pending) {
        napi_throw_type_error(env, "JSRT", "renderSync: scene handle is missing or destroyed");
        return nullptr;
    }
    jsrt_params p;
    memset(&p, 0, sizeof p);
    if (argc > 1) read_params(env, argv[1], &p);
    void *rgba = nullptr;
    size_t len = 0;
    if (argc < 3 || !get_bytes(env, argv[2], &rgba, &len)) {
        napi_throw_type_error(env, "JSRT", "renderSync: rgba must be a Uint8(Clamped)Array");
        return nullptr;
    }
    if ((size_t)p.width * (size_t)p.height * 4 != len || p.width <= 0 || p.height <= 0) {
        napi_throw_range_error(env, "JSRT", "renderSync: rgba length must be width*height*4");
        return nullptr;
    }
    SyncCtx ctx{env, nullptr};
    jsrt_progress_fn cb = nullptr;
    if (argc > 3) {
        napi_valuetype t;
        napi_typeof(env, argv[3], &t);
        if (t == napi_function) {
            ctx.fn = argv[3];
            cb = sync_progress;
        }
    }
    jsrt_stats st;
    memset(&st, 0, sizeof st);
    const int rc = jsrt_render(b->s, &p, static_cast<uint8_t *>(rgba), nullptr, cb, &ctx, &st);
    bool pending = false;
    napi_is_exception_pending(env, &pending);
    if (pending) return nullptr;
    if (rc != 0) return throw_jsrt(env, "jsrt_render");
    return stats_object(env, st);
}

// ---- asynchronous render: worker thread + threadsafe progress function + Promise ----
struct AsyncJob {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_threadsafe_function tsfn = nullptr;
    napi_ref buf_ref = nullptr;    // keeps the output array alive while the render writes into it
    napi_ref scene_ref = nullptr;  // keeps the scene external (and its GC finalizer) alive meanwhile
    SceneBox *box = nullptr;
    jsrt_scene *scene = nullptr;
    jsrt_params p;
    uint8_t *rgba = nullptr;
    jsrt_stats st;
    int rc = 0;
    std::string err;
};
struct ProgressMsg {
    int32_t pass;
    double completion;
};

void tsfn_call(napi_env env, napi_value js_cb, void *, void *data) {
    ProgressMsg *m = static_cast<ProgressMsg *>(data);
    if (env && js_cb) {
        napi_value args[2], global, ret;
        napi_create_int32(env, m->pass, &args[0]);
        napi_create_double(env, m->completion, &args[1]);
        napi_get_global(env, &global);
        napi_call_function(env, global, js_cb, 2, args, &ret);
    }
    delete m;
}

void async_progress(int32_t pass, double completion, void *user) {
    AsyncJob *j = static_cast<AsyncJob *>(user);
    if (!j->tsfn) return;
    ProgressMsg *m = new ProgressMsg{pass, completion};
    if (napi_call_threadsafe_function(j->tsfn, m, napi_tsfn_nonblocking) != napi_ok) delete m;
}

void async_execute(napi_env, void *data) {
    AsyncJob *j = static_cast<AsyncJob *>(data);
    memset(&j->st, 0, sizeof j->st);
    j->rc = jsrt_render(j->scene, &j->p, j->rgba, nullptr, j->tsfn ? async_progress : nullptr, j, &j->st);
    if (j->rc != 0) j->err = jsrt_last_error();  // thread-local: capture on this thread
}

void async_complete(napi_env env, napi_status, void *data) {
    AsyncJob *j = static_cast<AsyncJob *>(data);
    if (j->rc == 0) {
        napi_resolve_deferred(env, j->deferred, stats_object(env, j->st));
    } else {
        napi_value msg, err;
        std::string m = "jsrt_render: " + j->err;
        napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
        napi_create_error(env, nullptr, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    }
    if (j->tsfn) napi_release_threadsafe_function(j->tsfn, napi_tsfn_release);
    if (j->buf_ref) napi_delete_reference(env, j->buf_ref);
    if (j->box && --j->box->inflight == 0 && j->box->destroy_pending && j->box->s) {
        jsrt_scene_destroy(j->box->s);  // sceneDestroy was called while this render ran
        j->box->s = nullptr;
    }
    if (j->scene_ref) napi_delete_reference(env, j->scene_ref);
    napi_delete_async_work(env, j->work);
    delete j;
}

napi_value Render(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox *b = argc > 0 ? get_scene(env, argv[0]) : nullptr;
    if (!b || !b->s || b->destroy_pending) {
        napi_throw_type_error(env, "JSRT", "render: scene handle is missing or destroyed");
        return nullptr;
    }
    AsyncJob *j = new AsyncJob();
    j->scene = b->s;
    memset(&j->p, 0, sizeof j->p);
    if (argc > 1) read_params(env, argv[1], &j->p);
    void *rgba = nullptr;
    size_t len = 0;
    if (argc < 3 || !get_bytes(env, argv[2], &rgba, &len) ||
        (size_t)j->p.width * (size_t)j->p.height * 4 != len || j->p.width <= 0 || j->p.height <= 0) {
        delete j;
        napi_throw_range_error(env, "JSRT", "render: rgba must be a Uint8(Clamped)Array of width*height*4");
        return nullptr;
    }
    j->rgba = static_cast<uint8_t *>(rgba);
    napi_create_reference(env, argv[2], 1, &j->buf_ref);
    napi_create_reference(env, argv[0], 1, &j->scene_ref);
    j->box = b;
    ++b->inflight;
    napi_value promise, name;
    NAPI_OK(napi_create_promise(env, &j->deferred, &promise));
    napi_create_string_utf8(env, "jsrt_render", NAPI_AUTO_LENGTH, &name);
    if (argc > 3) {
        napi_valuetype t;
        napi_typeof(env, argv[3], &t);
        if (t == napi_function)
            NAPI_OK(napi_create_threadsafe_function(env, argv[3], nullptr, name, 0, 1, nullptr, nullptr, nullptr,
                                                    tsfn_call, &j->tsfn));
    }
    NAPI_OK(napi_create_async_work(env, nullptr, name, async_execute, async_complete, j, &j->work));
    NAPI_OK(napi_queue_async_work(env, j->work));
    return promise;
}

// attachObj(blob, objText, {bvhObject, minArea}?) -> {blob: Buffer, triangles, nodes, maxDepth}
// loadObjFile + BVHAggregate.build natively (include/jsrt_mesh.h; objloader.js:224-231, aggregates.js:33-41)
// string (UTF-8) or Uint8Array/Buffer contents
bool get_text(napi_env env, napi_value v, std::string &out) {
    void *b = nullptr;
    size_t l = 0;
    if (get_bytes(env, v, &b, &l)) {
        out.assign((const char *)b, l);
        return true;
    }
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, nullptr, 0, &n) != napi_ok) return false;
    out.resize(n + 1);
    napi_get_value_string_utf8(env, v, &out[0], n + 1, &n);
    out.resize(n);
    return true;
}

napi_value AttachObj(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    void *data = nullptr;
    size_t len = 0;
    if (argc < 2 || !get_bytes(env, argv[0], &data, &len)) {
        napi_throw_type_error(env, "JSRT", "attachObj(blob: Uint8Array, objText: string | Uint8Array, opts?)");
        return nullptr;
    }
    std::string text, mtl;
    if (!get_text(env, argv[1], text)) {
        napi_throw_type_error(env, "JSRT", "attachObj: objText must be a string or Uint8Array");
        return nullptr;
    }
    jsrt_mesh_options opt{-1, 0, 0.00001};
    if (argc > 2) {
        napi_valuetype t;
        napi_typeof(env, argv[2], &t);
        if (t == napi_object) {
            napi_value v;
            bool has = false;
            if (napi_has_named_property(env, argv[2], "bvhObject", &has) == napi_ok && has &&
                napi_get_named_property(env, argv[2], "bvhObject", &v) == napi_ok)
                napi_get_value_int32(env, v, &opt.bvh_object);
            if (napi_has_named_property(env, argv[2], "minArea", &has) == napi_ok && has &&
                napi_get_named_property(env, argv[2], "minArea", &v) == napi_ok)
                napi_get_value_double(env, v, &opt.min_area);
            // mtl: the mtllib files' texts (string | Uint8Array, or an array of them in mtllib order)
            if (napi_has_named_property(env, argv[2], "mtl", &has) == napi_ok && has &&
                napi_get_named_property(env, argv[2], "mtl", &v) == napi_ok) {
                bool arr = false;
                napi_is_array(env, v, &arr);
                uint32_t n = 1;
                if (arr) napi_get_array_length(env, v, &n);
                for (uint32_t i = 0; i < n; ++i) {
                    napi_value e = v;
                    if (arr) napi_get_element(env, v, i, &e);
                    std::string one;
                    if (!get_text(env, e, one)) {
                        napi_throw_type_error(env, "JSRT", "attachObj: opts.mtl must hold strings or Uint8Arrays");
                        return nullptr;
                    }
                    if (i) mtl.push_back('\0');
                    mtl += one;
                }
            }
        }
    }
    void *out = nullptr;
    size_t out_n = 0;
    jsrt_mesh_info mi;
    if (jsrt_blob_attach_obj_mtl(data, len, text.data(), text.size(), mtl.data(), mtl.size(), &opt, &out, &out_n,
                                 &mi) != 0)
        return throw_jsrt(env, "jsrt_blob_attach_obj");
    napi_value buf, o, v;
    void *dst = nullptr;
    napi_status st = napi_create_buffer_copy(env, out_n, out, &dst, &buf);
    jsrt_blob_free(out);
    NAPI_OK(st);
    NAPI_OK(napi_create_object(env, &o));
    napi_set_named_property(env, o, "blob", buf);
    napi_create_double(env, (double)mi.triangles, &v);
    napi_set_named_property(env, o, "triangles", v);
    napi_create_double(env, (double)mi.nodes, &v);
    napi_set_named_property(env, o, "nodes", v);
    napi_create_int32(env, mi.max_depth, &v);
    napi_set_named_property(env, o, "maxDepth", v);
    return o;
}

// blobFromJson(jsonText, {psdataObj}?) -> {blob: Buffer, objects, triangles, psdataMatched}
// Serializer.deserializeJSON (serializer.js:69-71) for the dragon_json-style flow, natively
// (include/jsrt_json.h); psdataObj: the OBJ text(s) the meshes came from (vertex normals / UVs).
napi_value BlobFromJson(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    std::string text, side;
    if (argc < 1 || !get_text(env, argv[0], text)) {
        napi_throw_type_error(env, "JSRT", "blobFromJson(jsonText: string | Uint8Array, opts?)");
        return nullptr;
    }
    if (argc > 1) {
        napi_valuetype t;
        napi_typeof(env, argv[1], &t);
        napi_value v;
        bool has = false;
        if (t == napi_object && napi_has_named_property(env, argv[1], "psdataObj", &has) == napi_ok && has &&
            napi_get_named_property(env, argv[1], "psdataObj", &v) == napi_ok) {
            bool arr = false;
            napi_is_array(env, v, &arr);
            uint32_t n = 1;
            if (arr) napi_get_array_length(env, v, &n);
            for (uint32_t i = 0; i < n; ++i) {
                napi_value e = v;
                if (arr) napi_get_element(env, v, i, &e);
                std::string one;
                if (!get_text(env, e, one)) {
                    napi_throw_type_error(env, "JSRT", "blobFromJson: opts.psdataObj must hold strings or Uint8Arrays");
                    return nullptr;
                }
                if (i) side.push_back('\0');
                side += one;
            }
        }
    }
    void *out = nullptr;
    size_t out_n = 0;
    jsrt_json_info ji;
    if (jsrt_blob_from_json(text.data(), text.size(), side.data(), side.size(), &out, &out_n, &ji) != 0)
        return throw_jsrt(env, "jsrt_blob_from_json");
    napi_value buf, o, v;
    void *dst = nullptr;
    napi_status st = napi_create_buffer_copy(env, out_n, out, &dst, &buf);
    jsrt_blob_free(out);
    NAPI_OK(st);
    NAPI_OK(napi_create_object(env, &o));
    napi_set_named_property(env, o, "blob", buf);
    napi_create_double(env, (double)ji.objects, &v);
    napi_set_named_property(env, o, "objects", v);
    napi_create_double(env, (double)ji.triangles, &v);
    napi_set_named_property(env, o, "triangles", v);
    napi_create_double(env, (double)ji.psdata_matched, &v);
    napi_set_named_property(env, o, "psdataMatched", v);
    return o;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
    napi_value v;
    napi_create_int32(env, jsrt_device_count(), &v);
    return v;
}

napi_value AbiVersion(napi_env env, napi_callback_info) {
    napi_value v;
    napi_create_int32(env, jsrt_abi_version(), &v);
    return v;
}

napi_value OwnedColumns(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    int32_t a[4] = {0, 0, 1, 1};
    for (size_t i = 0; i < argc && i < 4; ++i) napi_get_value_int32(env, argv[i], &a[i]);
    napi_value v;
    napi_create_int32(env, jsrt_owned_columns(a[0], a[1], a[2], a[3]), &v);
    return v;
}

napi_value Init(napi_env env, napi_value exports) {
    const napi_property_descriptor props[] = {
        {"sceneCreate", nullptr, SceneCreate, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"sceneDestroy", nullptr, SceneDestroy, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"renderSync", nullptr, RenderSync, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"render", nullptr, Render, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"abiVersion", nullptr, AbiVersion, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"ownedColumns", nullptr, OwnedColumns, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"attachObj", nullptr, AttachObj, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"blobFromJson", nullptr, BlobFromJson, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
