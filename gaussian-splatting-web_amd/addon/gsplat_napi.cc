// gsplat_napi.cc — Node N-API addon over the C ABI (include/gsplat.h).
//
// The reference's TypeScript host (src/gpu_context.ts, src/renderer.ts) talks to WebGPU; the
// JavaScript mirror in ../js/index.js talks to this addon instead.  The addon is deliberately
// thin: plain handles (napi_external), typed arrays passed as borrowed pointers, errors thrown
// as JS Error objects carrying the gs_status code (`err.code`) and gs_last_error() text.
// renderAsync runs gs_render on the libuv thread pool (napi_async_work) and resolves a Promise,
// so a frame never blocks the event loop.
//
// Build: see ../Makefile (target `addon`), output ../lib/gsplat_napi.node (rpath $ORIGIN).
#define NAPI_VERSION 6
#include <node_api.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gsplat.h"

namespace {

#define NAPI_OK(call)                                                             \
    do {                                                                          \
        napi_status s_ = (call);                                                  \
        if (s_ != napi_ok) {                                                      \
            napi_throw_error(env, nullptr, "N-API call failed: " #call);          \
            return nullptr;                                                       \
        }                                                                         \
    } while (0)

napi_value throw_gs(napi_env env, int code, const char* what) {
    std::string msg = std::string(what) + ": " + gs_last_error();
    napi_value m, c, err;
    napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
    napi_create_int32(env, code, &c);
    napi_create_error(env, nullptr, m, &err);
    napi_set_named_property(env, err, "code", c);
    napi_throw(env, err);
    return nullptr;
}

napi_value undefined(napi_env env) {
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value* argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
    for (size_t i = argc; i < want; ++i) napi_get_undefined(env, &argv[i]);
    return true;
}

// Pointer and byte length of an ArrayBuffer, TypedArray or DataView (borrowed).
bool get_bytes(napi_env env, napi_value v, void** data, size_t* len) {
    bool is = false;
    if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
        napi_typedarray_type t;
        size_t n, off;
        napi_value ab;
        void* p;
        if (napi_get_typedarray_info(env, v, &t, &n, &p, &ab, &off) != napi_ok) return false;
        size_t es = 1;
        switch (t) {
            case napi_int16_array: case napi_uint16_array: es = 2; break;
            case napi_int32_array: case napi_uint32_array: case napi_float32_array: es = 4; break;
            case napi_float64_array: case napi_bigint64_array: case napi_biguint64_array: es = 8; break;
            default: es = 1;
        }
        *data = p;
        *len = n * es;
        return true;
    }
    if (napi_is_arraybuffer(env, v, &is) == napi_ok && is)
        return napi_get_arraybuffer_info(env, v, data, len) == napi_ok;
    if (napi_is_dataview(env, v, &is) == napi_ok && is) {
        napi_value ab;
        size_t off;
        return napi_get_dataview_info(env, v, len, data, &ab, &off) == napi_ok;
    }
    return false;
}

template <class T>
bool get_handle(napi_env env, napi_value v, T** out) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) return false;
    *out = static_cast<T*>(p);
    return true;
}

double num(napi_env env, napi_value v, double dflt) {
    double d;
    return napi_get_value_double(env, v, &d) == napi_ok ? d : dflt;
}

// opts object -> gs_opts (missing fields keep gs_opts_default values)
void read_opts(napi_env env, napi_value o, gs_opts* opts) {
    gs_opts_default(opts);
    napi_valuetype t;
    if (napi_typeof(env, o, &t) != napi_ok || t != napi_object) return;
    auto field = [&](const char* name, double dflt) {
        bool has = false;
        napi_value v;
        if (napi_has_named_property(env, o, name, &has) != napi_ok || !has) return dflt;
        if (napi_get_named_property(env, o, name, &v) != napi_ok) return dflt;
        return num(env, v, dflt);
    };
    opts->accum = (int32_t)field("accum", opts->accum);
    opts->out_format = (int32_t)field("outFormat", opts->out_format);
    opts->t_min = (float)field("tMin", opts->t_min);
    opts->ref_quirks = (int32_t)field("refQuirks", opts->ref_quirks);
    opts->strip_index = (int32_t)field("stripIndex", opts->strip_index);
    opts->strip_count = (int32_t)field("stripCount", opts->strip_count);
    opts->timing = (int32_t)field("timing", opts->timing);
    opts->chunk_fraction = (float)field("chunkFraction", opts->chunk_fraction);
    opts->tile_row_begin = (int32_t)field("tileRowBegin", opts->tile_row_begin);
    opts->tile_row_end = (int32_t)field("tileRowEnd", opts->tile_row_end);
    opts->list_split = (int32_t)field("listSplit", opts->list_split);
}

// ---- library / device --------------------------------------------------------------------
napi_value AbiVersion(napi_env env, napi_callback_info) {
    napi_value r;
    NAPI_OK(napi_create_int32(env, gs_abi_version(), &r));
    return r;
}

napi_value LastError(napi_env env, napi_callback_info) {
    napi_value r;
    const char* e = gs_last_error();
    NAPI_OK(napi_create_string_utf8(env, e, strlen(e), &r));
    return r;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
    int n = 0;
    gs_device_count(&n);
    napi_value r;
    NAPI_OK(napi_create_int32(env, n, &r));
    return r;
}

// ctxCreate(deviceIndex | [device, ...]): one device, or a device group (row strips on each, one
// RCCL all-gather; gs_ctx_create)
napi_value CtxCreate(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    std::vector<int> devs;
    bool is_array = false;
    NAPI_OK(napi_is_array(env, argv[0], &is_array));
    if (is_array) {
        uint32_t len = 0;
        NAPI_OK(napi_get_array_length(env, argv[0], &len));
        for (uint32_t k = 0; k < len; ++k) {
            napi_value e;
            NAPI_OK(napi_get_element(env, argv[0], k, &e));
            devs.push_back((int)num(env, e, -1));
        }
        if (devs.empty()) return throw_gs(env, GS_ERR_INVALID, "ctxCreate: empty device list");
    } else {
        devs.push_back((int)num(env, argv[0], 0));
    }
    gs_ctx* c = nullptr;
    const int rc = gs_ctx_create(devs.data(), (int)devs.size(), &c);
    if (rc) return throw_gs(env, rc, "gs_ctx_create");
    napi_value r;
    NAPI_OK(napi_create_external(env, c, nullptr, nullptr, &r));
    return r;
}

napi_value CtxDestroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    gs_ctx* c;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "ctxDestroy: bad handle");
    gs_ctx_destroy(c);
    return undefined(env);
}

// ---- scenes ------------------------------------------------------------------------------
napi_value SceneUpload(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    get_args(env, info, 4, argv);
    gs_ctx* c;
    void* data;
    size_t len;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "sceneUpload: bad context");
    if (!get_bytes(env, argv[1], &data, &len)) return throw_gs(env, GS_ERR_INVALID, "sceneUpload: aos must be an ArrayBuffer/TypedArray");
    const double n = num(env, argv[2], -1), nsh = num(env, argv[3], 16);
    if (n < 0 || n * (64.0 + 16.0 * nsh) > (double)len)
        return throw_gs(env, GS_ERR_INVALID, "sceneUpload: buffer smaller than numGaussians records");
    gs_scene* s = nullptr;
    const int rc = gs_scene_upload(c, data, (uint64_t)n, (int)nsh, &s);
    if (rc) return throw_gs(env, rc, "gs_scene_upload");
    napi_value r;
    NAPI_OK(napi_create_external(env, s, nullptr, nullptr, &r));
    return r;
}

napi_value SceneFree(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    gs_scene* s;
    if (!get_handle(env, argv[0], &s)) return throw_gs(env, GS_ERR_INVALID, "sceneFree: bad handle");
    gs_scene_free(s);
    return undefined(env);
}

// ---- render ------------------------------------------------------------------------------
struct RenderArgs {
    gs_ctx* c = nullptr;
    gs_scene* s = nullptr;
    float uni[40];
    int W = 0, H = 0;
    gs_opts opts;
    void* out = nullptr;
    size_t out_len = 0;
};

// Parses (ctx, scene, uniforms, W, H, opts, out) and checks the output size.
napi_value parse_render(napi_env env, napi_value* argv, RenderArgs* a) {
    void* u;
    size_t ulen;
    if (!get_handle(env, argv[0], &a->c)) return throw_gs(env, GS_ERR_INVALID, "render: bad context");
    if (!get_handle(env, argv[1], &a->s)) return throw_gs(env, GS_ERR_INVALID, "render: bad scene");
    if (!get_bytes(env, argv[2], &u, &ulen) || ulen < 160)
        return throw_gs(env, GS_ERR_INVALID, "render: uniforms must hold 160 bytes");
    std::memcpy(a->uni, u, 160);
    a->W = (int)num(env, argv[3], 0);
    a->H = (int)num(env, argv[4], 0);
    read_opts(env, argv[5], &a->opts);
    napi_valuetype t;
    napi_typeof(env, argv[6], &t);
    if (t != napi_null && t != napi_undefined) {
        if (!get_bytes(env, argv[6], &a->out, &a->out_len))
            return throw_gs(env, GS_ERR_INVALID, "render: out must be a TypedArray or null");
        int row0 = 0, rows = a->H;
        bool sized = a->W > 0 && a->H > 0;  // a bad size or range: gs_render reports it, not the size check
        if (a->opts.tile_row_end > 0 || a->opts.tile_row_begin != 0) {
            const int TR = (a->H + 15) / 16;
            sized = sized && a->opts.strip_count == 1 && a->opts.tile_row_begin >= 0 &&
                    a->opts.tile_row_begin < a->opts.tile_row_end && a->opts.tile_row_end <= TR;
            if (sized) rows = std::min(16 * a->opts.tile_row_end, a->H) - 16 * a->opts.tile_row_begin;
        } else if (a->opts.strip_count > 1) {
            sized = sized && gs_strip_rows(a->H, a->opts.strip_index, a->opts.strip_count, &row0, &rows) == GS_OK;
        }
        const size_t need = sized ? (size_t)rows * (size_t)a->W * (a->opts.out_format == GS_OUT_RGBA_F16 ? 8 : 16) : 0;
        if (a->out_len < need) return throw_gs(env, GS_ERR_INVALID, "render: out buffer too small");
    }
    return undefined(env);
}

napi_value Render(napi_env env, napi_callback_info info) {
    napi_value argv[7];
    get_args(env, info, 7, argv);
    RenderArgs a;
    bool pending = false;
    if (!parse_render(env, argv, &a) || (napi_is_exception_pending(env, &pending), pending)) return nullptr;
    const int rc = gs_render(a.c, a.s, a.uni, a.W, a.H, &a.opts, a.out);
    if (rc) return throw_gs(env, rc, "gs_render");
    return undefined(env);
}

struct AsyncRender {
    RenderArgs a;
    int rc = 0;
    std::string err;
    napi_ref out_ref = nullptr;  // keeps the output array alive while the frame runs
    napi_deferred deferred = nullptr;
    napi_async_work work = nullptr;
};

void render_execute(napi_env, void* data) {
    auto* w = static_cast<AsyncRender*>(data);
    w->rc = gs_render(w->a.c, w->a.s, w->a.uni, w->a.W, w->a.H, &w->a.opts, w->a.out);
    if (w->rc) w->err = gs_last_error();  // thread-local: read on the worker thread
}

void render_complete(napi_env env, napi_status, void* data) {
    auto* w = static_cast<AsyncRender*>(data);
    if (w->rc == 0) {
        napi_resolve_deferred(env, w->deferred, undefined(env));
    } else {
        std::string msg = "gs_render: " + w->err;
        napi_value m, c, err;
        napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
        napi_create_int32(env, w->rc, &c);
        napi_create_error(env, nullptr, m, &err);
        napi_set_named_property(env, err, "code", c);
        napi_reject_deferred(env, w->deferred, err);
    }
    if (w->out_ref) napi_delete_reference(env, w->out_ref);
    napi_delete_async_work(env, w->work);
    delete w;
}

napi_value RenderAsync(napi_env env, napi_callback_info info) {
    napi_value argv[7];
    get_args(env, info, 7, argv);
    auto* w = new AsyncRender();
    bool pending = false;
    if (!parse_render(env, argv, &w->a) || (napi_is_exception_pending(env, &pending), pending)) {
        delete w;
        return nullptr;
    }
    napi_valuetype t;
    napi_typeof(env, argv[6], &t);
    if (t == napi_object) napi_create_reference(env, argv[6], 1, &w->out_ref);
    napi_value promise, name;
    napi_create_promise(env, &w->deferred, &promise);
    napi_create_string_utf8(env, "gs_render", NAPI_AUTO_LENGTH, &name);
    napi_create_async_work(env, nullptr, name, render_execute, render_complete, w, &w->work);
    napi_queue_async_work(env, w->work);
    return promise;
}

// ---- device-resident frames (the reference's GPU framebuffer texture) ----------------------
// fbAlloc(ctx, bytes) -> handle; fbFree(ctx, fb); fbRead(ctx, fb, typedArray): waits for the
// context's frames, then copies the array's byte length out of the framebuffer.
napi_value FbAlloc(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    get_args(env, info, 2, argv);
    gs_ctx* c;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "fbAlloc: bad context");
    void* dev = nullptr;
    const int rc = gs_framebuffer_alloc(c, (uint64_t)num(env, argv[1], 0), &dev);
    if (rc) return throw_gs(env, rc, "gs_framebuffer_alloc");
    napi_value r;
    NAPI_OK(napi_create_external(env, dev, nullptr, nullptr, &r));
    return r;
}

napi_value FbFree(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    get_args(env, info, 2, argv);
    gs_ctx* c;
    void* dev;
    if (!get_handle(env, argv[0], &c) || !get_handle(env, argv[1], &dev))
        return throw_gs(env, GS_ERR_INVALID, "fbFree: bad handle");
    const int rc = gs_framebuffer_free(c, dev);
    if (rc) return throw_gs(env, rc, "gs_framebuffer_free");
    return undefined(env);
}

napi_value FbRead(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    gs_ctx* c;
    void *dev, *host;
    size_t len;
    if (!get_handle(env, argv[0], &c) || !get_handle(env, argv[1], &dev))
        return throw_gs(env, GS_ERR_INVALID, "fbRead: bad handle");
    if (!get_bytes(env, argv[2], &host, &len)) return throw_gs(env, GS_ERR_INVALID, "fbRead: target must be a TypedArray");
    const int rc = gs_framebuffer_read(c, dev, host, len);
    if (rc) return throw_gs(env, rc, "gs_framebuffer_read");
    return undefined(env);
}

// hostRegister(ctx, typedArray) / hostUnregister(ctx, typedArray): page-lock a host array so
// readbacks into it are asynchronous DMA (gs_host_register); unregister before dropping it.
napi_value HostRegister(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    get_args(env, info, 2, argv);
    gs_ctx* c;
    void* host;
    size_t len;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "hostRegister: bad context");
    if (!get_bytes(env, argv[1], &host, &len)) return throw_gs(env, GS_ERR_INVALID, "hostRegister: not a TypedArray");
    const int rc = gs_host_register(c, host, len);
    if (rc) return throw_gs(env, rc, "gs_host_register");
    return undefined(env);
}

napi_value HostUnregister(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    get_args(env, info, 2, argv);
    gs_ctx* c;
    void* host;
    size_t len;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "hostUnregister: bad context");
    if (!get_bytes(env, argv[1], &host, &len)) return throw_gs(env, GS_ERR_INVALID, "hostUnregister: not a TypedArray");
    const int rc = gs_host_unregister(c, host);
    if (rc) return throw_gs(env, rc, "gs_host_unregister");
    return undefined(env);
}

// readbackAsync(ctx, fb, typedArray) -> Promise: enqueues the copy of the array's byte length out
// of the framebuffer behind the frames enqueued so far (gs_readback_start, on this thread, so in
// call order with renderDevice) and resolves once it has landed (gs_readback_wait on the libuv
// pool); the next frames render meanwhile.
struct AsyncReadback {
    gs_ctx* c = nullptr;
    uint32_t ticket = 0;
    int rc = 0;
    std::string err;
    napi_ref out_ref = nullptr;
    napi_deferred deferred = nullptr;
    napi_async_work work = nullptr;
};

void readback_execute(napi_env, void* data) {
    auto* w = static_cast<AsyncReadback*>(data);
    w->rc = gs_readback_wait(w->c, w->ticket);
    if (w->rc) w->err = gs_last_error();
}

void readback_complete(napi_env env, napi_status, void* data) {
    auto* w = static_cast<AsyncReadback*>(data);
    if (w->rc == 0) {
        napi_resolve_deferred(env, w->deferred, undefined(env));
    } else {
        std::string msg = "gs_readback_wait: " + w->err;
        napi_value m, c, err;
        napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
        napi_create_int32(env, w->rc, &c);
        napi_create_error(env, nullptr, m, &err);
        napi_set_named_property(env, err, "code", c);
        napi_reject_deferred(env, w->deferred, err);
    }
    if (w->out_ref) napi_delete_reference(env, w->out_ref);
    napi_delete_async_work(env, w->work);
    delete w;
}

napi_value ReadbackAsync(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    gs_ctx* c;
    void *dev, *host;
    size_t len;
    if (!get_handle(env, argv[0], &c) || !get_handle(env, argv[1], &dev))
        return throw_gs(env, GS_ERR_INVALID, "readbackAsync: bad handle");
    if (!get_bytes(env, argv[2], &host, &len)) return throw_gs(env, GS_ERR_INVALID, "readbackAsync: target must be a TypedArray");
    auto* w = new AsyncReadback();
    w->c = c;
    const int rc = gs_readback_start(c, dev, host, len, &w->ticket);
    if (rc) {
        delete w;
        return throw_gs(env, rc, "gs_readback_start");
    }
    napi_create_reference(env, argv[2], 1, &w->out_ref);  // the array stays alive until the copy lands
    napi_value promise, name;
    napi_create_promise(env, &w->deferred, &promise);
    napi_create_string_utf8(env, "gs_readback", NAPI_AUTO_LENGTH, &name);
    napi_create_async_work(env, nullptr, name, readback_execute, readback_complete, w, &w->work);
    napi_queue_async_work(env, w->work);
    return promise;
}

// renderDevice(ctx, scene, uniforms, W, H, opts, fb, fbBytes): enqueues the frame into the device
// framebuffer and returns (frames in flight; errors of earlier frames are thrown here).
napi_value RenderDevice(napi_env env, napi_callback_info info) {
    napi_value argv[8];
    get_args(env, info, 8, argv);
    RenderArgs a;
    napi_value args7[7] = {argv[0], argv[1], argv[2], argv[3], argv[4], argv[5], nullptr};
    napi_get_null(env, &args7[6]);
    bool pending = false;
    if (!parse_render(env, args7, &a) || (napi_is_exception_pending(env, &pending), pending)) return nullptr;
    void* dev;
    if (!get_handle(env, argv[6], &dev)) return throw_gs(env, GS_ERR_INVALID, "renderDevice: bad framebuffer");
    const int rc = gs_render_device(a.c, a.s, a.uni, a.W, a.H, &a.opts, dev, (uint64_t)num(env, argv[7], 0), nullptr);
    if (rc) return throw_gs(env, rc, "gs_render_device");
    return undefined(env);
}

// presentDevice(ctx, fb, fbFormat, W, H, outFormat, outFb, outBytes): PostProcessRenderer on the device
napi_value PresentDevice(napi_env env, napi_callback_info info) {
    napi_value argv[8];
    get_args(env, info, 8, argv);
    gs_ctx* c;
    void *fb, *out;
    if (!get_handle(env, argv[0], &c) || !get_handle(env, argv[1], &fb) || !get_handle(env, argv[6], &out))
        return throw_gs(env, GS_ERR_INVALID, "presentDevice: bad handle");
    const int rc = gs_present_device(c, fb, (int)num(env, argv[2], 0), (int)num(env, argv[3], 0),
                                     (int)num(env, argv[4], 0), (int)num(env, argv[5], 0), out,
                                     (uint64_t)num(env, argv[7], 0), nullptr);
    if (rc) return throw_gs(env, rc, "gs_present_device");
    return undefined(env);
}

napi_value Timings(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    gs_ctx* c;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "timings: bad context");
    gs_stats st;
    const int rc = gs_timings(c, &st);
    if (rc) return throw_gs(env, rc, "gs_timings");
    napi_value o;
    NAPI_OK(napi_create_object(env, &o));
    auto put = [&](const char* k, double v) {
        napi_value x;
        napi_create_double(env, v, &x);
        napi_set_named_property(env, o, k, x);
    };
    put("n", (double)st.n);
    put("nVis", (double)st.n_vis);
    put("kEntries", (double)st.k_entries);
    put("kTotal", (double)st.k_total);
    put("tilesUnsaturated", st.tiles_unsaturated);
    put("chunkFraction", st.chunk_fraction);
    put("frames", st.frames);
    put("msTotal", st.ms_total);
    put("msProject", st.ms_project);
    put("msSort", st.ms_sort);
    put("msBin", st.ms_bin);
    put("msTileSort", st.ms_tile_sort);
    put("msRanges", st.ms_ranges);
    put("msComposite", st.ms_composite);
    put("framesRendered", st.frames_rendered);
    put("framesChunked", st.frames_chunked);
    put("framesUnsat", st.frames_unsat);
    put("framesSeeded", st.frames_seeded);
    put("chunkDepth", st.chunk_depth);
    put("listMax", st.list_max);
    put("tilesLong", st.tiles_long);
    return o;
}

napi_value TimingsReset(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    gs_ctx* c;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "timingsReset: bad context");
    gs_timings_reset(c);
    return undefined(env);
}

napi_value Sync(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    gs_ctx* c;
    if (!get_handle(env, argv[0], &c)) return throw_gs(env, GS_ERR_INVALID, "sync: bad context");
    const int rc = gs_sync(c);
    if (rc) return throw_gs(env, rc, "gs_sync");
    return undefined(env);
}

// ---- host helpers ------------------------------------------------------------------------
napi_value Present(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    get_args(env, info, 4, argv);
    void *in, *out;
    size_t lin, lout;
    const int W = (int)num(env, argv[1], 0), H = (int)num(env, argv[2], 0);
    if (!get_bytes(env, argv[0], &in, &lin) || !get_bytes(env, argv[3], &out, &lout) ||
        W <= 0 || H <= 0 || lin < (size_t)W * H * 16 || lout < (size_t)W * H * 16)
        return throw_gs(env, GS_ERR_INVALID, "present: need W*H*4 float32 in and out");
    const int rc = gs_present((const float*)in, W, H, (float*)out);
    if (rc) return throw_gs(env, rc, "gs_present");
    return undefined(env);
}

napi_value new_f32(napi_env env, const float* v, size_t n) {
    void* p;
    napi_value ab, ta;
    napi_create_arraybuffer(env, n * 4, &p, &ab);
    std::memcpy(p, v, n * 4);
    napi_create_typedarray(env, napi_float32_array, n, ab, 0, &ta);
    return ta;
}

bool vec3(napi_env env, napi_value v, double out[3]) {
    for (uint32_t i = 0; i < 3; ++i) {
        napi_value e;
        if (napi_get_element(env, v, i, &e) != napi_ok) return false;
        if (napi_get_value_double(env, e, &out[i]) != napi_ok) return false;
    }
    return true;
}

napi_value LookAt(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    double e[3], t[3], u[3];
    if (!vec3(env, argv[0], e) || !vec3(env, argv[1], t) || !vec3(env, argv[2], u))
        return throw_gs(env, GS_ERR_INVALID, "lookAt: eye/target/up must be 3-vectors");
    float m[16];
    gs_look_at(e, t, u, m);
    return new_f32(env, m, 16);
}

napi_value Perspective(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    get_args(env, info, 4, argv);
    float m[16];
    const int rc = gs_perspective(num(env, argv[0], 0), num(env, argv[1], 1), num(env, argv[2], 0.03),
                                  num(env, argv[3], 1000), m);
    if (rc) return throw_gs(env, rc, "gs_perspective");
    return new_f32(env, m, 16);
}

// cameraFromJSON (src/camera.ts:476-503): (rawCamera, canvasW, canvasH) -> {viewMatrix, perspective,
// focalX, focalY}
napi_value CameraFromJSON(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    double pos[3], rot[9], fx = 0, fy = 0;
    napi_value vpos, vrot, vfx, vfy;
    bool ok = napi_get_named_property(env, argv[0], "position", &vpos) == napi_ok && vec3(env, vpos, pos) &&
              napi_get_named_property(env, argv[0], "rotation", &vrot) == napi_ok &&
              napi_get_named_property(env, argv[0], "fx", &vfx) == napi_ok &&
              napi_get_value_double(env, vfx, &fx) == napi_ok &&
              napi_get_named_property(env, argv[0], "fy", &vfy) == napi_ok &&
              napi_get_value_double(env, vfy, &fy) == napi_ok;
    for (uint32_t r = 0; ok && r < 3; ++r) {
        napi_value row;
        ok = napi_get_element(env, vrot, r, &row) == napi_ok && vec3(env, row, rot + 3 * r);
    }
    if (!ok) return throw_gs(env, GS_ERR_INVALID, "cameraFromJSON: needs position[3], rotation[3][3], fx, fy");
    float view[16], proj[16], focal[2];
    const int rc = gs_camera_from_json(pos, rot, fx, fy, (int)num(env, argv[1], 0), (int)num(env, argv[2], 0),
                                       view, proj, focal);
    if (rc) return throw_gs(env, rc, "gs_camera_from_json");
    napi_value o, fxv, fyv;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "viewMatrix", new_f32(env, view, 16));
    napi_set_named_property(env, o, "perspective", new_f32(env, proj, 16));
    napi_create_double(env, focal[0], &fxv);
    napi_create_double(env, focal[1], &fyv);
    napi_set_named_property(env, o, "focalX", fxv);
    napi_set_named_property(env, o, "focalY", fyv);
    return o;
}

napi_value CameraPosition(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    void* v;
    size_t len;
    if (!get_bytes(env, argv[0], &v, &len) || len < 64) return throw_gs(env, GS_ERR_INVALID, "cameraPosition: view must be 16 floats");
    float p[3];
    gs_camera_position((const float*)v, p);
    return new_f32(env, p, 3);
}

napi_value PackUniforms(napi_env env, napi_callback_info info) {
    napi_value argv[8];
    get_args(env, info, 8, argv);
    void *view, *proj, *pos;
    size_t l0, l1, l2;
    if (!get_bytes(env, argv[0], &view, &l0) || !get_bytes(env, argv[1], &proj, &l1) ||
        !get_bytes(env, argv[2], &pos, &l2) || l0 < 64 || l1 < 64 || l2 < 12)
        return throw_gs(env, GS_ERR_INVALID, "packUniforms: view/proj (16 floats) and camPos (3 floats)");
    void* p;
    napi_value ab;
    NAPI_OK(napi_create_arraybuffer(env, 160, &p, &ab));
    gs_pack_uniforms((const float*)view, (const float*)proj, (const float*)pos, (float)num(env, argv[3], 0),
                     (float)num(env, argv[4], 0), (float)num(env, argv[5], 0), (float)num(env, argv[6], 0),
                     (float)num(env, argv[7], 1), p);
    return ab;
}

// PackedGaussians(arrayBuffer) (src/ply.ts:200-355): {aos, numGaussians, shDegree, nShCoeffs, minPos, maxPos}
// synthAos(n, seed, W, H) -> ArrayBuffer of n SH-degree-3 records (SURVEY §8d generator)
napi_value SynthAos(napi_env env, napi_callback_info info) {
    napi_value argv[4];
    get_args(env, info, 4, argv);
    const double n = num(env, argv[0], -1);
    if (!(n >= 0) || n * 320.0 > 2147483647.0) return throw_gs(env, GS_ERR_INVALID, "synthAos: bad count");
    void* p = nullptr;
    napi_value ab;
    NAPI_OK(napi_create_arraybuffer(env, (size_t)n * 320, &p, &ab));
    const int rc = gs_synth_aos((uint64_t)n, (uint64_t)num(env, argv[1], 1), (int)num(env, argv[2], 1920),
                                (int)num(env, argv[3], 1080), p);
    if (rc) return throw_gs(env, rc, "gs_synth_aos");
    return ab;
}

napi_value PlyParse(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    get_args(env, info, 1, argv);
    void* data;
    size_t len;
    if (!get_bytes(env, argv[0], &data, &len)) return throw_gs(env, GS_ERR_INVALID, "plyParse: need an ArrayBuffer");
    gs_ply_info pi;
    int rc = gs_ply_parse(data, len, &pi, nullptr, 0);
    if (rc) return throw_gs(env, rc, "gs_ply_parse");
    void* out;
    napi_value ab;
    const size_t bytes = (size_t)(pi.num_gaussians * pi.record_bytes);
    NAPI_OK(napi_create_arraybuffer(env, bytes, &out, &ab));
    rc = gs_ply_parse(data, len, &pi, out, bytes);
    if (rc) return throw_gs(env, rc, "gs_ply_parse");
    napi_value o, v;
    NAPI_OK(napi_create_object(env, &o));
    napi_set_named_property(env, o, "aos", ab);
    napi_create_double(env, (double)pi.num_gaussians, &v);
    napi_set_named_property(env, o, "numGaussians", v);
    napi_create_int32(env, pi.sh_degree, &v);
    napi_set_named_property(env, o, "shDegree", v);
    napi_create_int32(env, pi.n_sh_coeffs, &v);
    napi_set_named_property(env, o, "nShCoeffs", v);
    for (int k = 0; k < 2; ++k) {
        napi_value arr;
        napi_create_array_with_length(env, 3, &arr);
        for (uint32_t c = 0; c < 3; ++c) {
            napi_create_double(env, k ? pi.max_pos_d[c] : pi.min_pos_d[c], &v);
            napi_set_element(env, arr, c, v);
        }
        napi_set_named_property(env, o, k ? "maxPos" : "minPos", arr);
    }
    return o;
}

// encodePng(rgba8, W, H) -> ArrayBuffer: PNG of an RGBA8 image (row 0 = top), gs_encode_png
napi_value EncodePng(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    void* data;
    size_t len;
    if (!get_bytes(env, argv[0], &data, &len)) return throw_gs(env, GS_ERR_INVALID, "encodePng: need RGBA8 bytes");
    const int W = (int)num(env, argv[1], 0), H = (int)num(env, argv[2], 0);
    if (W <= 0 || H <= 0 || (uint64_t)len < 4ull * (uint64_t)W * (uint64_t)H)
        return throw_gs(env, GS_ERR_INVALID, "encodePng: buffer smaller than W*H*4");
    uint64_t need = 0;
    int rc = gs_encode_png((const uint8_t*)data, W, H, nullptr, 0, &need);
    if (rc) return throw_gs(env, rc, "gs_encode_png");
    void* out;
    napi_value ab;
    NAPI_OK(napi_create_arraybuffer(env, (size_t)need, &out, &ab));
    rc = gs_encode_png((const uint8_t*)data, W, H, (uint8_t*)out, need, &need);
    if (rc) return throw_gs(env, rc, "gs_encode_png");
    return ab;
}

napi_value StripRows(napi_env env, napi_callback_info info) {
    napi_value argv[3];
    get_args(env, info, 3, argv);
    int row0 = 0, rows = 0;
    const int rc = gs_strip_rows((int)num(env, argv[0], 0), (int)num(env, argv[1], 0), (int)num(env, argv[2], 1),
                                 &row0, &rows);
    if (rc) return throw_gs(env, rc, "gs_strip_rows");
    napi_value o, a, b;
    napi_create_object(env, &o);
    napi_create_int32(env, row0, &a);
    napi_create_int32(env, rows, &b);
    napi_set_named_property(env, o, "row0", a);
    napi_set_named_property(env, o, "rowsPadded", b);
    return o;
}

napi_value Init(napi_env env, napi_value exports) {
    const struct {
        const char* name;
        napi_callback cb;
    } fns[] = {
        {"abiVersion", AbiVersion}, {"lastError", LastError}, {"deviceCount", DeviceCount},
        {"ctxCreate", CtxCreate}, {"ctxDestroy", CtxDestroy}, {"sceneUpload", SceneUpload},
        {"sceneFree", SceneFree}, {"render", Render}, {"renderAsync", RenderAsync},
        {"timings", Timings}, {"timingsReset", TimingsReset}, {"sync", Sync}, {"present", Present},
        {"lookAt", LookAt}, {"perspective", Perspective}, {"cameraPosition", CameraPosition},
        {"cameraFromJSON", CameraFromJSON}, {"fbAlloc", FbAlloc}, {"fbFree", FbFree}, {"fbRead", FbRead},
        {"renderDevice", RenderDevice}, {"presentDevice", PresentDevice}, {"synthAos", SynthAos},
        {"hostRegister", HostRegister}, {"hostUnregister", HostUnregister}, {"readbackAsync", ReadbackAsync},
        {"packUniforms", PackUniforms}, {"stripRows", StripRows}, {"plyParse", PlyParse}, {"encodePng", EncodePng},
    };
    for (const auto& f : fns) {
        napi_value fn;
        NAPI_OK(napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &fn));
        NAPI_OK(napi_set_named_property(env, exports, f.name, fn));
    }
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
