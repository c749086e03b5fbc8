// napi_addon.cpp — Node N-API binding of librt_hip.so (rt_napi.node).
//
// The JS host (blenderraytracer_amd/js/gpu-ray-tracer.mjs) keeps the reference's RayTracer surface
// and calls into this addon for the part under RayTracer.render (js/ray-tracer.js:166-281):
//   createScene(desc, device)          -> External   (rt_scene_create: scene copied into HBM)
//   render(scene, settings, progress?) -> Promise<{mean?, post?, rgba8, segments?, draws?, stats}>
//                                         (rt_render on a libuv worker thread: the event loop stays live)
//   cancel(scene)                      -> rt_cancel (the queued batches stop at their next item)
//   checkpoint(scene) -> {sums, samplesDone}; checkpointSamples(scene) -> samplesDone (sums stay resident)
//   destroyScene(scene), deviceCount(), abiVersion()
// Progress reaches JS through a napi_threadsafe_function, in order and before the Promise settles (the
// worker waits until the main thread has run each call, as the reference calls onProgress inside its
// loop, ray-tracer.js:256-261); with settings.preview the caller's imageData receives the frame of the
// samples traced so far at every progress call (the reference's per-row putImageData, :224-241).  The
// worker thread never writes into JS memory: frames land in job-owned buffers and are copied into the
// caller's array on the main thread, after checking it was not detached.  C errors reject the Promise
// with Error(rt_last_error()).  Built with plain g++ against node_api.h (no node-gyp).
#define NAPI_VERSION 6
#include <node_api.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <string>
#include <vector>

#include "rt_hip.h"

namespace {

#define NAPI_OK(call)                                                       \
    do {                                                                    \
        if ((call) != napi_ok) {                                            \
            napi_throw_error(env, nullptr, "N-API call failed: " #call);   \
            return nullptr;                                                 \
        }                                                                   \
    } while (0)

napi_value throw_err(napi_env env, const std::string& msg) {
    napi_throw_error(env, nullptr, msg.c_str());
    return nullptr;
}

bool get_prop(napi_env env, napi_value obj, const char* key, napi_value* out) {
    bool has = false;
    if (napi_has_named_property(env, obj, key, &has) != napi_ok || !has) return false;
    if (napi_get_named_property(env, obj, key, out) != napi_ok) return false;
    napi_valuetype t;
    napi_typeof(env, *out, &t);
    return t != napi_undefined && t != napi_null;
}

double get_num(napi_env env, napi_value obj, const char* key, double dflt) {
    napi_value v;
    double d = dflt;
    if (get_prop(env, obj, key, &v)) napi_get_value_double(env, v, &d);
    return d;
}

// Up to `max` numbers of an Array property (e.g. settings.devices); returns how many were read.
int get_int_array(napi_env env, napi_value obj, const char* key, int32_t* out, int max) {
    napi_value v;
    if (!get_prop(env, obj, key, &v)) return 0;
    bool is = false;
    if (napi_is_array(env, v, &is) != napi_ok || !is) return 0;
    uint32_t len = 0;
    napi_get_array_length(env, v, &len);
    int n = 0;
    for (uint32_t i = 0; i < len && n < max; ++i) {
        napi_value e;
        double d = 0;
        if (napi_get_element(env, v, i, &e) != napi_ok || napi_get_value_double(env, e, &d) != napi_ok) return -1;
        out[n++] = (int32_t)d;
    }
    return len > (uint32_t)max ? -1 : n;
}

// Raw bytes of a TypedArray / ArrayBuffer / DataView value.
bool get_bytes_value(napi_env env, napi_value v, void** data, size_t* bytes) {
    *data = nullptr;
    *bytes = 0;
    bool is;
    if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
        napi_typedarray_type t;
        size_t len, off;
        napi_value ab;
        void* p;
        napi_get_typedarray_info(env, v, &t, &len, &p, &ab, &off);
        size_t el = (t == napi_float64_array || t == napi_bigint64_array || t == napi_biguint64_array) ? 8
                    : (t == napi_int32_array || t == napi_uint32_array || t == napi_float32_array) ? 4
                    : (t == napi_int16_array || t == napi_uint16_array) ? 2 : 1;
        *data = p;
        *bytes = len * el;
        return true;
    }
    if (napi_is_arraybuffer(env, v, &is) == napi_ok && is) {
        napi_get_arraybuffer_info(env, v, data, bytes);
        return true;
    }
    if (napi_is_dataview(env, v, &is) == napi_ok && is) {
        napi_value ab;
        size_t off;
        napi_get_dataview_info(env, v, bytes, data, &ab, &off);
        return true;
    }
    return false;
}

// ... of a property
bool get_bytes(napi_env env, napi_value obj, const char* key, void** data, size_t* bytes) {
    napi_value v;
    *data = nullptr;
    *bytes = 0;
    if (!get_prop(env, obj, key, &v)) return false;
    return get_bytes_value(env, v, data, bytes);
}

// The External owns a SceneBox: destroyScene() frees the device scene eagerly, the GC finalizer
// frees whatever is left; one render may be in flight per scene (rt_hip.h threading rule).
struct SceneBox {
    rt_scene* sc = nullptr;
    bool busy = false;
    size_t last_pixels = 0;         // crop pixels of the last render (checkpoint size)
    // frame buffers of render() into a caller's imageData, reused from render to render (no per-frame
    // allocation or page faults): the finished RGBA8 frame and the running preview frame
    std::vector<uint8_t> frame, preview;
};

void scene_finalize(napi_env, void* data, void*) {
    SceneBox* box = static_cast<SceneBox*>(data);
    if (box->sc) rt_scene_destroy(box->sc);
    delete box;
}

SceneBox* get_box(napi_env env, napi_value v) {
    void* p = nullptr;
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok || t != napi_external) return nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok) return nullptr;
    return static_cast<SceneBox*>(p);
}

// createScene(desc, device): desc holds the rt_scene_desc records as typed arrays (layout: rt_hip.h)
napi_value create_scene(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 1) return throw_err(env, "createScene(desc, device)");
    napi_value d = argv[0];
    int32_t device = 0;
    if (argc > 1) napi_get_value_int32(env, argv[1], &device);
    rt_scene_desc desc;
    std::memset(&desc, 0, sizeof desc);
    desc.abi_version = RT_ABI_VERSION;
    void* p;
    size_t n;
    if (get_bytes(env, d, "objects", &p, &n)) {
        desc.objects = static_cast<const rt_object_desc*>(p);
        desc.num_objects = (int32_t)(n / sizeof(rt_object_desc));
    }
    if (get_bytes(env, d, "materials", &p, &n)) {
        desc.materials = static_cast<const rt_material_desc*>(p);
        desc.num_materials = (int32_t)(n / sizeof(rt_material_desc));
    }
    if (get_bytes(env, d, "triangles", &p, &n)) {
        desc.triangles = static_cast<const double*>(p);
        desc.num_triangles = (int32_t)(n / (12 * sizeof(double)));
    }
    if (!get_bytes(env, d, "camera", &p, &n) || n != 22 * sizeof(double))
        return throw_err(env, "desc.camera must be a Float64Array(22): origin, lowerLeft, horizontal, vertical, u, v, w, lensRadius");
    const double* c = static_cast<const double*>(p);
    std::memcpy(desc.camera.origin, c + 0, 24);
    std::memcpy(desc.camera.lower_left, c + 3, 24);
    std::memcpy(desc.camera.horizontal, c + 6, 24);
    std::memcpy(desc.camera.vertical, c + 9, 24);
    std::memcpy(desc.camera.u, c + 12, 24);
    std::memcpy(desc.camera.v, c + 15, 24);
    std::memcpy(desc.camera.w, c + 18, 24);
    desc.camera.lens_radius = c[21];
    desc.camera.type = (int32_t)get_num(env, d, "cameraType", RT_CAM_PERSPECTIVE);
    desc.background = (int32_t)get_num(env, d, "background", RT_BG_GRADIENT);
    desc.sky_intensity = get_num(env, d, "skyIntensity", 1.0);
    if (get_bytes(env, d, "solidColor", &p, &n) && n == 3 * sizeof(double)) std::memcpy(desc.solid_color, p, 24);
    if (!get_bytes(env, d, "perm", &p, &n) || n != 512 * sizeof(int32_t))
        return throw_err(env, "desc.perm must be an Int32Array(512) (World.cloudNoise.p)");
    std::memcpy(desc.perm, p, sizeof desc.perm);
    rt_scene* sc = nullptr;
    if (rt_scene_create(&desc, device, &sc) != RT_OK) return throw_err(env, std::string("rt_scene_create: ") + rt_last_error());
    SceneBox* box = new SceneBox();
    box->sc = sc;
    napi_value ext;
    NAPI_OK(napi_create_external(env, box, scene_finalize, nullptr, &ext));
    return ext;
}

struct RenderJob {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_threadsafe_function tsfn = nullptr;
    napi_ref scene_ref = nullptr;   // keeps the External (and its rt_scene) alive while rendering
    SceneBox* box = nullptr;
    rt_scene* scene = nullptr;
    rt_settings st{};
    size_t n = 0;
    bool want_mean = false, want_counts = false, want_post = true;
    // outputs live in JS ArrayBuffers created on the main thread before the work is queued (kept alive
    // by references, not visible to JS until the promise resolves): rt_render copies the frames from
    // HBM straight into them.  settings.outRgba8 (the caller's imageData.data) is written only on the
    // main thread: the final frame in complete(), preview frames in call_progress.
    enum { OUT_POST, OUT_RGBA, OUT_MEAN, OUT_SEGS, OUT_DRAWS, OUT_N };
    napi_ref out_ref[OUT_N] = {};
    void* out_ptr[OUT_N] = {};
    napi_ref caller_rgba = nullptr;  // settings.outRgba8
    uint8_t* frame = nullptr;        // rt_output.rgba8 when the caller gave outRgba8 (SceneBox::frame)
    uint8_t* preview = nullptr;      // rt_output.preview_rgba8 (settings.preview; SceneBox::preview)
    int32_t preview_samples = 0;     // rt_output.preview_samples: the frame's samples (written by the worker)
    int32_t shown_samples = 0;       // the frame last copied into the caller's imageData (main thread)
    // progress hand-off: the worker waits until the main thread ran the JS callback
    std::mutex m;
    std::condition_variable cv;
    bool pending = false;
    double fraction = 0;
    rt_stats stats{};
    int status = 0;
    std::string error;
    std::atomic<int> cancel_from_js{0};
    std::vector<double> resume;     // settings.resumeSums (rt_render_resume)
    int32_t resume_done = -1;
    bool resume_resident = false;   // settings.resumeResident: the scene's own checkpoint (sums NULL)
};

// The caller's typed array behind `ref` if it is still attached and holds `bytes` bytes, else nullptr.
uint8_t* live_bytes(napi_env env, napi_ref ref, size_t bytes) {
    napi_value v;
    if (!ref || napi_get_reference_value(env, ref, &v) != napi_ok || !v) return nullptr;
    void* p = nullptr;
    size_t got = 0;
    if (!get_bytes_value(env, v, &p, &got) || got != bytes) return nullptr;   // detached: length 0
    return static_cast<uint8_t*>(p);
}

void call_progress(napi_env env, napi_value js_cb, void*, void* data) {
    RenderJob* job = static_cast<RenderJob*>(data);     // alive: the worker waits for this call
    if (env) {
        if (job->preview && job->preview_samples != job->shown_samples)   // a newer frame only
            if (uint8_t* dst = live_bytes(env, job->caller_rgba, job->n * 4)) {
                std::memcpy(dst, job->preview, job->n * 4);
                job->shown_samples = job->preview_samples;
            }
        if (js_cb) {
            napi_value arg, undef;
            napi_create_double(env, job->fraction, &arg);
            napi_get_undefined(env, &undef);
            napi_call_function(env, undef, js_cb, 1, &arg, nullptr);
        }
    }
    std::lock_guard<std::mutex> lk(job->m);
    job->pending = false;
    job->cv.notify_all();
}

// RT_NAPI_TRACE=1 (developer A/B): stderr timestamps of the progress hand-off
double trace_ms() {
    static const bool on = getenv("RT_NAPI_TRACE") && getenv("RT_NAPI_TRACE")[0] == '1';
    if (!on) return -1;
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int progress_hook(double fraction, void* user) {
    RenderJob* job = static_cast<RenderJob*>(user);
    const double t0 = trace_ms();
    if (job->tsfn) {
        {
            std::lock_guard<std::mutex> lk(job->m);
            job->pending = true;
            job->fraction = fraction;
        }
        if (napi_call_threadsafe_function(job->tsfn, job, napi_tsfn_blocking) == napi_ok) {
            std::unique_lock<std::mutex> lk(job->m);
            job->cv.wait(lk, [job] { return !job->pending; });
        }
    }
    if (t0 >= 0) fprintf(stderr, "[napi] progress %.3f at %.3f ms, hand-off %.3f ms\n", fraction, t0, trace_ms() - t0);
    return job->cancel_from_js.load();
}

void execute(napi_env, void* data) {
    RenderJob* job = static_cast<RenderJob*>(data);
    rt_output out{};
    out.post = static_cast<float*>(job->out_ptr[RenderJob::OUT_POST]);
    out.rgba8 = job->frame ? job->frame : static_cast<uint8_t*>(job->out_ptr[RenderJob::OUT_RGBA]);
    out.mean = static_cast<double*>(job->out_ptr[RenderJob::OUT_MEAN]);
    out.segments = static_cast<uint32_t*>(job->out_ptr[RenderJob::OUT_SEGS]);
    out.draws = static_cast<uint32_t*>(job->out_ptr[RenderJob::OUT_DRAWS]);
    out.preview_rgba8 = job->preview;
    out.preview_samples = &job->preview_samples;
    const double t0 = trace_ms();
    if (t0 >= 0) fprintf(stderr, "[napi] rt_render start %.3f ms\n", t0);
    if (job->resume_done >= 0)
        job->status = rt_render_resume(job->scene, &job->st, job->resume_resident ? nullptr : job->resume.data(),
                                       job->resume_done, &out, progress_hook, job, &job->stats);
    else
        job->status = rt_render(job->scene, &job->st, &out, progress_hook, job, &job->stats);
    if (job->status != RT_OK) job->error = rt_last_error();
    if (t0 >= 0) fprintf(stderr, "[napi] rt_render end %.3f ms (%.3f)\n", trace_ms(), trace_ms() - t0);
}

// A new ArrayBuffer of `bytes` on the main thread, referenced by the job until it completes.
bool make_out(napi_env env, RenderJob* job, int slot, size_t bytes) {
    napi_value ab;
    if (napi_create_arraybuffer(env, bytes, &job->out_ptr[slot], &ab) != napi_ok) return false;
    return napi_create_reference(env, ab, 1, &job->out_ref[slot]) == napi_ok;
}

// The typed array over output slot `slot` (the ArrayBuffer, or the caller's own typed array).
napi_value out_array(napi_env env, RenderJob* job, int slot, napi_typedarray_type t, size_t len) {
    napi_value v, arr;
    napi_get_reference_value(env, job->out_ref[slot], &v);
    napi_create_typedarray(env, t, len, v, 0, &arr);
    return arr;
}

template <class T>
napi_value to_typed(napi_env env, const std::vector<T>& v, napi_typedarray_type t) {
    napi_value ab, arr;
    void* p = nullptr;
    napi_create_arraybuffer(env, v.size() * sizeof(T), &p, &ab);
    if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    napi_create_typedarray(env, t, v.size(), ab, 0, &arr);
    return arr;
}

void complete(napi_env env, napi_status, void* data) {
    RenderJob* job = static_cast<RenderJob*>(data);
    if (job->tsfn) napi_release_threadsafe_function(job->tsfn, napi_tsfn_release);
    // the caller's imageData.data: the finished frame, or after a cancel the frame of the checkpointed
    // samples (rt_output.preview_rgba8); a buffer detached or transferred meanwhile fails the render
    if (job->caller_rgba && (job->status == RT_OK || (job->status == RT_ERR_CANCELLED && job->preview))) {
        uint8_t* dst = live_bytes(env, job->caller_rgba, job->n * 4);
        const uint8_t* src = job->status == RT_OK ? job->frame : job->preview;
        if (dst) std::memcpy(dst, src, job->n * 4);
        else if (job->status == RT_OK) {
            job->status = RT_ERR_INVALID;
            job->error = "render: settings.outRgba8 was detached or resized while rendering";
        }
    }
    if (job->status != RT_OK) {
        napi_value msg, err, code;
        napi_create_string_utf8(env, job->error.c_str(), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, nullptr, msg, &err);
        napi_create_int32(env, job->status, &code);
        napi_set_named_property(env, err, "status", code);
        napi_reject_deferred(env, job->deferred, err);
    } else {
        napi_value res, stats, v;
        napi_create_object(env, &res);
        if (job->want_post)
            napi_set_named_property(env, res, "post", out_array(env, job, RenderJob::OUT_POST, napi_float32_array, job->n * 4));
        napi_value rgba;
        if (job->caller_rgba) napi_get_reference_value(env, job->caller_rgba, &rgba);
        else rgba = out_array(env, job, RenderJob::OUT_RGBA, napi_uint8_clamped_array, job->n * 4);
        napi_set_named_property(env, res, "rgba8", rgba);
        if (job->want_mean) napi_set_named_property(env, res, "mean", out_array(env, job, RenderJob::OUT_MEAN, napi_float64_array, job->n * 3));
        if (job->want_counts) {
            napi_set_named_property(env, res, "segments", out_array(env, job, RenderJob::OUT_SEGS, napi_uint32_array, job->n));
            napi_set_named_property(env, res, "draws", out_array(env, job, RenderJob::OUT_DRAWS, napi_uint32_array, job->n));
        }
        napi_create_object(env, &stats);
        const struct { const char* k; double v; } fields[] = {
            {"kernelMs", job->stats.kernel_ms}, {"finalizeMs", job->stats.finalize_ms}, {"wallMs", job->stats.wall_ms},
            {"samples", (double)job->stats.samples}, {"segments", (double)job->stats.segments},
            {"primTests", (double)job->stats.prim_tests}, {"algorithmicBytes", job->stats.algorithmic_bytes},
            {"nodeVisits", (double)job->stats.node_visits}};
        for (const auto& f : fields) {
            napi_create_double(env, f.v, &v);
            napi_set_named_property(env, stats, f.k, v);
        }
        napi_set_named_property(env, res, "stats", stats);
        napi_resolve_deferred(env, job->deferred, res);
    }
    job->box->busy = false;
    for (napi_ref r : job->out_ref)
        if (r) napi_delete_reference(env, r);
    if (job->caller_rgba) napi_delete_reference(env, job->caller_rgba);
    napi_delete_reference(env, job->scene_ref);
    napi_delete_async_work(env, job->work);
    delete job;
}

// render(scene, settings, onProgress?) -> Promise
napi_value render(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 2) return throw_err(env, "render(scene, settings, onProgress?)");
    SceneBox* box = get_box(env, argv[0]);
    if (!box || !box->sc) return throw_err(env, "render: first argument is not a live scene");
    if (box->busy) return throw_err(env, "render: a render is already in flight on this scene");
    napi_value s = argv[1];
    RenderJob* job = new RenderJob();
    job->box = box;
    job->scene = box->sc;
    rt_settings& st = job->st;
    st.width = (int32_t)get_num(env, s, "width", 0);
    st.height = (int32_t)get_num(env, s, "height", 0);
    st.samples = (int32_t)get_num(env, s, "samples", 4);
    st.max_depth = (int32_t)get_num(env, s, "maxDepth", 5);
    st.aa_mode = (int32_t)get_num(env, s, "aaMode", RT_AA_SUPERSAMPLING);
    st.tone_map = (int32_t)get_num(env, s, "toneMap", RT_TM_REINHARD);
    st.exposure = get_num(env, s, "exposure", 1.0);
    st.gamma = get_num(env, s, "gamma", 2.2);
    st.seed = (uint32_t)get_num(env, s, "seed", 0);
    st.sample_begin = (int32_t)get_num(env, s, "sampleBegin", 0);
    st.sample_end = (int32_t)get_num(env, s, "sampleEnd", 0);
    st.crop_x0 = (int32_t)get_num(env, s, "cropX0", 0);
    st.crop_y0 = (int32_t)get_num(env, s, "cropY0", 0);
    st.crop_w = (int32_t)get_num(env, s, "cropW", 0);
    st.crop_h = (int32_t)get_num(env, s, "cropH", 0);
    st.precision = (int32_t)get_num(env, s, "precision", RT_PREC_F64);
    st.batch_samples = (int32_t)get_num(env, s, "batchSamples", 0);
    st.denoise = (int32_t)get_num(env, s, "denoise", 0);
    st.accel = (int32_t)get_num(env, s, "accel", RT_ACCEL_AUTO);
    st.denoise_weights[0] = get_num(env, s, "denoiseW1", 0.0);
    st.denoise_weights[1] = get_num(env, s, "denoiseW2", 0.0);
    // settings.devices: [ordinals] -> rt_settings.device_count / devices (multi-GPU sample split)
    const int nd = get_int_array(env, s, "devices", st.devices, RT_MAX_DEVICES);
    if (nd < 0) {
        delete job;
        return throw_err(env, "render: settings.devices must be an Array of at most 8 device ordinals");
    }
    st.device_count = nd;
    job->want_mean = get_num(env, s, "wantMean", 0) != 0;
    job->want_counts = get_num(env, s, "wantCounts", 0) != 0;
    job->want_post = get_num(env, s, "wantPost", 1) != 0;      // the post-gamma Float32 frame (default on)
    const int cw = st.crop_w > 0 ? st.crop_w : st.width, ch = st.crop_h > 0 ? st.crop_h : st.height;
    if (cw <= 0 || ch <= 0) {
        delete job;
        return throw_err(env, "render: width/height must be positive");
    }
    job->n = (size_t)cw * ch;
    void* rs = nullptr;
    size_t rs_bytes = 0;
    if (get_bytes(env, s, "resumeSums", &rs, &rs_bytes)) {        // continue from checkpoint(scene)
        if (rs_bytes != job->n * 3 * sizeof(double)) {
            delete job;
            return throw_err(env, "render: resumeSums must hold 3 float64 per pixel of the frame");
        }
        job->resume.assign(static_cast<double*>(rs), static_cast<double*>(rs) + job->n * 3);
        job->resume_done = (int32_t)get_num(env, s, "resumeSamplesDone", 0);
    } else if (get_num(env, s, "resumeResident", 0) != 0) {      // continue from the checkpoint on the device
        job->resume_resident = true;
        job->resume_done = (int32_t)get_num(env, s, "resumeSamplesDone", 0);
    }
    st.sum_order = (int32_t)get_num(env, s, "sumOrder", RT_SUM_POOL);
    // output buffers (see RenderJob): post unless settings.wantPost is 0; the RGBA8 frame also goes into
    // settings.outRgba8 when that is the frame's size; settings.preview: running frames into it too
    bool ok = !job->want_post || make_out(env, job, RenderJob::OUT_POST, job->n * 4 * sizeof(float));
    void* rgba_p = nullptr;
    size_t rgba_bytes = 0;
    napi_value rgba_v;
    if (ok && get_bytes(env, s, "outRgba8", &rgba_p, &rgba_bytes) && rgba_bytes == job->n * 4 &&
        get_prop(env, s, "outRgba8", &rgba_v)) {
        ok = napi_create_reference(env, rgba_v, 1, &job->caller_rgba) == napi_ok;
        if (box->frame.size() != job->n * 4) box->frame.resize(job->n * 4);
        job->frame = box->frame.data();
        if (ok && get_num(env, s, "preview", 0) != 0) {
            if (box->preview.size() != job->n * 4) box->preview.resize(job->n * 4);
            job->preview = box->preview.data();
        }
    } else if (ok) {
        ok = make_out(env, job, RenderJob::OUT_RGBA, job->n * 4);
    }
    if (ok && job->want_mean) ok = make_out(env, job, RenderJob::OUT_MEAN, job->n * 3 * sizeof(double));
    if (ok && job->want_counts) ok = make_out(env, job, RenderJob::OUT_SEGS, job->n * sizeof(uint32_t)) &&
                                     make_out(env, job, RenderJob::OUT_DRAWS, job->n * sizeof(uint32_t));
    if (!ok) {
        for (napi_ref r : job->out_ref)
            if (r) napi_delete_reference(env, r);
        if (job->caller_rgba) napi_delete_reference(env, job->caller_rgba);
        delete job;
        return throw_err(env, "render: cannot allocate the output buffers");
    }
    box->last_pixels = job->n;
    napi_value promise, name;
    NAPI_OK(napi_create_promise(env, &job->deferred, &promise));
    NAPI_OK(napi_create_reference(env, argv[0], 1, &job->scene_ref));
    NAPI_OK(napi_create_string_utf8(env, "rt_render", NAPI_AUTO_LENGTH, &name));
    if (argc > 2) {
        napi_valuetype t;
        napi_typeof(env, argv[2], &t);
        if (t == napi_function)
            NAPI_OK(napi_create_threadsafe_function(env, argv[2], nullptr, name, 0, 1, nullptr, nullptr, nullptr,
                                                    call_progress, &job->tsfn));
    }
    NAPI_OK(napi_create_async_work(env, nullptr, name, execute, complete, job, &job->work));
    NAPI_OK(napi_queue_async_work(env, job->work));
    box->busy = true;
    return promise;
}

napi_value cancel(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox* box = argc ? get_box(env, argv[0]) : nullptr;
    if (!box) return throw_err(env, "cancel(scene)");
    if (box->sc) rt_cancel(box->sc);
    return nullptr;
}

// checkpoint(scene) -> {sums: Float64Array(3 per pixel), samplesDone}: the progressive state after a
// finished or cancelled render (rt_render_checkpoint); render(scene, {..., resumeSums, resumeSamplesDone})
// continues from it
napi_value checkpoint(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox* box = argc ? get_box(env, argv[0]) : nullptr;
    if (!box || !box->sc) return throw_err(env, "checkpoint(scene)");
    if (box->busy) return throw_err(env, "checkpoint: a render is in flight");
    // the sums go straight from the device into the ArrayBuffer handed to JS (no staging vector: a
    // cancelled config-3 render's 50 MB checkpoint is part of the cancel's return time)
    const size_t count = box->last_pixels * 3;
    napi_value ab, arr;
    void* p = nullptr;
    NAPI_OK(napi_create_arraybuffer(env, count * sizeof(double), &p, &ab));
    int32_t done = 0;
    if (rt_render_checkpoint(box->sc, static_cast<double*>(p), count, &done) != RT_OK) return throw_err(env, rt_last_error());
    NAPI_OK(napi_create_typedarray(env, napi_float64_array, count, ab, 0, &arr));
    napi_value res, d;
    NAPI_OK(napi_create_object(env, &res));
    NAPI_OK(napi_set_named_property(env, res, "sums", arr));
    NAPI_OK(napi_create_int32(env, done, &d));
    NAPI_OK(napi_set_named_property(env, res, "samplesDone", d));
    return res;
}

// checkpointSamples(scene) -> samplesDone of the scene's checkpoint, without copying its sums (they stay
// on the device until the scene's next render: render(scene, {..., resumeResident: 1, resumeSamplesDone})
// continues from them, checkpoint(scene) copies them out)
napi_value checkpoint_samples(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox* box = argc ? get_box(env, argv[0]) : nullptr;
    if (!box || !box->sc) return throw_err(env, "checkpointSamples(scene)");
    if (box->busy) return throw_err(env, "checkpointSamples: a render is in flight");
    int32_t done = 0;
    if (rt_render_checkpoint(box->sc, nullptr, 0, &done) != RT_OK) return throw_err(env, rt_last_error());
    napi_value d;
    NAPI_OK(napi_create_int32(env, done, &d));
    return d;
}

napi_value destroy_scene(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    SceneBox* box = argc ? get_box(env, argv[0]) : nullptr;
    if (!box) return throw_err(env, "destroyScene(scene)");
    if (box->busy) return throw_err(env, "destroyScene: a render is in flight");
    if (box->sc) rt_scene_destroy(box->sc);
    box->sc = nullptr;
    return nullptr;
}

napi_value device_count(napi_env env, napi_callback_info) {
    int n = 0;
    rt_device_count(&n);
    napi_value v;
    napi_create_int32(env, n, &v);
    return v;
}

napi_value abi_version(napi_env env, napi_callback_info) {
    napi_value v;
    napi_create_int32(env, rt_abi_version(), &v);
    return v;
}

napi_value init(napi_env env, napi_value exports) {
    const napi_property_descriptor props[] = {
        {"createScene", nullptr, create_scene, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"render", nullptr, render, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"cancel", nullptr, cancel, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"checkpoint", nullptr, checkpoint, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"checkpointSamples", nullptr, checkpoint_samples, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"destroyScene", nullptr, destroy_scene, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"deviceCount", nullptr, device_count, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"abiVersion", nullptr, abi_version, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
    };
    napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
