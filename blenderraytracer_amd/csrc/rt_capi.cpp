// rt_capi.cpp — extern "C" ABI of librt_hip.so (include/rt_hip.h).
//
// Replaces RayTracer.render (js/ray-tracer.js:166-281): the host hands over the packed World /
// Camera once (rt_scene_create uploads it to HBM), then each render traces sample batches on the
// GPU, runs the epilogue on the GPU and copies back only the per-pixel outputs.
// There is no CPU fallback anywhere in this library: without a HIP device every call fails with
// RT_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_hip.h"
#include "pt_launch.h"
#include "pool_order.h"
#include "scene_pack.h"

using namespace rt;

namespace {

thread_local std::string g_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_error = buf;
    return code;
}

}  // namespace

namespace rt {
int set_error(int code, const char* msg) {   // for the other translation units (scene_json.cpp)
    g_error = msg;
    return code;
}
}  // namespace rt

namespace {

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(RT_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = std::max<size_t>(count, 1);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

template <class T>
hipError_t upload(DevBuf<T>& b, const std::vector<T>& v) {
    hipError_t e = b.ensure(v.size());
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

// Scene arrays of one precision, resident in HBM.
template <class R>
struct DeviceScene {
    DevBuf<Run> runs;
    DevBuf<SphereRec<R>> spheres;
    DevBuf<SphereFilter> sphere_filter;
    DevBuf<R> sphere_r, sphere_inv_r;
    DevBuf<PlaneRec<R>> planes;
    DevBuf<BoxRec<R>> boxes;
    DevBuf<TriRec<R>> tris;
    DevBuf<int> sphere_mat, plane_mat, box_mat, tri_mat, perm;
    DevBuf<MatRec<R>> mats;
    DevBuf<int> plane_obj, box_obj;
    DevBuf<BvhNode> sphere_nodes, tri_nodes;
    DevBuf<SphereLeaf<R>> bvh_sphere_leaf;
    DevBuf<TriLeaf<R>> bvh_tri_leaf;
    DevBuf<TriFilter> tri_filter;
    DevBuf<double> tri_exit;
    DevBuf<SphereLeaf<R>> big_sphere_leaf;
    DevBuf<Bvh2Node> sphere_wide, tri_wide;
    DevBuf<int> grid_cell;
    DevBuf<SphereLeaf<R>> grid_leaf;
    SceneView<R> view{};
    void release() {
        runs.release(); spheres.release(); sphere_filter.release(); sphere_r.release(); sphere_inv_r.release(); planes.release(); boxes.release(); tris.release();
        sphere_mat.release(); plane_mat.release(); box_mat.release(); tri_mat.release(); perm.release(); mats.release();
        plane_obj.release(); box_obj.release(); sphere_nodes.release(); tri_nodes.release(); bvh_sphere_leaf.release();
        bvh_tri_leaf.release(); tri_filter.release(); tri_exit.release(); big_sphere_leaf.release();
        sphere_wide.release(); tri_wide.release(); grid_cell.release(); grid_leaf.release();
    }
};

template <class R>
int build_device(DeviceScene<R>& ds, const HostScene& hs, const rt_scene_desc& d) {
    HostRecords<R> rec;
    make_records(hs, d, rec);
    hipError_t e = hipSuccess;
#define UP(buf, vec) if (e == hipSuccess) e = upload(ds.buf, vec)
    UP(runs, hs.runs); UP(spheres, rec.spheres); UP(sphere_filter, rec.sphere_filter); UP(sphere_r, rec.sphere_r); UP(sphere_inv_r, rec.sphere_inv_r); UP(planes, rec.planes);
    UP(boxes, rec.boxes); UP(tris, rec.tris); UP(sphere_mat, hs.sphere_mat); UP(plane_mat, hs.plane_mat);
    UP(box_mat, hs.box_mat); UP(tri_mat, hs.tri_mat); UP(perm, rec.perm); UP(mats, rec.mats);
    UP(plane_obj, hs.plane_obj); UP(box_obj, hs.box_obj); UP(sphere_nodes, hs.sphere_bvh); UP(tri_nodes, hs.tri_bvh);
    UP(bvh_sphere_leaf, rec.bvh_sphere_leaf); UP(bvh_tri_leaf, rec.bvh_tri_leaf); UP(tri_filter, rec.tri_filter); UP(big_sphere_leaf, rec.big_sphere_leaf); UP(sphere_wide, hs.sphere_wide); UP(tri_wide, hs.tri_wide);
    UP(grid_cell, hs.grid_cell); UP(grid_leaf, rec.grid_leaf); UP(tri_exit, hs.tri_exit);
#undef UP
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, "scene upload: %s", hipGetErrorString(e));
    SceneView<R>& v = ds.view;
    v.runs = ds.runs.p;
    v.spheres = ds.spheres.p; v.sphere_filter = ds.sphere_filter.p; v.sphere_r = ds.sphere_r.p; v.sphere_inv_r = ds.sphere_inv_r.p; v.planes = ds.planes.p; v.boxes = ds.boxes.p;
    v.tris = ds.tris.p; v.sphere_mat = ds.sphere_mat.p; v.plane_mat = ds.plane_mat.p; v.box_mat = ds.box_mat.p;
    v.tri_mat = ds.tri_mat.p; v.mats = ds.mats.p; v.perm = ds.perm.p;
    v.plane_obj = ds.plane_obj.p; v.box_obj = ds.box_obj.p; v.sphere_nodes = ds.sphere_nodes.p; v.tri_nodes = ds.tri_nodes.p;
    v.bvh_sphere_leaf = ds.bvh_sphere_leaf.p; v.bvh_tri_leaf = ds.bvh_tri_leaf.p; v.tri_filter = ds.tri_filter.p;
    v.tri_exit = ds.tri_exit.p;
    v.big_spheres = ds.big_sphere_leaf.p;
    v.sphere_wide = ds.sphere_wide.p; v.tri_wide = ds.tri_wide.p;
    v.grid_cell = ds.grid_cell.p; v.grid_leaf = ds.grid_leaf.p;
    fill_view_constants(v, hs, d);
    return RT_OK;
}

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Batches in flight per render (render_impl): kSlots partial slots / trace streams per device; the host
// queues up to kSlots batches per device beyond the one it waits for (lookahead()), each with its own
// preview staging and completion event (lookahead() + kSlots of them, so a queued batch never writes a
// frame the host has not read yet).
constexpr int kSlots = 3;
inline int lookahead(int devices) { return kSlots * std::max(1, devices); }

// The render's control words (rt_scene::ctl, mapped coherent host memory, read and written by the host
// and by the kernels of every device): the cancel word, the sticky stop word and the samples the sums
// hold (ReduceGate), and one `aborted` word per batch slot of the ring.
// kCtlCancel: kCancelCopies copies of the cancel word, one per 128-B line (pt_launch.h).
constexpr int kCtlStop = 1, kCtlDone = 2, kCtlAborted = 4;
constexpr int kCtlCancel = 128;
// fused batches (render_impl): per batch, the flag its last item raises; two `aborted` words (the gates'
// stand-in, never written; the skipping waves', never read)
constexpr int kMaxFused = 64;
constexpr int kCtlFlag = kCtlCancel + kCancelCopies * kCancelStride;
constexpr int kCtlFusedAborted = kCtlFlag + kMaxFused;
constexpr int kCtlWords = kCtlFusedAborted + 2;
static_assert(kCtlAborted + kSlots * RT_MAX_DEVICES + kSlots <= kCtlCancel, "one aborted word per ring slot");
inline uint32_t ctl_load(const uint32_t* ctl, int k) { return __atomic_load_n(ctl + k, __ATOMIC_SEQ_CST); }
inline void ctl_store(uint32_t* ctl, int k, uint32_t v) { __atomic_store_n(ctl + k, v, __ATOMIC_SEQ_CST); }
inline void ctl_cancel(uint32_t* ctl, uint32_t v) {
    for (int k = 0; k < kCancelCopies; ++k) ctl_store(ctl, kCtlCancel + k * kCancelStride, v);
}

// Everything one device holds for a scene: the scene arrays in its HBM, a stream, the running sums
// and counters of the samples it traces, the pool's chunk partials and the work totals (scratch).
struct DeviceState {
    int device = 0;
    DeviceScene<double> s64;
    DeviceScene<float> s32;
    hipStream_t stream = nullptr;      // accumulation stream: zeroing, reduces, merges, epilogue
    hipEvent_t ev[2] = {};             // trace timing
    DevBuf<double> sum;
    DevBuf<uint32_t> segs, draws;
    DevBuf<unsigned long long> total;
    DevBuf<double> part;               // sample-pool chunk partials (ensure_partials; overlapped batches: slot 0)
    DevBuf<uint32_t> gate_skip;        // ReduceGate::skip of the reduces on this device's stream
    hipEvent_t scratch_ev = nullptr;   // recorded after every use of part / total (order_scratch)
    hipStream_t scratch_stream = nullptr;
    bool scratch_used = false;
    hipEvent_t copy_ev = nullptr;      // a replica's batch sums copied out to the home device (merge_shards)
    // overlapped batches (render_impl): batch k traces on tstream[k % kSlots] into its own partials
    // (slot 0: `part`), so the next batches' waves fill the CUs while this one drains; its reduce runs on
    // `stream` in batch order
    hipStream_t tstream[kSlots] = {};
    DevBuf<double> part_more[kSlots - 1];   // partials of slots 1 ..
    hipEvent_t traced[kSlots] = {}, reduced[kSlots] = {}, setup_ev = nullptr;
    DevBuf<double>& slot_part(int j) { return j == 0 ? part : part_more[j - 1]; }
    // fused batches (render_impl): every batch's chunk partials, the items done per batch, and the
    // event recorded after the one launch on tstream[0]
    DevBuf<double> fused_part;
    DevBuf<uint32_t> fused_count;
    hipEvent_t fused_done = nullptr;
    // the one-wave pool kernel's cancel word in device memory (Counters::cancel_dev), zeroed once; each
    // render matches its own generation
    DevBuf<uint32_t> cancel_word;

    int init(int dev, const HostScene& hs, const rt_scene_desc& d) {
        device = dev;
        hipError_t e = hipSetDevice(dev);
        if (e != hipSuccess) return fail(RT_ERR_DEVICE, "hipSetDevice(%d): %s", dev, hipGetErrorString(e));
        int rc;
        if ((rc = build_device(s64, hs, d)) || (rc = build_device(s32, hs, d))) return rc;
        // the accumulation stream at the device's highest priority: a batch's reduce (and preview frame)
        // would otherwise wait for free wave slots behind the next batch's trace waves — measured: a
        // 0.1-ms reduce took 7.8 ms, and the batch after next started late
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, greatest);
        for (int k = 0; k < kSlots && e == hipSuccess; ++k) e = hipStreamCreateWithFlags(&tstream[k], hipStreamNonBlocking);
        for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipEventCreate(&ev[k]);
        for (int k = 0; k < kSlots && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&traced[k], hipEventDisableTiming);
        for (int k = 0; k < kSlots && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&reduced[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&setup_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&fused_done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&scratch_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&copy_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = cancel_word.ensure((size_t)kDevCancelCopies * kCancelStride);
        if (e == hipSuccess) e = hipMemset(cancel_word.p, 0, (size_t)kDevCancelCopies * kCancelStride * sizeof(uint32_t));
        if (e != hipSuccess) return fail(RT_ERR_DEVICE, "stream/event create: %s", hipGetErrorString(e));
        return RT_OK;
    }
    void sync_all() {                  // every stream of this device (error paths, release)
        (void)hipSetDevice(device);
        for (hipStream_t s : tstream)
            if (s) (void)hipStreamSynchronize(s);
        if (stream) (void)hipStreamSynchronize(stream);
    }
    void release() {
        sync_all();
        s64.release();
        s32.release();
        sum.release(); segs.release(); draws.release(); total.release(); part.release(); gate_skip.release();
        fused_part.release(); fused_count.release(); cancel_word.release();
        for (DevBuf<double>& b : part_more) b.release();
        for (hipEvent_t e : {ev[0], ev[1], setup_ev, scratch_ev, copy_ev, fused_done})
            if (e) (void)hipEventDestroy(e);
        for (int k = 0; k < kSlots; ++k) {
            if (traced[k]) (void)hipEventDestroy(traced[k]);
            if (reduced[k]) (void)hipEventDestroy(reduced[k]);
            if (tstream[k]) (void)hipStreamDestroy(tstream[k]);
        }
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// A deep copy of the scene descriptor, so replicas can be uploaded to more devices later.
struct DescCopy {
    rt_scene_desc d{};
    std::vector<rt_object_desc> objects;
    std::vector<rt_material_desc> materials;
    std::vector<double> triangles;
    void set(const rt_scene_desc& src) {
        d = src;
        objects.assign(src.objects, src.objects + std::max(0, src.num_objects));
        materials.assign(src.materials, src.materials + std::max(0, src.num_materials));
        triangles.assign(src.triangles, src.triangles + 12 * (size_t)std::max(0, src.num_triangles));
        d.objects = objects.data();
        d.materials = materials.data();
        d.triangles = triangles.data();
    }
};

}  // namespace

// The RGBA8 threshold table of one gamma (launch_gamma_thresholds) on the scene's device.  A table is
// built once and then only read: an asynchronous epilogue on any stream reads its own gamma's table, so
// a later call with another gamma can never overwrite the bytes an earlier one is still reading (ADVICE
// r5).  `used` is recorded after every kernel that reads the table; a slot is rebuilt for another gamma
// (the least recently used one, when kGammaSlots gammas are in use) only after it has completed.
struct GammaSlot {
    DevBuf<unsigned char> buf;
    double gamma = NAN;
    bool ok = false;                 // no exception overflow: the table may be used
    hipEvent_t used = nullptr;
    bool used_recorded = false;
    uint64_t tick = 0;               // last use (LRU)
    const GammaTable* table() const { return reinterpret_cast<const GammaTable*>(buf.p); }
    void release() {
        buf.release();
        if (used) (void)hipEventDestroy(used);
        used = nullptr;
    }
};
constexpr int kGammaSlots = 8;

// What a resident checkpoint's sums are sums of: a resume from the sums left on the device
// (rt_render_resume with sums NULL) must name the same frame, crop window, first sample, precision, seed,
// anti-aliasing mode and depth, not only the same pixel count.
struct CkptKey {
    int32_t width, height, x0, y0, cw, ch, sample_begin, precision, aa_mode, max_depth;
    uint64_t seed;
    bool operator==(const CkptKey& o) const {
        return width == o.width && height == o.height && x0 == o.x0 && y0 == o.y0 && cw == o.cw && ch == o.ch &&
               sample_begin == o.sample_begin && precision == o.precision && aa_mode == o.aa_mode &&
               max_depth == o.max_depth && seed == o.seed;
    }
};
inline CkptKey ckpt_key(const rt_settings* s, int cw, int ch) {
    return CkptKey{s->width, s->height, s->crop_x0, s->crop_y0, cw, ch, std::max(0, s->sample_begin), s->precision,
                   s->aa_mode, s->max_depth, (uint64_t)s->seed};
}

// A shard's staging buffers on the home device and the events that free them (merge_shards,
// trace_replica).
struct MergeSlot {
    DevBuf<double> sum;
    DevBuf<uint32_t> segs, draws;
    hipEvent_t added = nullptr;     // recorded on the home stream after this slot's adds
    bool pending = false;           // `added` has been recorded
    // whole-batch split (trace_replica): the chunk partials of the replica's batch in its partial slot j
    // land in stage[j] on the home device, reduced there in batch order; stage_free[j] is recorded on the
    // home stream after that reduce
    DevBuf<double> stage[kSlots];
    hipEvent_t stage_free[kSlots] = {};
    bool stage_used[kSlots] = {};
    void release() {
        sum.release(); segs.release(); draws.release();
        for (DevBuf<double>& b : stage) b.release();
        if (added) (void)hipEventDestroy(added);
        for (hipEvent_t e : stage_free)
            if (e) (void)hipEventDestroy(e);
    }
};

struct rt_scene {
    DeviceState home;               // the device of rt_scene_create: epilogue, outputs, checkpoint
    std::vector<DeviceState*> replicas;   // rt_settings.devices[k] for k >= 1 (created on first use)
    HostScene hs;
    DescCopy desc;
    int num_prims = 0;
    int bvh_prims = 0;              // spheres + triangles (the primitives the BVHs cover)
    bool bvh_ok = true;             // both trees fit the traversal stack (depth <= RT_BVH_STACK)
    bool tri_bvh = false;           // the scene has a triangle BVH (pool chunk choice)
    double record_bytes = 0;
    hipEvent_t ev[2] = {};          // epilogue timing
    DevBuf<double> mean;
    std::vector<MergeSlot> merge;   // per shard (index in the render's device list): its staging on home
    DevBuf<float> post, post_raw;   // post_raw: pre-denoise floatData
    DevBuf<uint8_t> rgba;
    // rt_output.preview_rgba8: the running frame of each batch in flight, in mapped pinned host memory
    std::vector<uint8_t*> preview_host;
    std::vector<uint8_t*> preview_dev;    // the same buffers' device addresses
    size_t preview_host_n = 0;
    std::vector<hipEvent_t> batch_done;   // home stream: batch k's reduce, merges and preview done (slot k % ring)
    // preview frames / RGBA8-only epilogues: the gamma tables (launch_gamma_thresholds), one per gamma,
    // never rebuilt while a kernel may read them (gamma_table)
    std::vector<GammaSlot> gamma_slots;
    uint64_t gamma_tick = 0;
    std::atomic<int> cancel{0};
    uint32_t render_gen = 0;        // generation of the current render (device cancel words)
    uint32_t* ctl = nullptr;        // the render's control words (kCtl*), host address
    uint32_t* ctl_dev = nullptr;    // ... their device address (portable mapping: valid on every device)
    size_t ckpt_pixels = 0;         // progressive state of the last rt_render / rt_render_resume:
    int ckpt_done = 0;              // `home.sum` holds samples [sample_begin, ckpt_done) of ckpt_pixels pixels
    CkptKey ckpt_key{};             // ... of this frame, crop, first sample, precision and seed
};

namespace {

int check_settings(const rt_settings* s, int* cw, int* ch) {
    if (!s) return fail(RT_ERR_INVALID, "settings is NULL");
    if (s->width <= 0 || s->height <= 0) return fail(RT_ERR_INVALID, "image %dx%d", s->width, s->height);
    if ((long long)s->width * s->height > 0xFFFFFFFFLL) return fail(RT_ERR_INVALID, "image too large for 32-bit pixel keys");
    *cw = s->crop_w > 0 ? s->crop_w : s->width;
    *ch = s->crop_h > 0 ? s->crop_h : s->height;
    if (s->crop_x0 < 0 || s->crop_y0 < 0 || s->crop_x0 + *cw > s->width || s->crop_y0 + *ch > s->height)
        return fail(RT_ERR_INVALID, "crop [%d,%d %dx%d] outside %dx%d", s->crop_x0, s->crop_y0, *cw, *ch, s->width,
                    s->height);
    if (s->samples < 0) return fail(RT_ERR_INVALID, "samples %d", s->samples);
    if (s->precision != RT_PREC_F64 && s->precision != RT_PREC_F32) return fail(RT_ERR_INVALID, "precision %d", s->precision);
    if (s->aa_mode < 0 || s->aa_mode > 2) return fail(RT_ERR_INVALID, "aa_mode %d", s->aa_mode);
    if (s->accel < RT_ACCEL_AUTO || s->accel > RT_ACCEL_BVH) return fail(RT_ERR_INVALID, "accel %d", s->accel);
    if (s->denoise && (*cw != s->width || *ch != s->height))
        return fail(RT_ERR_INVALID, "denoise needs the full frame (PostProcessor.denoise clamps to the image edge)");
    if (s->device_count < 0 || s->device_count > RT_MAX_DEVICES)
        return fail(RT_ERR_INVALID, "device_count %d (at most %d)", s->device_count, RT_MAX_DEVICES);
    if (s->device_count > 1) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
        for (int k = 0; k < s->device_count; ++k)
            if (s->devices[k] < 0 || s->devices[k] >= ndev) return fail(RT_ERR_INVALID, "devices[%d] = %d of %d", k, s->devices[k], ndev);
    }
    return RT_OK;
}

// The gamma table of `gamma` on the scene's device (current), or nullptr when previews must take
// finalize_kernel.  A new gamma's table is built on the scene's own stream (`home.stream`, waited for:
// its exception count is read back) into a slot no kernel is reading: a free one, else the least
// recently used slot once its last reader has completed.  The caller's stream is never synchronized.
GammaSlot* gamma_table(rt_scene* sc, double gamma) {
    if (!preview_thresholds_ok(gamma)) return nullptr;
    GammaSlot* g = nullptr;
    for (GammaSlot& x : sc->gamma_slots)
        if (x.gamma == gamma) g = &x;
    if (!g) {
        sc->gamma_slots.reserve(kGammaSlots);      // never reallocated: a render keeps its slot's address
        if ((int)sc->gamma_slots.size() < kGammaSlots) {
            sc->gamma_slots.emplace_back();
            g = &sc->gamma_slots.back();
        } else {
            g = &sc->gamma_slots[0];
            for (GammaSlot& x : sc->gamma_slots)
                if (x.tick < g->tick) g = &x;
        }
        hipError_t e = g->used_recorded ? hipEventSynchronize(g->used) : hipSuccess;
        g->gamma = NAN;
        g->used_recorded = false;
        uint32_t words[2] = {0, 1};
        hipStream_t st = sc->home.stream;
        if (e == hipSuccess && !g->used) e = hipEventCreateWithFlags(&g->used, hipEventDisableTiming);
        if (e == hipSuccess) e = g->buf.ensure(sizeof(GammaTable));
        GammaTable* t = reinterpret_cast<GammaTable*>(g->buf.p);
        if (e == hipSuccess) e = launch_gamma_thresholds(gamma, t, st);
        if (e == hipSuccess) e = hipMemcpyAsync(words, &t->n_exc, sizeof words, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        g->gamma = gamma;
        g->ok = words[1] == 0;
    }
    g->tick = ++sc->gamma_tick;
    return g->ok ? g : nullptr;
}

// after a kernel reading g's table was enqueued on `st`
hipError_t gamma_used(GammaSlot* g, hipStream_t st) {
    const hipError_t e = hipEventRecord(g->used, st);
    if (e == hipSuccess) g->used_recorded = true;
    return e;
}

// mean, toneMap, gammaCorrect (+ PostProcessor.denoise), RGBA8 on `st` (ray-tracer.js:208-276).
// thresholds: an RGBA8-only epilogue through the gamma table (preview_kernel: the same bytes, 29 VGPRs
// instead of finalize_kernel's 80)
hipError_t epilogue(rt_scene* sc, const rt_settings* s, int cw, int ch, const double* sum, double* mean, float* post,
                    uint8_t* rgba, hipStream_t st, bool thresholds = false) {
    FinalizeParams fp{cw * ch, s->samples, s->tone_map, s->exposure, s->gamma};
    if (thresholds && !s->denoise && !mean && !post && rgba)
        if (GammaSlot* g = gamma_table(sc, s->gamma)) {
            const hipError_t e = launch_finalize(fp, sum, nullptr, nullptr, rgba, st, g->table());
            return e == hipSuccess ? gamma_used(g, st) : e;
        }
    if (!s->denoise) return launch_finalize(fp, sum, mean, post, rgba, st);
    hipError_t e = sc->post_raw.ensure(4 * (size_t)cw * ch);
    if (e == hipSuccess) e = launch_finalize(fp, sum, mean, sc->post_raw.p, nullptr, st);
    if (e == hipSuccess) e = launch_denoise(cw, ch, s->denoise_weights[0], s->denoise_weights[1], sc->post_raw.p, post, rgba, st);
    return e;
}

ImageParams image_params(const rt_settings* s, int cw, int ch) {
    ImageParams im{};
    im.width = s->width; im.height = s->height;
    im.x0 = s->crop_x0; im.y0 = s->crop_y0; im.cw = cw; im.ch = ch;
    im.samples = s->samples;
    im.s_begin = std::max(0, s->sample_begin);
    im.s_end = s->sample_end > 0 ? std::min(s->sample_end, s->samples) : s->samples;
    im.max_depth = s->max_depth;
    im.aa_mode = s->aa_mode;
    im.seedm = host_seed_mix(s->seed);
    return im;
}

// RT_ACCEL_AUTO: the BVH unless the scene has almost no spheres/triangles (measured faster from 10
// primitives (Cornell) to 50k (mesh50k), DESIGN.md "BVH")
constexpr int kAutoBvhPrims = 8;

bool use_bvh(const rt_scene* sc, const rt_settings* s) {
    if (!sc->bvh_ok) return false;
    return s->accel == RT_ACCEL_BVH || (s->accel == RT_ACCEL_AUTO && sc->bvh_prims >= kAutoBvhPrims);
}

int check_accel(const rt_scene* sc, const rt_settings* s) {
    if (s->accel == RT_ACCEL_BVH && !sc->bvh_ok)
        return fail(RT_ERR_INVALID, "BVH deeper than the %d-entry traversal stack (too many primitives): use "
                    "RT_ACCEL_AUTO or RT_ACCEL_BRUTE", RT_BVH_STACK);
    return RT_OK;
}

// rt_settings.sum_order: the sample pool unless the caller asks for sample order (or RT_SAMPLE_POOL=0)
bool use_pool(const rt_settings* s) { return s->sum_order == RT_SUM_POOL && trace_uses_pool(); }

hipError_t trace(const rt_scene* sc, const DeviceState& ds, const rt_settings* s, const ImageParams& im,
                 const Counters& c, hipStream_t st) {
    if (im.max_depth <= 0) return hipSuccess;   // rayColor(ray, depth<=0) is 0: nothing to trace
    const bool bvh = use_bvh(sc, s), pool = use_pool(s);
    if (s->precision == RT_PREC_F32) return launch_trace<float>(ds.s32.view, im, c, bvh, pool, st);
    return launch_trace<double>(ds.s64.view, im, c, bvh, pool, st);
}

// One overlapped batch on one device: the pool kernel writes the batch's chunk partials into slot `j`
// on tstream[j] (after the reduce that last read slot j), and `stream` adds them to the sums in chunk
// order once the trace is done.  Sums see the same additions in the same order as trace() of the batch
// (bit-identical), while the trace of batch k+1 may already run beside batch k's draining waves.
hipError_t trace_overlapped(const rt_scene* sc, DeviceState& ds, const rt_settings* s, const ImageParams& im,
                            const Counters& c, int j, bool slot_used, const ReduceGate* gate) {
    if (im.max_depth <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    const bool bvh = use_bvh(sc, s);
    DevBuf<double>& part = ds.slot_part(j);
    hipStream_t ts = ds.tstream[j];
    hipError_t e = hipSuccess;
    if (slot_used) e = hipStreamWaitEvent(ts, ds.reduced[j], 0);
    if (e == hipSuccess)
        e = s->precision == RT_PREC_F32
                ? launch_trace_partials<float>(ds.s32.view, im, c, bvh, part.p, part.n * sizeof(double), ts)
                : launch_trace_partials<double>(ds.s64.view, im, c, bvh, part.p, part.n * sizeof(double), ts);
    if (e == hipSuccess) e = hipEventRecord(ds.traced[j], ts);
    if (e == hipSuccess) e = hipStreamWaitEvent(ds.stream, ds.traced[j], 0);
    if (e == hipSuccess) e = launch_reduce(im, c.sum, part.p, sc->tri_bvh, ds.stream, gate);
    if (e == hipSuccess) e = hipEventRecord(ds.reduced[j], ds.stream);
    return e;
}

// One whole batch on a replica (the whole-batch split of render_impl): the pool kernel writes the
// batch's chunk partials into the replica's slot j on its tstream[j]; the same stream then copies them
// into the home device's staging slot j (once the home stream's last reduce of that slot is done), and
// the home stream adds them to the home sums in chunk order after the copy — exactly the reduce that
// trace_overlapped runs for a batch traced on the home device, in the same (batch) order, so the sums
// are bit-identical to the same batches on one device.  The replica's next trace into slot j follows
// the copy on the same stream.
int trace_replica(rt_scene* sc, DeviceState& ds, MergeSlot& m, const rt_settings* s, const ImageParams& im,
                  const Counters& c, int j, const ReduceGate* gate) {
    if (im.max_depth <= 0 || im.s_end <= im.s_begin) return RT_OK;
    DeviceState& h = sc->home;
    const int cw = im.cw, ch = im.ch;
    const size_t bytes = pool_plan(cw, ch, im.s_end - im.s_begin, sc->tri_bvh, im.pool_chunk).part_bytes;
    const bool bvh = use_bvh(sc, s);
    DevBuf<double>& part = ds.slot_part(j);
    hipStream_t ts = ds.tstream[j];
    HIP_TRY(hipSetDevice(h.device));
    HIP_TRY(m.stage[j].ensure(bytes / sizeof(double)));
    if (!m.stage_free[j]) HIP_TRY(hipEventCreateWithFlags(&m.stage_free[j], hipEventDisableTiming));
    HIP_TRY(hipSetDevice(ds.device));
    HIP_TRY(s->precision == RT_PREC_F32
                ? launch_trace_partials<float>(ds.s32.view, im, c, bvh, part.p, part.n * sizeof(double), ts)
                : launch_trace_partials<double>(ds.s64.view, im, c, bvh, part.p, part.n * sizeof(double), ts));
    if (m.stage_used[j]) HIP_TRY(hipStreamWaitEvent(ts, m.stage_free[j], 0));
    HIP_TRY(hipMemcpyPeerAsync(m.stage[j].p, h.device, part.p, ds.device, bytes, ts));
    HIP_TRY(hipEventRecord(ds.traced[j], ts));              // trace + copy out done
    HIP_TRY(hipSetDevice(h.device));
    HIP_TRY(hipStreamWaitEvent(h.stream, ds.traced[j], 0));
    HIP_TRY(launch_reduce(im, h.sum.p, m.stage[j].p, sc->tri_bvh, h.stream, gate));
    HIP_TRY(hipEventRecord(m.stage_free[j], h.stream));
    m.stage_used[j] = true;
    return RT_OK;
}

// The per-pixel counters (segments, draws) of the replicas of a whole-batch split, added into the home
// device's once all their batches are traced (integer sums: any order).  The replica's accumulation
// stream first waits for its trace streams.
int merge_counters(rt_scene* sc, const std::vector<DeviceState*>& states, size_t n, bool segs, bool draws) {
    DeviceState& h = sc->home;
    for (size_t k = 0; k < states.size(); ++k) {
        DeviceState* ds = states[k];
        if (ds == &h || !(segs || draws)) continue;
        MergeSlot& m = sc->merge[k];
        HIP_TRY(hipSetDevice(h.device));
        if (segs) HIP_TRY(m.segs.ensure(n));
        if (draws) HIP_TRY(m.draws.ensure(n));
        HIP_TRY(hipSetDevice(ds->device));
        if (segs) HIP_TRY(hipMemcpyPeerAsync(m.segs.p, h.device, ds->segs.p, ds->device, n * sizeof(uint32_t), ds->stream));
        if (draws) HIP_TRY(hipMemcpyPeerAsync(m.draws.p, h.device, ds->draws.p, ds->device, n * sizeof(uint32_t), ds->stream));
        HIP_TRY(hipEventRecord(ds->copy_ev, ds->stream));
        HIP_TRY(hipSetDevice(h.device));
        HIP_TRY(hipStreamWaitEvent(h.stream, ds->copy_ev, 0));
        if (segs) HIP_TRY(launch_add<uint32_t>(h.segs.p, m.segs.p, n, h.stream));
        if (draws) HIP_TRY(launch_add<uint32_t>(h.draws.p, m.draws.p, n, h.stream));
    }
    return RT_OK;
}

// Peer access between the scene's device and a replica's (hipMemcpyPeerAsync then runs over xGMI
// directly instead of a staged copy).  Without a peer path (PCIe-only topologies, device subsets across
// root complexes) the copies still work — HIP stages them through host memory — so that is not an
// error: it is reported once on stderr and the render goes on.  Only an unexpected failure of
// hipDeviceEnablePeerAccess fails the render.
int enable_peer(int a, int b) {
    if (a == b) return RT_OK;
    for (int k = 0; k < 2; ++k) {
        const int from = k ? b : a, to = k ? a : b;
        int can = 0;
        HIP_TRY(hipDeviceCanAccessPeer(&can, from, to));
        if (!can) {
            static std::atomic<bool> told{false};
            if (!told.exchange(true))
                fprintf(stderr, "[rt_hip] device %d has no peer access to device %d: the sample split's copies are "
                        "staged through host memory\n", from, to);
            continue;
        }
        HIP_TRY(hipSetDevice(from));
        const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        else if (e != hipSuccess) return fail(RT_ERR_DEVICE, "hipDeviceEnablePeerAccess(%d -> %d): %s", from, to, hipGetErrorString(e));
    }
    return RT_OK;
}

// Sample-pool chunk partials (pool_partial_bytes, pt_trace.hip): all of a launch's chunks when they fit
// the budget (RT_PART_MB, default 2 GiB, at most 10 % of the free device memory), else as many
// chunks as fit (launch_trace then splits the samples over several launches).  RTOW 1080p x 512 spp
// needs 0.3 GB; a launch with a single chunk needs none.  Kept by the device state between renders.
size_t part_budget() {
    static const size_t budget = [] {
        const char* e = getenv("RT_PART_MB");
        return (size_t)(e ? std::max(1LL, atoll(e)) : 2048LL) << 20;
    }();
    return budget;
}

// A device state's scratch may still be read by an asynchronous call on another stream (rt_trace_device):
// wait for its last user before freeing or reallocating it (hipFree's implicit device synchronization is
// not relied upon).
hipError_t scratch_idle(DeviceState& ds) {
    return ds.scratch_used ? hipEventSynchronize(ds.scratch_ev) : hipSuccess;
}

int ensure_partials(const rt_scene* sc, DeviceState& ds, int cw, int ch, int samples, bool pool, Counters& c,
                    int chunk = 0) {
    if (!pool || samples <= 0 || cw <= 0 || ch <= 0) return RT_OK;
    const size_t want_all = pool_partial_bytes(cw, ch, samples, sc->tri_bvh, chunk);
    if (want_all == 0) return RT_OK;
    const size_t per_chunk = (size_t)((cw + 7) / 8) * ((ch + 7) / 8) * kPartialBytesPerTile;
    size_t want = want_all;
    if (want > ds.part.n * sizeof(double)) {
        HIP_TRY(scratch_idle(ds));
        size_t free_b = 0, total_b = 0, cap = part_budget();
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) cap = std::min(cap, (free_b + ds.part.n * sizeof(double)) / 10);
        want = std::min(want, std::max<size_t>(cap / per_chunk, 1) * per_chunk);
        while (want > ds.part.n * sizeof(double)) {
            if (ds.part.ensure(want / sizeof(double)) == hipSuccess) break;
            (void)hipGetLastError();
            if (want == per_chunk) return fail(RT_ERR_DEVICE, "sample pool: cannot allocate %zu bytes", per_chunk);
            want = std::max<size_t>(want / per_chunk / 2, 1) * per_chunk;
        }
    }
    c.part = ds.part.p;
    c.part_bytes = ds.part.n * sizeof(double);
    return RT_OK;
}

// Both partial slots of the overlapped batches, `bytes` each (one batch's chunks: pool_plan).  False
// (no error) when they do not fit the budget: the render then runs its batches one after the other.
bool ensure_overlap_partials(DeviceState& ds, size_t bytes) {
    bool have = true;
    size_t held = 0;
    for (int j = 0; j < kSlots; ++j) {
        have = have && ds.slot_part(j).p && ds.slot_part(j).n * sizeof(double) >= bytes;
        held += ds.slot_part(j).n * sizeof(double);
    }
    if (bytes == 0 || have) return true;
    if (scratch_idle(ds) != hipSuccess) return false;
    size_t free_b = 0, total_b = 0, cap = part_budget();
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) cap = std::min(cap, (free_b + held) / 10);
    if (kSlots * bytes > cap) return false;
    for (int j = 0; j < kSlots; ++j)
        if (ds.slot_part(j).ensure(bytes / sizeof(double)) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
    return true;
}

// Fused batches: the chunk partials of all `nb` batches of a render (`doubles` each) and their item
// counters.  The partials budget is RT_FUSED_MB (default 8 GiB, at most 10 % of the free device
// memory; config 3 in 16 batches needs 0.8 GB); false (no error) when they do not fit: the render then
// launches its batches one by one.
bool ensure_fused(DeviceState& ds, size_t doubles, int nb) {
    const size_t bytes = doubles * (size_t)nb * sizeof(double);
    if (bytes == 0) return false;
    if (ds.fused_part.n * sizeof(double) < bytes) {
        static const size_t budget = [] {   // thread-safe initialization (concurrent renders of other scenes)
            const char* e = getenv("RT_FUSED_MB");
            return (size_t)(e ? std::max(0LL, atoll(e)) : 8192LL) << 20;
        }();
        size_t free_b = 0, total_b = 0, cap = budget;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) cap = std::min(cap, (free_b + ds.fused_part.n * sizeof(double)) / 10);
        if (bytes > cap) return false;
        ds.fused_part.release();
        if (ds.fused_part.ensure(bytes / sizeof(double)) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
    }
    if (ds.fused_count.ensure((size_t)nb) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

// A device state's scratch buffers (chunk partials, work totals) are shared by every call on it.  A
// call on stream `st` first waits for the previous user of the scratch (possibly another stream:
// rt_trace_device on a caller's stream, rt_render on the scene's own) and records the event again
// when it has enqueued its last use, so asynchronous calls on different streams never overlap on it.
hipError_t order_scratch(DeviceState& ds, hipStream_t st) {
    if (!ds.scratch_used || ds.scratch_stream == st) return hipSuccess;
    return hipStreamWaitEvent(st, ds.scratch_ev, 0);
}
hipError_t release_scratch(DeviceState& ds, hipStream_t st) {
    ds.scratch_stream = st;
    ds.scratch_used = true;
    return hipEventRecord(ds.scratch_ev, st);
}

// totals = [segments, BVH nodes, sphere tests, triangle tests] of the launches
void fill_stats(rt_stats* st, const rt_scene* sc, const rt_settings* s, const unsigned long long* totals, size_t n,
                const ImageParams& im) {
    st->samples = (uint64_t)n * (uint64_t)std::max(0, im.s_end - im.s_begin);
    st->segments = totals[0];
    if (use_bvh(sc, s)) {
        const uint64_t brute = (uint64_t)sc->home.s64.view.num_planes + sc->home.s64.view.num_boxes;
        st->node_visits = totals[1];
        st->sphere_tests = totals[2];
        st->tri_tests = totals[3];
        st->prim_tests = totals[2] + totals[3] + totals[0] * brute;
        // a walk step reads a 64-B two-child node, or a grid cell's 8-B record range (node_visits then
        // counts cells)
        const bool grid = s->precision == RT_PREC_F32 ? trace_walks_grid(sc->home.s32.view) : trace_walks_grid(sc->home.s64.view);
        st->algorithmic_bytes = (grid ? 8.0 : 64.0) * totals[1] + 16.0 * totals[2] + 36.0 * totals[3] +
                                24.0 * totals[0] * brute + 12.0 * (double)n;
    } else {
        st->node_visits = st->sphere_tests = st->tri_tests = 0;
        st->prim_tests = totals[0] * (uint64_t)sc->num_prims;
        st->algorithmic_bytes = (double)totals[0] * sc->record_bytes + 12.0 * (double)n;
    }
}

// The device states of a render: shard k of rt_settings.devices (k = 0: the scene's own device when
// it is listed first, else a replica), created and uploaded on first use.
int shard_states(rt_scene* sc, const rt_settings* s, std::vector<DeviceState*>& out) {
    out.clear();
    const int n = s->device_count > 1 ? s->device_count : 1;
    if (n == 1) {
        out.push_back(&sc->home);
        return RT_OK;
    }
    for (int k = 0; k < n; ++k) {
        const int dev = s->devices[k];
        if (k == 0 && dev == sc->home.device) {
            out.push_back(&sc->home);
            continue;
        }
        const size_t slot = (size_t)k;                     // replica of shard k
        if (sc->replicas.size() <= slot) sc->replicas.resize(slot + 1, nullptr);
        DeviceState*& r = sc->replicas[slot];
        if (r && r->device != dev) {                       // the device list changed: re-create
            r->release();
            delete r;
            r = nullptr;
        }
        if (!r) {
            int rc = enable_peer(sc->home.device, dev);
            if (rc) return rc;
            r = new DeviceState();
            rc = r->init(dev, sc->hs, sc->desc.d);
            if (rc) {
                r->release();
                delete r;
                r = nullptr;
                return rc;
            }
        }
        out.push_back(r);
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char* rt_last_error(void) { return g_error.c_str(); }

int rt_device_count(int* count) {
    if (!count) return fail(RT_ERR_INVALID, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        *count = 0;
        return fail(RT_ERR_NO_DEVICE, "no HIP device: %s", hipGetErrorString(e));
    }
    *count = n;
    return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out) {
    if (!desc || !out) return fail(RT_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (desc->abi_version != RT_ABI_VERSION) return fail(RT_ERR_INVALID, "abi_version %d != %d", desc->abi_version, RT_ABI_VERSION);
    if (desc->num_objects < 0 || (desc->num_objects > 0 && !desc->objects)) return fail(RT_ERR_INVALID, "objects");
    if (desc->num_materials < 0 || (desc->num_materials > 0 && !desc->materials)) return fail(RT_ERR_INVALID, "materials");
    if (desc->num_triangles < 0 || (desc->num_triangles > 0 && !desc->triangles)) return fail(RT_ERR_INVALID, "triangles");
    if (desc->background < 0 || desc->background > RT_BG_NAN) return fail(RT_ERR_INVALID, "background %d", desc->background);
    for (int i = 0; i < 512; ++i)
        if (desc->perm[i] < 0 || desc->perm[i] > 255) return fail(RT_ERR_INVALID, "perm[%d] = %d", i, desc->perm[i]);
    for (int i = 0; i < desc->num_materials; ++i)
        if (desc->materials[i].type < 0 || desc->materials[i].type > RT_MAT_EMISSIVE)
            return fail(RT_ERR_INVALID, "material %d: type %d", i, desc->materials[i].type);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID, "device %d of %d", device, ndev);
    rt_scene* sc = new rt_scene();
    std::string err;
    if (!pack_host(*desc, sc->hs, err)) {
        delete sc;
        return fail(RT_ERR_INVALID, "%s", err.c_str());
    }
    build_bvhs(sc->hs);
    choose_walk(sc->hs, *desc);
    sc->desc.set(*desc);
    sc->num_prims = sc->hs.num_prims;
    sc->bvh_prims = (int)(sc->hs.sphere_r.size() + sc->hs.tri_mat.size());
    sc->bvh_ok = sc->hs.bvh_depth <= RT_BVH_STACK;
    sc->tri_bvh = !sc->hs.tri_wide.empty();
    sc->record_bytes = sc->hs.record_bytes;
    int rc = sc->home.init(device, sc->hs, sc->desc.d);
    hipError_t e = hipSuccess;
    for (int k = 0; k < 2 && !rc && e == hipSuccess; ++k) e = hipEventCreate(&sc->ev[k]);
    if (!rc && e == hipSuccess)
        e = hipHostMalloc((void**)&sc->ctl, kCtlWords * sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent);
    if (!rc && e == hipSuccess) {
        memset(sc->ctl, 0, kCtlWords * sizeof(uint32_t));
        e = hipHostGetDevicePointer((void**)&sc->ctl_dev, sc->ctl, 0);
    }
    if (!rc && e != hipSuccess) rc = fail(RT_ERR_DEVICE, "event create: %s", hipGetErrorString(e));
    if (rc) {
        rt_scene_destroy(sc);
        return rc;
    }
    *out = sc;
    return RT_OK;
}

void rt_scene_destroy(rt_scene* sc) {
    if (!sc) return;
    for (DeviceState* r : sc->replicas)
        if (r) {
            r->release();
            delete r;
        }
    sc->home.release();
    (void)hipSetDevice(sc->home.device);
    sc->mean.release(); sc->post.release(); sc->post_raw.release();
    for (MergeSlot& m : sc->merge) m.release();
    sc->rgba.release();
    for (GammaSlot& g : sc->gamma_slots) g.release();
    for (uint8_t* p : sc->preview_host)
        if (p) (void)hipHostFree(p);
    if (sc->ctl) (void)hipHostFree(sc->ctl);
    for (hipEvent_t e : {sc->ev[0], sc->ev[1]})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : sc->batch_done)
        if (e) (void)hipEventDestroy(e);
    delete sc;
}

int rt_cancel(rt_scene* sc) {
    if (!sc) return fail(RT_ERR_INVALID, "scene is NULL");
    sc->cancel.store(1);
    if (sc->ctl) {
        ctl_cancel(sc->ctl, 1);             // the one-wave pool kernels skip their items from here on
        (void)cancel_pool_launches(sc->ctl_dev + kCtlCancel);   // the LDS pool launches' queues end
    }
    return RT_OK;
}

}  // extern "C"

namespace {

// Shard k of the sample range [b, e) over n shards (contiguous, sizes differ by at most one).
void shard_range(int b, int e, int k, int n, int& sb, int& se) {
    const long long len = e - b;
    sb = b + (int)(len * k / n);
    se = b + (int)(len * (k + 1) / n);
}

// Adds the replicas' sums (and counters) of the batch just traced into the home device's, in shard
// order, without a host wait: each replica copies its batch sums over xGMI into its own staging slot on
// the home device from its own stream (the copies of all replicas run at once, one link each) and then
// zeroes them for its next batch; the home stream waits for each copy and adds the slots in shard
// order, then records that the slot is free (the replica's next copy waits for that).  The home
// device's own trace of the next batch follows the adds on its stream, so the running sums see the same
// sequence of additions as a merge after every batch done synchronously: a checkpoint holds exactly
// the merged batches and a resumed render is bit-identical.
int merge_shards(rt_scene* sc, const std::vector<DeviceState*>& states, size_t n, bool segs, bool draws) {
    DeviceState& h = sc->home;
    if (sc->merge.size() < states.size()) sc->merge.resize(states.size());
    for (size_t k = 0; k < states.size(); ++k) {
        DeviceState* ds = states[k];
        if (ds == &h) continue;
        MergeSlot& m = sc->merge[k];
        HIP_TRY(hipSetDevice(h.device));
        HIP_TRY(m.sum.ensure(3 * n));
        if (segs) HIP_TRY(m.segs.ensure(n));
        if (draws) HIP_TRY(m.draws.ensure(n));
        if (!m.added) HIP_TRY(hipEventCreateWithFlags(&m.added, hipEventDisableTiming));
        HIP_TRY(hipSetDevice(ds->device));
        if (m.pending) HIP_TRY(hipStreamWaitEvent(ds->stream, m.added, 0));    // the slot's last adds are done
        HIP_TRY(hipMemcpyPeerAsync(m.sum.p, h.device, ds->sum.p, ds->device, 3 * n * sizeof(double), ds->stream));
        if (segs) HIP_TRY(hipMemcpyPeerAsync(m.segs.p, h.device, ds->segs.p, ds->device, n * sizeof(uint32_t), ds->stream));
        if (draws) HIP_TRY(hipMemcpyPeerAsync(m.draws.p, h.device, ds->draws.p, ds->device, n * sizeof(uint32_t), ds->stream));
        HIP_TRY(hipEventRecord(ds->copy_ev, ds->stream));
        HIP_TRY(hipMemsetAsync(ds->sum.p, 0, 3 * n * sizeof(double), ds->stream));
        if (segs) HIP_TRY(hipMemsetAsync(ds->segs.p, 0, n * sizeof(uint32_t), ds->stream));
        if (draws) HIP_TRY(hipMemsetAsync(ds->draws.p, 0, n * sizeof(uint32_t), ds->stream));
        HIP_TRY(hipSetDevice(h.device));
        HIP_TRY(hipStreamWaitEvent(h.stream, ds->copy_ev, 0));
        HIP_TRY(launch_add<double>(h.sum.p, m.sum.p, 3 * n, h.stream));
        if (segs) HIP_TRY(launch_add<uint32_t>(h.segs.p, m.segs.p, n, h.stream));
        if (draws) HIP_TRY(launch_add<uint32_t>(h.draws.p, m.draws.p, n, h.stream));
        HIP_TRY(hipEventRecord(m.added, h.stream));
        m.pending = true;
    }
    return RT_OK;
}

// rt_render and rt_render_resume: trace samples [first, sample_end) on top of `sums_in` (NULL: zeros;
// `resident`: the sums the scene's home device already holds, its checkpoint).
//
// Batches (rt_settings.batch_samples) are pipelined: batch k+1 is enqueued before the host waits for
// batch k, so the GPU never idles on the host's progress call.  With the sample pool and more than one
// batch, consecutive batches also trace on two streams into their own chunk partials (trace_overlapped):
// the next batch's waves fill the CUs while the previous one drains, and the reduces add the partials in
// batch order, so the sums are bit-identical to running the batches one after the other (and to a
// checkpoint + resume at any batch boundary).  A cancel (progress() returning non-zero, rt_cancel) stops
// the overlapped batches at their next (tile, chunk) item — a wave's item, about a millisecond — and
// the checkpoint is the batches fully reduced by then (`gated`); without overlapped batches it is
// observed after a batch, and the batches already queued complete.  Several devices: whole batches
// round-robin (trace_replica), or every batch split over the devices (merge_shards).
// rt_settings.batch_samples = -N: about N progress batches whose size is a multiple of the sample pool's
// chunk for the render (its rule for the whole sample range [sample_begin, samples), as for one device), so
// that every batch's items are the one-batch render's items.  Batches of ceil(S / N) samples otherwise cut
// the chunks: mesh50k (chunk 12) in 16 batches of 16 spp takes one 16-sample chunk per batch, +4 % against
// one batch.  The resolution depends only on the settings and the scene, so a resume sees
// the same batches.
int progress_batch(const rt_scene* sc, const rt_settings* s, int cw, int ch, int steps) {
    const int base = std::max(0, s->sample_begin);
    const int end = s->sample_end > 0 ? std::min(s->sample_end, s->samples) : s->samples;
    const int total = std::max(1, end - base);
    const int target = std::max(1, (total + steps - 1) / steps);
    if (!use_pool(s)) return target;
    const int h = pool_plan(cw, ch, total, sc->tri_bvh).chunk;
    if (h <= 0 || h >= target) return target;
    return h * std::max(1, (int)std::lround((double)target / (double)h));
}

int render_impl(rt_scene* sc, const rt_settings* s_in, const rt_output* out, rt_progress_fn progress, void* user,
                rt_stats* stats, const double* sums_in, int first, bool resident = false) {
    const double t_start = now_ms();
    if (!sc) return fail(RT_ERR_INVALID, "scene is NULL");
    int cw, ch;
    int rc = check_settings(s_in, &cw, &ch);
    rt_settings s_local = s_in ? *s_in : rt_settings{};
    if (!rc && s_local.batch_samples < 0) s_local.batch_samples = progress_batch(sc, s_in, cw, ch, -s_local.batch_samples);
    const rt_settings* s = &s_local;
    if (!rc) rc = check_accel(sc, s);
    if (rc) return rc;
    std::vector<DeviceState*> states;
    if ((rc = shard_states(sc, s, states))) return rc;
    // no checkpoint from here until the new sums are consistent (set below, with the samples they hold):
    // a render that fails in between leaves none, rather than old metadata over overwritten sums
    sc->ckpt_pixels = 0;
    sc->cancel.store(0);
    ctl_cancel(sc->ctl, 0);
    // this render's LDS pool launches are registered under its cancel word until it returns
    struct LaunchScope {
        const uint32_t* word;
        ~LaunchScope() { forget_pool_launches(word); }
    } launch_scope{sc->ctl_dev + kCtlCancel};
    if (++sc->render_gen == 0) sc->render_gen = 1;   // 0 is the words' initial value
    for (DeviceState* ds : states) register_cancel_word(sc->ctl_dev + kCtlCancel, ds->device, ds->cancel_word.p, sc->render_gen);
    const size_t n = (size_t)cw * ch;
    const bool want_segs = out && out->segments, want_draws = out && out->draws;
    const bool pool = use_pool(s);
    ImageParams im = image_params(s, cw, ch);
    const int base = im.s_begin;                  // the sums hold samples [base, done) of every pixel
    im.s_begin = std::max(im.s_begin, first);
    const int s0 = im.s_begin, s1 = std::max(im.s_end, s0);
    const int nsh = (int)states.size();
    DeviceState& h = sc->home;
    static const bool overlap_env = !(getenv("RT_OVERLAP") && getenv("RT_OVERLAP")[0] == '0');   // A/B runs
    // Several devices with the sample pool: whole batches round-robin (batch k on states[k % nsh],
    // trace_replica), at least one batch per device — the batch size counts from sample_begin, so a
    // resume at a batch boundary sees the same batches.  Every batch's pool waves take min(batch, chunk)
    // samples, chunk being the pool's rule for the whole render (as one device's batches do), so the
    // sums are bit-identical to the same batches on one device.
    bool whole = nsh > 1 && pool && s->max_depth > 0 && overlap_env && s1 > s0;
    // A batch of B samples is split into round(B / h) equal chunks (at least one), h being the pool's
    // rule for the render's whole share: min(h, B)-sample chunks left a short remainder chunk in every
    // batch (mesh50k in 16 batches of 16 spp: chunks of 12 + 4, 77.2 ms vs 75.0 ms as one 16-sample
    // chunk).  B is the batch setting, not the samples left, so a resume sees the same chunks.
    auto balanced = [](int h, int b) {
        if (h <= 0 || b <= 0) return h;
        const int n = std::max(1, (int)std::lround((double)b / (double)h));
        return (b + n - 1) / n;
    };
    int whole_batch = 0, whole_chunk = 0;
    if (whole) {
        const int full = s->batch_samples > 0 ? s->batch_samples : std::max(1, s1 - base);
        whole_batch = std::max(1, std::min(full, (s1 - base + nsh - 1) / nsh));
        whole_chunk = balanced(pool_plan(cw, ch, std::max(1, s1 - base), sc->tri_bvh).chunk, whole_batch);
        const int ns = std::min(whole_batch, s1 - s0);
        const size_t bytes = pool_plan(cw, ch, ns, sc->tri_bvh, std::min(whole_chunk, ns)).part_bytes;
        for (int k = 0; k < nsh && whole; ++k) {    // every device's partial slots must fit, else split batches
            HIP_TRY(hipSetDevice(states[k]->device));
            whole = ensure_overlap_partials(*states[k], bytes);
        }
    }
    const int batch = whole ? whole_batch : s->batch_samples > 0 ? s->batch_samples : std::max(1, s1 - s0);
    const int nb = s1 > s0 ? (s1 - s0 + batch - 1) / batch : 0;
    const bool want_preview = out && out->preview_rgba8 && nb > 1;
    std::vector<Counters> cs(nsh);
    // Several batches (split mode): every batch's pool waves take min(batch, chunk) samples, chunk being
    // the pool's rule for the shard's whole share of the render (not for one batch: short chunks lengthen
    // each wave's drain relative to its work), balanced over the shard's part of a full batch.  The same
    // batches give the same chunks on a resume (the share is counted from sample_begin), so a resumed
    // render stays bit-identical — also when the resume has a single batch left (the render as a whole,
    // from sample_begin, has several: before round 5 that batch took the pool's rule for its own
    // samples, 1-ulp differences in the resumed sums).
    std::vector<int> chunk_hint(nsh, whole ? whole_chunk : 0);
    if (pool && !whole && (nb > 1 || (s->batch_samples > 0 && s->batch_samples < s1 - base)))
        for (int k = 0; k < nsh; ++k) {
            int a, b, fa, fb;
            shard_range(base, s1, k, nsh, a, b);
            shard_range(0, batch, k, nsh, fa, fb);
            chunk_hint[k] = balanced(pool_plan(cw, ch, std::max(1, b - a), sc->tri_bvh).chunk, fb - fa);
        }
    auto batch_chunk = [&](int k, int ns) { return chunk_hint[k] > 0 ? std::max(1, std::min(chunk_hint[k], ns)) : 0; };
    // overlapped batches: the pool with several batches (always in whole-batch mode).  Not with per-pixel
    // counters over a split of every batch: the trace kernels add those directly, and a replica's merge
    // zeroes them between batches
    bool overlap = whole || (overlap_env && pool && nb > 1 && s->max_depth > 0 && !(nsh > 1 && (want_segs || want_draws)));
    for (int k = 0; k < nsh; ++k) {
        DeviceState& ds = *states[k];
        HIP_TRY(hipSetDevice(ds.device));
        HIP_TRY(ds.sum.ensure(3 * n));
        HIP_TRY(ds.total.ensure(kTotalSlots));
        if (whole) continue;
        int b0, b1;
        shard_range(s0, s0 + std::min(batch, s1 - s0), k, nsh, b0, b1);
        const int ns = std::max(1, b1 - b0);
        if (overlap) overlap = ensure_overlap_partials(ds, pool_plan(cw, ch, ns, sc->tri_bvh, batch_chunk(k, ns)).part_bytes);
    }
    if (whole && sc->merge.size() < states.size()) sc->merge.resize(states.size());
    const int ahead = whole ? lookahead(nsh) : kSlots;   // batches queued beyond the one the host waits for
    const int ring = ahead + kSlots;                      // completion events / preview frames
    // A cancel inside a batch: the pool kernels read the cancel word before every item, and a batch with
    // untraced items is never reduced (ReduceGate), nor is any batch after it, so the sums always hold
    // the batches [0, k) for some k.  For batches reduced on one stream in batch order: one device, or
    // the whole-batch split.  The split of every batch over devices observes a cancel between batches.
    static const bool item_cancel = !(getenv("RT_ITEM_CANCEL") && getenv("RT_ITEM_CANCEL")[0] == '0');   // A/B runs
    static const bool fuse_env = !(getenv("RT_FUSED_BATCHES") && getenv("RT_FUSED_BATCHES")[0] == '0');   // A/B runs
    // (RT_ITEM_CANCEL=0 with fused batches: the gates run, the kernels poll no cancel word — A/B only)
    const bool gated = (item_cancel || (fuse_env && nsh == 1)) && overlap && (nsh == 1 || whole);
    if (gated) {
        HIP_TRY(hipSetDevice(h.device));
        HIP_TRY(h.gate_skip.ensure(1));
    }
    // Fused batches (one device, overlapped gated batches): every batch in ONE pool launch, its items
    // batch-major in the pool's queue (launch_trace_batches: the same items, chunks and partials as one
    // launch per batch), and each batch's reduce enqueued by the host once the batch's last item has
    // raised its flag — the persistent workgroups never drain between batches (16 batches of config 3
    // drained for 3.5 % of the trace time).  The reduces (16 VGPRs) and the preview frames (gamma
    // thresholds, 29 VGPRs) run beside the trace waves, which leave 32 of a SIMD's 512 VGPRs free.
    // Several devices (the whole-batch split): device d traces its batches k = d, d + N, ... in one launch
    // (ImageParams::batch_ways), raising batch k's flag; the host then copies that batch's partials to
    // the home device and reduces them there in batch order — the copies and reduces of trace_replica,
    // from one launch per device instead of one per batch.
    int fchunk = 0;
    size_t fdoubles = 0;
    bool fused = fuse_env && gated && nb > 1 && nb <= kMaxFused && (whole || (nsh == 1 && states[0] == &h));
    if (fused) {
        fchunk = batch_chunk(0, batch);
        fdoubles = fused_batch_doubles(cw, ch, batch, sc->tri_bvh, fchunk);
        for (int d = 0; d < nsh && fused; ++d) {
            HIP_TRY(hipSetDevice(states[d]->device));
            fused = ensure_fused(*states[d], fdoubles, (nb - d + nsh - 1) / nsh);
        }
    }
    bool fused_launched = false;
    for (int k = 0; k < nsh; ++k) {
        DeviceState& ds = *states[k];
        HIP_TRY(hipSetDevice(ds.device));
        Counters& c = cs[k];
        c = Counters{ds.sum.p, nullptr, nullptr, ds.total.p};
        c.cancel_dev = ds.cancel_word.p;
        c.cancel_gen = sc->render_gen;
        int b0, b1;
        shard_range(s0, s0 + std::min(batch, s1 - s0), k, nsh, b0, b1);
        const int ns = std::max(1, b1 - b0);
        if (!overlap && s->max_depth > 0 && (rc = ensure_partials(sc, ds, cw, ch, ns, pool, c, batch_chunk(k, ns)))) return rc;
        HIP_TRY(order_scratch(ds, ds.stream));
        if (resident && &ds == &h) {
            // the scene's checkpoint is already in place
        } else if (sums_in && &ds == &h)
            HIP_TRY(hipMemcpyAsync(ds.sum.p, sums_in, 3 * n * sizeof(double), hipMemcpyHostToDevice, ds.stream));
        else
            HIP_TRY(hipMemsetAsync(ds.sum.p, 0, 3 * n * sizeof(double), ds.stream));
        HIP_TRY(hipMemsetAsync(ds.total.p, 0, kTotalSlots * sizeof(unsigned long long), ds.stream));
        if (want_segs) {
            HIP_TRY(ds.segs.ensure(n));
            HIP_TRY(hipMemsetAsync(ds.segs.p, 0, n * sizeof(uint32_t), ds.stream));
            c.segs = ds.segs.p;
        }
        if (want_draws) {
            HIP_TRY(ds.draws.ensure(n));
            HIP_TRY(hipMemsetAsync(ds.draws.p, 0, n * sizeof(uint32_t), ds.stream));
            c.draws = ds.draws.p;
        }
        HIP_TRY(hipEventRecord(ds.ev[0], ds.stream));
        if (overlap) {                            // the trace streams start after this set-up
            HIP_TRY(hipEventRecord(ds.setup_ev, ds.stream));
            for (hipStream_t t : ds.tstream) HIP_TRY(hipStreamWaitEvent(t, ds.setup_ev, 0));
        }
    }
    if (states[0] != &h) {                        // the home device only merges: its buffers start here
        HIP_TRY(hipSetDevice(h.device));
        HIP_TRY(h.sum.ensure(3 * n));
        if (resident) {
            // the scene's checkpoint is already in place
        } else if (sums_in) HIP_TRY(hipMemcpyAsync(h.sum.p, sums_in, 3 * n * sizeof(double), hipMemcpyHostToDevice, h.stream));
        else HIP_TRY(hipMemsetAsync(h.sum.p, 0, 3 * n * sizeof(double), h.stream));
        if (want_segs) {
            HIP_TRY(h.segs.ensure(n));
            HIP_TRY(hipMemsetAsync(h.segs.p, 0, n * sizeof(uint32_t), h.stream));
        }
        if (want_draws) {
            HIP_TRY(h.draws.ensure(n));
            HIP_TRY(hipMemsetAsync(h.draws.p, 0, n * sizeof(uint32_t), h.stream));
        }
    }
    HIP_TRY(hipSetDevice(h.device));
    if ((int)sc->batch_done.size() < ring) sc->batch_done.resize(ring, nullptr);
    for (hipEvent_t& e : sc->batch_done)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (want_preview) {
        if (sc->preview_host_n < 4 * n || (int)sc->preview_host.size() < ring) {
            for (uint8_t*& p : sc->preview_host) {
                if (p) (void)hipHostFree(p);
                p = nullptr;
            }
            sc->preview_host_n = 0;
            sc->preview_host.assign(ring, nullptr);
            sc->preview_dev.assign(ring, nullptr);
            for (int k = 0; k < ring; ++k) {
                HIP_TRY(hipHostMalloc((void**)&sc->preview_host[k], 4 * n, hipHostMallocMapped));
                HIP_TRY(hipHostGetDevicePointer((void**)&sc->preview_dev[k], sc->preview_host[k], 0));
            }
            sc->preview_host_n = 4 * n;
        }
    }
    // the running frames' RGBA8 thresholds for this gamma (exact bytes without a binary64 pow: preview_kernel)
    GammaSlot* thresholds = nullptr;
    if (want_preview) {
        HIP_TRY(hipSetDevice(h.device));
        thresholds = gamma_table(sc, s->gamma);
    }
    sc->ckpt_pixels = n;
    sc->ckpt_done = s0;
    sc->ckpt_key = ckpt_key(s, cw, ch);
    ctl_store(sc->ctl, kCtlStop, 0);
    ctl_store(sc->ctl, kCtlDone, (uint32_t)s0);

    int enqueued = 0;                             // batches [0, enqueued) are queued on the GPU
    std::vector<unsigned> slots_used(nsh, 0);     // whole-batch split: the partial slots each device traced into
    // enqueue batch kb (no host wait): every shard's trace, the merge of the shards into the home device,
    // the preview frame, then batch_done[kb % ring] on the home stream
    auto enqueue = [&](int kb) -> int {
        const int b = s0 + kb * batch, be = std::min(s1, b + batch);
        ReduceGate gate;                          // gated: batch kb's cancel and commit words
        const ReduceGate* gp = nullptr;
        if (gated) {
            // fused: the batch's flag commits it (a word no kernel writes stands in for `aborted`)
            const int w = fused ? kCtlFusedAborted : kCtlAborted + kb % ring;
            if (!fused) ctl_store(sc->ctl, w, 0);   // batch kb - ring, the slot's last user, has completed
            gate.aborted = sc->ctl_dev + w;
            if (fused) gate.complete = sc->ctl_dev + kCtlFlag + kb;
            gate.stop = sc->ctl_dev + kCtlStop;
            gate.done = reinterpret_cast<int32_t*>(sc->ctl_dev + kCtlDone);
            gate.done_value = be;
            gate.skip = h.gate_skip.p;
            gp = &gate;
        }
        // fused batches with running frames: RT_FUSED_PREVIEW=1 (A/B) the batch's reduce and its frame in one
        // kernel (reduce_preview_kernel) — measured slower: mesh50k 22 batches with running frames 77.6 vs
        // 76.1 ms kernel time for the two kernels (config 3: 96.0 vs 95.9), DESIGN.md §4
        static const bool fused_preview_env = getenv("RT_FUSED_PREVIEW") && getenv("RT_FUSED_PREVIEW")[0] == '1';
        const bool fuse_prev = fused && fused_preview_env && want_preview && be < s1 && thresholds;
        bool previewed = false;
        auto reduce_batch = [&](const ImageParams& bi, const double* src) -> hipError_t {
            if (!fuse_prev) return launch_reduce(bi, h.sum.p, src, sc->tri_bvh, h.stream, gp);
            FinalizeParams fp{(int)n, be - base, s->tone_map, s->exposure, s->gamma};
            hipError_t e = launch_reduce_preview(bi, h.sum.p, src, sc->tri_bvh, h.stream, gp, fp, thresholds->table(),
                                                 sc->preview_dev[kb % ring]);
            if (e == hipSuccess) e = gamma_used(thresholds, h.stream);
            previewed = e == hipSuccess;
            return e;
        };
        auto with_cancel = [&](Counters c) {
            if (gated) {
                if (item_cancel) c.cancel = sc->ctl_dev + kCtlCancel;
                c.aborted = const_cast<uint32_t*>(gate.aborted);
            }
            return c;
        };
        if (fused) {                              // one launch per device, then batch kb's reduce
            const bool bvh = use_bvh(sc, s);
            if (kb == 0) {
                for (int k = 0; k < nb; ++k) ctl_store(sc->ctl, kCtlFlag + k, 0);
                ctl_store(sc->ctl, kCtlFusedAborted, 0);
                ctl_store(sc->ctl, kCtlFusedAborted + 1, 0);
                for (int e = 0; e < nsh; ++e) {   // device e: batches e, e + nsh, ... (all of them when nsh = 1)
                    DeviceState& de = *states[e];
                    HIP_TRY(hipSetDevice(de.device));
                    const int nbe = (nb - e + nsh - 1) / nsh;
                    HIP_TRY(hipMemsetAsync(de.fused_count.p, 0, nbe * sizeof(uint32_t), de.tstream[0]));
                    Counters c = with_cancel(cs[e]);
                    c.aborted = sc->ctl_dev + kCtlFusedAborted + 1;   // written by skipping waves, read by no gate
                    c.batch_count = de.fused_count.p;
                    c.batch_flag = sc->ctl_dev + kCtlFlag + e;          // batch k = e + lb * nsh
                    ImageParams fi = im;
                    fi.s_begin = s0 + e * batch;
                    fi.s_end = s1;
                    fi.pool_chunk = fchunk;
                    fi.batch_ways = nsh;
                    const size_t fb = de.fused_part.n * sizeof(double);
                    HIP_TRY(s->precision == RT_PREC_F32
                                ? launch_trace_batches<float>(de.s32.view, fi, c, bvh, batch, de.fused_part.p, fb, de.tstream[0])
                                : launch_trace_batches<double>(de.s64.view, fi, c, bvh, batch, de.fused_part.p, fb, de.tstream[0]));
                    HIP_TRY(hipEventRecord(de.fused_done, de.tstream[0]));
                }
                fused_launched = true;
            }
            const int d = kb % nsh, lb = kb / nsh;
            DeviceState& ds = *states[d];
            // the host waits for batch kb's flag; without it (a cancel: its items stay untraced) the
            // consumer stream waits for the device's launch to end, so the gate reads the final words
            for (;;) {
                if (ctl_load(sc->ctl, kCtlFlag + kb)) break;
                if (sc->cancel.load()) {          // (launches registered after rt_cancel's call, too)
                    (void)cancel_pool_launches(sc->ctl_dev + kCtlCancel);
                    break;
                }
                const hipError_t q = hipEventQuery(ds.fused_done);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) {      // a device fault, not a cancel: fail with the HIP error
                    (void)hipGetLastError();
                    return fail(RT_ERR_DEVICE, "fused batch %d: %s", kb, hipGetErrorString(q));
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            const bool flagged = ctl_load(sc->ctl, kCtlFlag + kb) != 0;
            ImageParams bi = im;
            bi.s_begin = b;
            bi.s_end = be;
            bi.pool_chunk = fchunk;
            const double* src = ds.fused_part.p + (size_t)lb * fdoubles;
            if (&ds == &h) {
                HIP_TRY(hipSetDevice(h.device));
                if (!flagged) HIP_TRY(hipStreamWaitEvent(h.stream, h.fused_done, 0));
                HIP_TRY(reduce_batch(bi, src));
            } else {                              // a replica's batch: its partials to the home device first
                MergeSlot& m = sc->merge[d];
                const int j = lb % kSlots;
                const size_t bytes = pool_plan(cw, ch, be - b, sc->tri_bvh, fchunk).part_bytes;
                HIP_TRY(hipSetDevice(h.device));
                HIP_TRY(m.stage[j].ensure(fdoubles));
                if (!m.stage_free[j]) HIP_TRY(hipEventCreateWithFlags(&m.stage_free[j], hipEventDisableTiming));
                HIP_TRY(hipSetDevice(ds.device));
                if (!flagged) HIP_TRY(hipStreamWaitEvent(ds.stream, ds.fused_done, 0));
                if (m.stage_used[j]) HIP_TRY(hipStreamWaitEvent(ds.stream, m.stage_free[j], 0));
                HIP_TRY(hipMemcpyPeerAsync(m.stage[j].p, h.device, src, ds.device, bytes, ds.stream));
                HIP_TRY(hipEventRecord(ds.traced[j], ds.stream));
                HIP_TRY(hipSetDevice(h.device));
                HIP_TRY(hipStreamWaitEvent(h.stream, ds.traced[j], 0));
                HIP_TRY(reduce_batch(bi, m.stage[j].p));
                HIP_TRY(hipEventRecord(m.stage_free[j], h.stream));
                m.stage_used[j] = true;
            }
        }
        if (whole && !fused) {                    // the whole batch on one device, reduced on the home device
            const int k = kb % nsh, lj = kb / nsh, j = lj % kSlots;
            DeviceState& ds = *states[k];
            ImageParams bi = im;
            bi.s_begin = b;
            bi.s_end = be;
            bi.pool_chunk = batch_chunk(k, be - b);
            HIP_TRY(hipSetDevice(ds.device));
            slots_used[k] |= 1u << j;
            if (&ds == &h) HIP_TRY(trace_overlapped(sc, ds, s, bi, with_cancel(cs[k]), j, lj >= kSlots, gp));
            else if (int r = trace_replica(sc, ds, sc->merge[k], s, bi, with_cancel(cs[k]), j, gp)) return r;
        }
        for (int k = 0; k < nsh && !whole && !fused; ++k) { // every shard's launches first: the devices run together
            DeviceState& ds = *states[k];
            ImageParams bi = im;
            shard_range(b, be, k, nsh, bi.s_begin, bi.s_end);
            bi.pool_chunk = batch_chunk(k, bi.s_end - bi.s_begin);
            HIP_TRY(hipSetDevice(ds.device));
            if (overlap) HIP_TRY(trace_overlapped(sc, ds, s, bi, with_cancel(cs[k]), kb % kSlots, kb >= kSlots, gp));
            else HIP_TRY(trace(sc, ds, s, bi, cs[k], ds.stream));
        }
        int r;
        if (nsh > 1 && !whole && (r = merge_shards(sc, states, n, want_segs, want_draws))) return r;
        HIP_TRY(hipSetDevice(h.device));
        if (want_preview && be < s1 && !previewed) {   // the running frame: mean over the samples so far
            // written by the epilogue kernel straight into pinned host memory (over PCIe): a
            // hipMemcpyAsync here is a blit kernel that waits for wave slots behind the trace waves
            // (measured 7-15 ms per 8-MB frame while batches overlap)
            FinalizeParams fp{(int)n, be - base, s->tone_map, s->exposure, s->gamma};
            HIP_TRY(launch_finalize(fp, h.sum.p, nullptr, nullptr, sc->preview_dev[kb % ring], h.stream,
                                    thresholds ? thresholds->table() : nullptr));
            if (thresholds) HIP_TRY(gamma_used(thresholds, h.stream));
        }
        HIP_TRY(hipEventRecord(sc->batch_done[kb % ring], h.stream));
        return RT_OK;
    };
    // host side of batch kb once batch_done: checkpoint state and the preview frame.  merged: the batch
    // is in the sums (gated renders: not if a cancel left it unfinished)
    auto complete = [&](int kb, bool& merged) -> int {
        HIP_TRY(hipEventSynchronize(sc->batch_done[kb % ring]));
        const int be = std::min(s1, s0 + (kb + 1) * batch);
        merged = !gated || (int)ctl_load(sc->ctl, kCtlDone) >= be;
        if (!merged) return RT_OK;
        sc->ckpt_done = be;
        // the running frame, unless the next batch has finished too (its frame supersedes this one: the
        // host does not fall further behind the GPU copying frames nobody will see)
        if (want_preview && be < s1 &&
            !(kb + 1 < enqueued && hipEventQuery(sc->batch_done[(kb + 1) % ring]) == hipSuccess)) {
            memcpy(out->preview_rgba8, sc->preview_host[kb % ring], 4 * n);
            if (out->preview_samples) *out->preview_samples = be - base;
        }
        return RT_OK;
    };
    // the host keeps up to kSlots batches queued beyond the one it waits for (their ordering on the
    // partial slots is device-side: trace_overlapped), so neither the host's progress call nor a preview
    // frame ever delays the start of a batch
    int status = RT_OK;
    auto fill = [&](int upto) -> int {          // enqueue batches [enqueued, upto)
        for (; enqueued < std::min(upto, nb) && !sc->cancel.load(); ++enqueued) {
            const int r = enqueue(enqueued);
            if (r) return r;
        }
        return RT_OK;
    };
    for (int kb = 0; kb < nb && status == RT_OK; ++kb) {
        if ((status = fill(kb + (fused ? 0 : ahead) + 1))) break;   // fused: enqueue(kb) waits for batch kb
        bool merged = true;
        if ((status = complete(kb, merged))) break;
        if (!merged && !sc->cancel.load()) {
            // a gate skipped a batch although nobody cancelled (rt_cancel sets `cancel` before the word the
            // kernels read): an item-count mismatch or a lost flag — an internal failure, not a cancel
            status = fail(RT_ERR_DEVICE, "batch %d was not committed (internal error)", kb);
            break;
        }
        const int be = sc->ckpt_done;
        if (merged && progress && be < s1 && progress((double)(be - s0) / (double)(s1 - s0), user)) {
            sc->cancel.store(1);
            ctl_cancel(sc->ctl, 1);
        }
        if (!merged || sc->cancel.load()) {
            if (gated) {
                // the queued batches stop at their next item and are not reduced; once every stream has
                // drained, the sums hold exactly the batches the gates committed
                ctl_cancel(sc->ctl, 1);
                (void)cancel_pool_launches(sc->ctl_dev + kCtlCancel);
                for (DeviceState* ds : states) ds->sync_all();
                h.sync_all();
                sc->ckpt_done = (int)ctl_load(sc->ctl, kCtlDone);
                if (want_preview && sc->ckpt_done > base && sc->ckpt_done < s1) {   // the checkpoint's frame
                    HIP_TRY(hipSetDevice(h.device));
                    FinalizeParams fp{(int)n, sc->ckpt_done - base, s->tone_map, s->exposure, s->gamma};
                    HIP_TRY(launch_finalize(fp, h.sum.p, nullptr, nullptr, sc->preview_dev[0], h.stream));
                    HIP_TRY(hipStreamSynchronize(h.stream));
                    memcpy(out->preview_rgba8, sc->preview_host[0], 4 * n);
                    if (out->preview_samples) *out->preview_samples = sc->ckpt_done - base;
                }
            } else {
                // the batches in flight finish (and if the last one was among them, the render completed)
                for (int k = kb + 1; k < enqueued && status == RT_OK; ++k) status = complete(k, merged);
            }
            if (status == RT_OK && sc->ckpt_done < s1)
                status = fail(RT_ERR_CANCELLED, "render cancelled after %d samples", sc->ckpt_done);
            break;
        }
    }
    if (status != RT_OK && status != RT_ERR_CANCELLED) {
        // a HIP error inside the pipeline: drain every stream; the checkpoint keeps the last batch whose
        // merge is known to be complete (complete() ran for it), and the scratch is released
        const std::string err = g_error;
        for (DeviceState* ds : states) {
            ds->sync_all();
            (void)release_scratch(*ds, ds->stream);
        }
        h.sync_all();
        (void)hipGetLastError();
        g_error = err;
        return status;
    }
    if (fused_launched)                           // every launch's last waves (counters, work totals) first
        for (DeviceState* ds : states) {
            HIP_TRY(hipSetDevice(ds->device));
            HIP_TRY(hipStreamWaitEvent(ds->stream, ds->fused_done, 0));
        }
    if (whole) {   // every device's accumulation stream after its trace streams; the replicas' counters
        for (int k = 0; k < nsh; ++k) {
            DeviceState* ds = states[k];
            HIP_TRY(hipSetDevice(ds->device));
            for (int j = 0; j < kSlots; ++j)
                if (slots_used[k] & (1u << j)) HIP_TRY(hipStreamWaitEvent(ds->stream, ds->traced[j], 0));
        }
        if ((rc = merge_counters(sc, states, n, want_segs, want_draws))) return rc;
    }
    unsigned long long totals[kTotalSlots] = {};
    float kernel_ms = 0;
    for (DeviceState* ds : states) {
        unsigned long long t[kTotalSlots] = {};
        HIP_TRY(hipSetDevice(ds->device));
        HIP_TRY(hipEventRecord(ds->ev[1], ds->stream));
        HIP_TRY(hipMemcpyAsync(t, ds->total.p, sizeof t, hipMemcpyDeviceToHost, ds->stream));
        HIP_TRY(release_scratch(*ds, ds->stream));
        HIP_TRY(hipStreamSynchronize(ds->stream));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ds->ev[0], ds->ev[1]));
        kernel_ms = std::max(kernel_ms, ms);
        for (int k = 0; k < kTotalSlots; ++k) totals[k] += t[k];
    }
    HIP_TRY(hipSetDevice(h.device));
    HIP_TRY(hipStreamSynchronize(h.stream));          // the merges of the last batch (checkpoint state)
    if (status != RT_OK) return status;
    const bool want_mean = out && out->mean, want_post = out && out->post, want_rgba = out && out->rgba8;
    if (want_mean) HIP_TRY(sc->mean.ensure(3 * n));
    if (want_post) HIP_TRY(sc->post.ensure(4 * n));
    if (want_rgba) HIP_TRY(sc->rgba.ensure(4 * n));
    HIP_TRY(hipEventRecord(sc->ev[0], h.stream));
    HIP_TRY(epilogue(sc, s, cw, ch, h.sum.p, want_mean ? sc->mean.p : nullptr, want_post ? sc->post.p : nullptr,
                     want_rgba ? sc->rgba.p : nullptr, h.stream));
    HIP_TRY(hipEventRecord(sc->ev[1], h.stream));
    if (want_mean) HIP_TRY(hipMemcpyAsync(out->mean, sc->mean.p, 3 * n * sizeof(double), hipMemcpyDeviceToHost, h.stream));
    if (want_post) HIP_TRY(hipMemcpyAsync(out->post, sc->post.p, 4 * n * sizeof(float), hipMemcpyDeviceToHost, h.stream));
    if (want_rgba) HIP_TRY(hipMemcpyAsync(out->rgba8, sc->rgba.p, 4 * n, hipMemcpyDeviceToHost, h.stream));
    if (want_segs) HIP_TRY(hipMemcpyAsync(out->segments, h.segs.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h.stream));
    if (want_draws) HIP_TRY(hipMemcpyAsync(out->draws, h.draws.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h.stream));
    HIP_TRY(hipStreamSynchronize(h.stream));
    if (stats) {
        float fms = 0;
        HIP_TRY(hipEventElapsedTime(&fms, sc->ev[0], sc->ev[1]));
        stats->kernel_ms = kernel_ms;
        stats->finalize_ms = fms;
        fill_stats(stats, sc, s, totals, n, im);
        stats->wall_ms = now_ms() - t_start;
    }
#if RT_PROFILE
    const double cyc = (double)(totals[4] + totals[5] + totals[6]);
    fprintf(stderr, "[rt_profile] wave-max cycles: closest hit %.3f, shading %.3f, regeneration %.3f (%.3e total); "
            "walk iterations: %.3e per lane, %.3e per wave, lane efficiency %.3f, wave-uniform inner-node share %.3f\n",
            totals[4] / cyc, totals[5] / cyc, totals[6] / cyc, cyc, (double)totals[7], (double)totals[8],
            totals[8] ? (double)totals[7] / (64.0 * (double)totals[8]) : 0.0,
            totals[8] ? (double)totals[9] / (double)totals[8] : 0.0);
    fprintf(stderr, "[rt_profile] wave walk iterations with <= 8 lanes walking %.3f, <= 16 %.3f\n",
            totals[8] ? (double)totals[10] / (double)totals[8] : 0.0, totals[8] ? (double)totals[11] / (double)totals[8] : 0.0);
#endif
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_render(rt_scene* sc, const rt_settings* s, const rt_output* out, rt_progress_fn progress, void* user,
              rt_stats* stats) {
    return render_impl(sc, s, out, progress, user, stats, nullptr, 0);
}

int rt_render_checkpoint(rt_scene* sc, double* sums, size_t count, int32_t* samples_done) {
    if (!sc || !samples_done) return fail(RT_ERR_INVALID, "NULL argument");
    if (sc->ckpt_pixels == 0) return fail(RT_ERR_INVALID, "no render to checkpoint");
    if (!sums && count == 0) {                     // samples_done only (the sums stay on the device)
        *samples_done = sc->ckpt_done;
        return RT_OK;
    }
    if (!sums) return fail(RT_ERR_INVALID, "NULL argument");
    if (count != 3 * sc->ckpt_pixels)
        return fail(RT_ERR_INVALID, "checkpoint holds %zu doubles, caller gave %zu", 3 * sc->ckpt_pixels, count);
    HIP_TRY(hipSetDevice(sc->home.device));
    HIP_TRY(hipMemcpyAsync(sums, sc->home.sum.p, count * sizeof(double), hipMemcpyDeviceToHost, sc->home.stream));
    HIP_TRY(hipStreamSynchronize(sc->home.stream));
    *samples_done = sc->ckpt_done;
    return RT_OK;
}

int rt_render_resume(rt_scene* sc, const rt_settings* s, const double* sums, int32_t samples_done,
                     const rt_output* out, rt_progress_fn progress, void* user, rt_stats* stats) {
    if (s && (samples_done < std::max(0, s->sample_begin) || samples_done > s->samples))
        return fail(RT_ERR_INVALID, "samples_done %d outside [sample_begin, samples]", samples_done);
    if (!sums) {                                   // from the scene's own checkpoint, still on its device
        int cw = 0, ch = 0;
        if (!sc) return fail(RT_ERR_INVALID, "scene is NULL");
        if (int rc = check_settings(s, &cw, &ch)) return rc;
        if (sc->ckpt_pixels == 0 || sc->ckpt_pixels != (size_t)cw * ch || samples_done != sc->ckpt_done)
            return fail(RT_ERR_INVALID, "no resident checkpoint of %d samples over %d x %d pixels (sums NULL)",
                        samples_done, cw, ch);
        if (!(sc->ckpt_key == ckpt_key(s, cw, ch)))
            return fail(RT_ERR_INVALID, "the resident checkpoint is of another frame, crop, sample_begin, precision, "
                        "seed, aa_mode or max_depth (sums NULL)");
        return render_impl(sc, s, out, progress, user, stats, nullptr, samples_done, true);
    }
    return render_impl(sc, s, out, progress, user, stats, sums, samples_done);
}

int rt_trace_device(rt_scene* sc, const rt_settings* s, double* d_sum, void* hip_stream, int sync, rt_stats* stats) {
    const double t_start = now_ms();
    if (!sc || !d_sum) return fail(RT_ERR_INVALID, "NULL argument");
    int cw, ch;
    int rc = check_settings(s, &cw, &ch);
    if (!rc) rc = check_accel(sc, s);
    if (rc) return rc;
    if (s->device_count > 1)
        return fail(RT_ERR_INVALID, "rt_trace_device traces on the scene's device (device_count %d): split the "
                    "samples over processes, or use rt_render", s->device_count);
    DeviceState& ds = sc->home;
    HIP_TRY(hipSetDevice(ds.device));
    // NULL is the default (null) stream, as for rt_finalize_device: the caller's zeroing of d_sum and
    // its reduce / epilogue on that stream are ordered with this trace (the scene's own non-blocking
    // stream would not be: a zeroing enqueued on the default stream could run after the trace's
    // reduce pass)
    hipStream_t st = (hipStream_t)hip_stream;
    HIP_TRY(ds.total.ensure(kTotalSlots));
    ImageParams im = image_params(s, cw, ch);
    Counters c{d_sum, nullptr, nullptr, ds.total.p};
    if (s->max_depth > 0 && (rc = ensure_partials(sc, ds, cw, ch, im.s_end - im.s_begin, use_pool(s), c))) return rc;
    HIP_TRY(order_scratch(ds, st));
    HIP_TRY(hipMemsetAsync(ds.total.p, 0, kTotalSlots * sizeof(unsigned long long), st));
    HIP_TRY(hipEventRecord(ds.ev[0], st));
    HIP_TRY(trace(sc, ds, s, im, c, st));
    HIP_TRY(hipEventRecord(ds.ev[1], st));
    unsigned long long totals[kTotalSlots] = {};
    if (sync || stats) HIP_TRY(hipMemcpyAsync(totals, ds.total.p, sizeof totals, hipMemcpyDeviceToHost, st));
    HIP_TRY(release_scratch(ds, st));
    if (sync || stats) {
        HIP_TRY(hipStreamSynchronize(st));
        if (stats) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, ds.ev[0], ds.ev[1]));
            stats->kernel_ms = ms;
            stats->finalize_ms = 0;
            fill_stats(stats, sc, s, totals, (size_t)cw * ch, im);
            stats->wall_ms = now_ms() - t_start;
        }
    }
    return RT_OK;
}

int rt_trace_device_bands(rt_scene* sc, const rt_settings* s, double* d_sum, void* hip_stream, int32_t bands,
                          rt_band_fn band_ready, void* user, rt_stats* stats) {
    const double t_start = now_ms();
    if (!sc || !d_sum) return fail(RT_ERR_INVALID, "NULL argument");
    int cw, ch;
    int rc = check_settings(s, &cw, &ch);
    if (!rc) rc = check_accel(sc, s);
    if (rc) return rc;
    if (s->device_count > 1) return fail(RT_ERR_INVALID, "rt_trace_device_bands traces on the scene's device");
    const int tile_rows = (ch + 7) / 8;
    const int nb = std::max(1, std::min({(int)bands, tile_rows, kMaxFused}));
    ImageParams im = image_params(s, cw, ch);
    auto deliver_all = [&](int from) -> int {   // bands [from, nb) at once (nothing left to overlap)
        for (int b = from; b < nb && band_ready; ++b) {
            im.bands = nb;
            const int r0 = band_row0(im, b) * 8, r1 = std::min(ch, band_row0(im, b + 1) * 8);
            if (band_ready(b, r0, r1 - r0, user)) return fail(RT_ERR_CANCELLED, "band_ready stopped at band %d", b);
        }
        return RT_OK;
    };
    // no pool (sample order) or nothing to trace: rt_trace_device, then every band
    if (!use_pool(s) || s->max_depth <= 0 || im.s_end <= im.s_begin) {
        if ((rc = rt_trace_device(sc, s, d_sum, hip_stream, 0, stats))) return rc;
        return deliver_all(0);
    }
    DeviceState& ds = sc->home;
    HIP_TRY(hipSetDevice(ds.device));
    hipStream_t st = (hipStream_t)hip_stream;
    const PoolPlan plan = pool_plan(cw, ch, im.s_end - im.s_begin, sc->tri_bvh, 0);
    HIP_TRY(ds.total.ensure(kTotalSlots));
    HIP_TRY(ds.fused_count.ensure((size_t)nb));
    HIP_TRY(ds.gate_skip.ensure(1));
    if (ds.part.n * sizeof(double) < plan.part_bytes) {     // every chunk's partials (even one chunk)
        HIP_TRY(scratch_idle(ds));
        HIP_TRY(ds.part.ensure(plan.part_bytes / sizeof(double)));
    }
    HIP_TRY(order_scratch(ds, st));
    for (int b = 0; b < nb; ++b) ctl_store(sc->ctl, kCtlFlag + b, 0);
    ctl_store(sc->ctl, kCtlStop, 0);
    ctl_store(sc->ctl, kCtlFusedAborted, 0);
    // the trace runs on the scene's own trace stream, after the caller's work so far (d_sum's zeroing);
    // the band reduces run on the caller's stream as the bands complete, beside the trace
    hipStream_t ts = ds.tstream[0];
    HIP_TRY(hipMemsetAsync(ds.total.p, 0, kTotalSlots * sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(ds.fused_count.p, 0, (size_t)nb * sizeof(uint32_t), st));
    HIP_TRY(hipEventRecord(ds.setup_ev, st));
    HIP_TRY(hipStreamWaitEvent(ts, ds.setup_ev, 0));
    Counters c{d_sum, nullptr, nullptr, ds.total.p};
    c.batch_count = ds.fused_count.p;
    c.batch_flag = sc->ctl_dev + kCtlFlag;
    const bool bvh = use_bvh(sc, s);
    PoolPlan used{};
    HIP_TRY(hipEventRecord(ds.ev[0], ts));
    HIP_TRY(s->precision == RT_PREC_F32
                ? launch_trace_bands<float>(ds.s32.view, im, c, bvh, nb, ds.part.p, ds.part.n * sizeof(double), &used, ts)
                : launch_trace_bands<double>(ds.s64.view, im, c, bvh, nb, ds.part.p, ds.part.n * sizeof(double), &used, ts));
    HIP_TRY(hipEventRecord(ds.ev[1], ts));
    HIP_TRY(hipEventRecord(ds.fused_done, ts));
    im.bands = nb;
    im.band_chunks = used.chunks;
    im.pool_chunk = used.chunk;
    const int tiles_x = (cw + 7) / 8;
    int status = RT_OK;
    for (int b = 0; b < nb && status == RT_OK; ++b) {
        for (;;) {                                  // band b's items are all done
            if (ctl_load(sc->ctl, kCtlFlag + b)) break;
            const hipError_t q = hipEventQuery(ds.fused_done);
            if (q == hipSuccess) {
                if (!ctl_load(sc->ctl, kCtlFlag + b)) status = fail(RT_ERR_DEVICE, "band %d was not completed (internal error)", b);
                break;
            }
            if (q != hipErrorNotReady) {
                (void)hipGetLastError();
                status = fail(RT_ERR_DEVICE, "band %d: %s", b, hipGetErrorString(q));
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        if (status != RT_OK) break;
        ReduceGate gate;                            // the acquire end of the band's commit (item_done)
        gate.aborted = sc->ctl_dev + kCtlFusedAborted;
        gate.stop = sc->ctl_dev + kCtlStop;
        gate.done = reinterpret_cast<int32_t*>(sc->ctl_dev + kCtlDone);
        gate.done_value = 0;
        gate.skip = ds.gate_skip.p;
        gate.complete = sc->ctl_dev + kCtlFlag + b;
        const int r0 = band_row0(im, b), r1 = band_row0(im, b + 1);
        hipError_t e = launch_reduce_tiles(im, d_sum, ds.part.p, used.tiles, used.chunks, r0 * tiles_x,
                                           (r1 - r0) * tiles_x, st, &gate);
        if (e != hipSuccess) { status = fail(RT_ERR_DEVICE, "band reduce: %s", hipGetErrorString(e)); break; }
        if (band_ready && band_ready(b, r0 * 8, std::min(ch, r1 * 8) - r0 * 8, user))
            status = fail(RT_ERR_CANCELLED, "band_ready stopped at band %d", b);
    }
    // the caller's stream after the whole launch (work totals, and the scratch's next user)
    HIP_TRY(hipStreamWaitEvent(st, ds.fused_done, 0));
    unsigned long long totals[kTotalSlots] = {};
    if (stats) HIP_TRY(hipMemcpyAsync(totals, ds.total.p, sizeof totals, hipMemcpyDeviceToHost, st));
    HIP_TRY(release_scratch(ds, st));
    if (status != RT_OK) {
        const std::string err = g_error;
        (void)hipStreamSynchronize(st);
        g_error = err;
        return status;
    }
    if (stats) {
        HIP_TRY(hipStreamSynchronize(st));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ds.ev[0], ds.ev[1]));
        stats->kernel_ms = ms;
        stats->finalize_ms = 0;
        fill_stats(stats, sc, s, totals, (size_t)cw * ch, im);
        stats->wall_ms = now_ms() - t_start;
    }
    return RT_OK;
}

int rt_scene_walk(rt_scene* sc, int32_t precision, int32_t accel) {
    if (!sc) return fail(RT_ERR_INVALID, "NULL argument");
    if (precision != RT_PREC_F64 && precision != RT_PREC_F32) return fail(RT_ERR_INVALID, "precision %d", precision);
    rt_settings s{};
    s.accel = accel;
    if (s.accel < RT_ACCEL_AUTO || s.accel > RT_ACCEL_BVH) return fail(RT_ERR_INVALID, "accel %d", accel);
    const int rc = check_accel(sc, &s);
    if (rc) return rc;
    if (!use_bvh(sc, &s)) return 0;
    const bool grid = precision == RT_PREC_F32 ? trace_walks_grid(sc->home.s32.view) : trace_walks_grid(sc->home.s64.view);
    return grid ? 2 : 1;
}

int rt_closest_hits(rt_scene* sc, int32_t precision, int32_t accel, const double* rays, size_t n, double* t,
                    int32_t* kind, int32_t* index) {
    if (!sc || (n > 0 && !rays)) return fail(RT_ERR_INVALID, "NULL argument");
    if (precision != RT_PREC_F64 && precision != RT_PREC_F32) return fail(RT_ERR_INVALID, "precision %d", precision);
    rt_settings s{};
    s.accel = accel;
    if (s.accel < RT_ACCEL_AUTO || s.accel > RT_ACCEL_BVH) return fail(RT_ERR_INVALID, "accel %d", accel);
    int rc = check_accel(sc, &s);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    DeviceState& ds = sc->home;
    HIP_TRY(hipSetDevice(ds.device));
    DevBuf<double> d_rays, d_t;
    DevBuf<int> d_kind, d_idx;
    auto cleanup = [&] { d_rays.release(); d_t.release(); d_kind.release(); d_idx.release(); };
    hipError_t e = d_rays.ensure(6 * n);
    if (e == hipSuccess) e = d_t.ensure(n);
    if (e == hipSuccess) e = d_kind.ensure(n);
    if (e == hipSuccess) e = d_idx.ensure(n);
    if (e == hipSuccess) e = hipMemcpyAsync(d_rays.p, rays, 6 * n * sizeof(double), hipMemcpyHostToDevice, ds.stream);
    const bool bvh = use_bvh(sc, &s);
    if (e == hipSuccess)
        e = precision == RT_PREC_F32 ? launch_closest_hits<float>(ds.s32.view, bvh, d_rays.p, n, d_t.p, d_kind.p, d_idx.p, ds.stream)
                                     : launch_closest_hits<double>(ds.s64.view, bvh, d_rays.p, n, d_t.p, d_kind.p, d_idx.p, ds.stream);
    if (e == hipSuccess && t) e = hipMemcpyAsync(t, d_t.p, n * sizeof(double), hipMemcpyDeviceToHost, ds.stream);
    if (e == hipSuccess && kind) e = hipMemcpyAsync(kind, d_kind.p, n * sizeof(int), hipMemcpyDeviceToHost, ds.stream);
    if (e == hipSuccess && index) e = hipMemcpyAsync(index, d_idx.p, n * sizeof(int), hipMemcpyDeviceToHost, ds.stream);
    const hipError_t es = hipStreamSynchronize(ds.stream);
    if (e == hipSuccess) e = es;
    cleanup();
    if (e != hipSuccess) return fail(RT_ERR_DEVICE, "rt_closest_hits: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_finalize_device(rt_scene* sc, const rt_settings* s, const double* d_sum, double* d_mean, float* d_post,
                       uint8_t* d_rgba8, void* hip_stream) {
    if (!sc || !d_sum) return fail(RT_ERR_INVALID, "NULL argument");
    int cw, ch;
    int rc = check_settings(s, &cw, &ch);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(sc->home.device));
    HIP_TRY(epilogue(sc, s, cw, ch, d_sum, d_mean, d_post, d_rgba8, (hipStream_t)hip_stream, true));
    return RT_OK;
}

}  // extern "C"
