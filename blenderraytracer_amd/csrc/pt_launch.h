// pt_launch.h — host-visible launch interface of the path-tracing kernels (pt_trace.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_path.h"

namespace rt {

// Counters::totals slots: 0 segments, 1 BVH nodes, 2 sphere tests, 3 triangle tests; RT_PROFILE builds:
// 4..6 cycles (closest hit, shading, regeneration), 7 / 8 walk iterations per lane / per wave, 9 wave
// iterations whose active lanes all sit at one inner node, 10 / 11 wave iterations with <= 8 / <= 16 lanes walking
constexpr int kTotalSlots = 12;

// chunk partial sums of one 8x8 tile: 3 channels x 64 pixels, binary64
constexpr size_t kPartialBytesPerTile = 3 * 64 * sizeof(double);

struct Counters {
    double* sum;               // n*3 running per-pixel radiance sums (read-modify-write)
    uint32_t* segs;            // optional n per-pixel world.hit counts
    uint32_t* draws;           // optional n per-pixel RNG draws
    unsigned long long* totals;   // optional [segments, BVH nodes, sphere tests, triangle tests]
    double* part = nullptr;    // sample-pool chunk partials (scratch, pool_partial_bytes)
    size_t part_bytes = 0;
    // progressive renders (render_impl): the render's cancel word in mapped host memory.  The one-wave
    // pool kernel reads it as each (tile, chunk) item starts; a workgroup that finds it set leaves its
    // item untraced and sets *aborted (this batch's word, mapped host memory too), so that the batch is
    // never reduced.  The LDS pool kernels read no cancel word: their launches are registered under it,
    // and cancel_pool_launches(cancel) moves their queues past the last item (and sets *aborted).
    // kCancelCopies copies of the word, one per 128-B line (cancel[k * kCancelStride]), the host writes
    // all of them: the waves' reads spread over many lines instead of queueing on one
    const uint32_t* cancel = nullptr;
    uint32_t* aborted = nullptr;
    // what the one-wave pool kernel actually reads: a copy of the cancel word in device memory
    // (kDevCancelCopies words, one per 128-B line), set to cancel_gen by cancel_pool_launches from a
    // high-priority stream — an L2 hit instead of a read over PCIe per workgroup (mesh50k cancel 25 ms ->
    // DESIGN.md §1).  cancel_gen: the render's generation, so a set left over from an earlier render of
    // the scene never matches.  A fused launch's skipping workgroups leave `aborted` alone (its batches
    // are committed by their flags)
    const uint32_t* cancel_dev = nullptr;
    uint32_t cancel_gen = 0;
    // fused batches (launch_trace_batches): per batch, the items done (device memory, zeroed before the
    // launch) and the flag the item completing the batch raises (mapped host memory: the host enqueues
    // the batch's reduce once it is set, and its gate commits the batch only if it is set)
    uint32_t* batch_count = nullptr;
    uint32_t* batch_flag = nullptr;      // batch b's flag: batch_flag[b * ImageParams::batch_ways]
};
constexpr int kCancelCopies = 128, kCancelStride = 32;
constexpr int kDevCancelCopies = 16;      // device-memory copies (Counters::cancel_dev)

// The commit of one batch's chunk partials (render_impl with a cancel word): a one-thread gate kernel
// before the reduce reads the batch's `aborted` word and the render's sticky `stop` word (both mapped
// host memory); if either is set the batch is not added (and `stop` is set, so no later batch is
// either: the sums always hold a prefix of the batches), else `done` = done_value (the samples the sums
// hold once this reduce has run).  The decision goes to `skip` (device memory), which every reduce
// thread reads, so that the host-memory words are read once per batch.
struct ReduceGate {
    const uint32_t* aborted = nullptr;
    uint32_t* stop = nullptr;
    int32_t* done = nullptr;
    int32_t done_value = 0;
    uint32_t* skip = nullptr;
    // a fused launch's batch: its completion flag (Counters::batch_flag; 0 = items left untraced)
    const uint32_t* complete = nullptr;
};

// bvh: walk the BVHs (ACC_BVH_STACK, the ordered two-child walk), else World order (ACC_BRUTE).
// pool: the sample-pool kernel (+ reduce_kernel when there are several chunks), else the lane-per-pixel
// kernel (samples added in sample order, rt_settings.sum_order = RT_SUM_SAMPLE_ORDER)
template <class R>
hipError_t launch_trace(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh, bool pool,
                        hipStream_t stream);

// the sample pool's split of `ns` samples of a cw x ch crop: 8x8 tiles, samples per chunk, chunks and the
// bytes of all chunk partials of one launch
struct PoolPlan { int tiles, chunk, chunks; size_t part_bytes; };
PoolPlan pool_plan(int cw, int ch, int ns, bool tri_bvh, int chunk = 0);
// the pool kernel writing every chunk (even one) into `part` (>= pool_plan(..).part_bytes), sums untouched:
// batches may trace concurrently on several streams; launch_reduce then adds part to sum in chunk order
template <class R>
hipError_t launch_trace_partials(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh,
                                 double* part, size_t part_bytes, hipStream_t stream);
hipError_t launch_reduce(const ImageParams& im, double* sum, const double* part, bool tri_bvh, hipStream_t stream,
                         const ReduceGate* gate = nullptr);
// All batches of a progressive render in ONE pool launch (items batch-major in the pool's queue): batch
// b = samples [im.s_begin + b * stride, + batch) (stride = batch x im.batch_ways) into part + b *
// fused_batch_doubles(...), each batch's items signalled through c.batch_count / c.batch_flag.  The same items, chunks and partials as one
// launch_trace_partials per batch, so launch_reduce of each batch's partials adds the same bits.
template <class R>
hipError_t launch_trace_batches(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh, int batch,
                                double* part, size_t part_bytes, hipStream_t stream);
// The LDS pool launches of a render (Counters::cancel != nullptr) are registered under its cancel word
// until forget_pool_launches(cancel).  cancel_pool_launches(cancel): for each registered launch not yet
// cancelled, set its `aborted` word, then move its queue past the last item (a one-thread kernel on a
// high-priority stream of the launch's device, beside the trace waves), so that every wave's next take
// ends its loop; the items already taken finish.  A queue moved after its launch ended is zeroed again
// on the launch's stream.  Thread-safe (rt_cancel calls it from any thread); the caller's current
// device is kept.  A launch cancelled after all its items were taken still counts as aborted.
hipError_t cancel_pool_launches(const uint32_t* cancel);
void forget_pool_launches(const uint32_t* cancel);
// the device-memory cancel word (Counters::cancel_dev) of one device of a render registered under its host
// cancel word: cancel_pool_launches(cancel) writes `gen` into it (a one-thread kernel on the device's
// high-priority stream); forget_pool_launches(cancel) drops the registration
void register_cancel_word(const uint32_t* cancel, int device, uint32_t* word, uint32_t gen);

// One launch with its items band-major over `bands` horizontal bands of whole tile rows (pool_order.h
// band_item): every chunk's partials into `part` (>= plan.part_bytes, even for one chunk), band b's items
// counted in c.batch_count[b] and its flag c.batch_flag[b] raised when they are all done.  The same items,
// chunk and partials as launch_trace of the same samples, so reducing every band's tiles
// (launch_reduce_tiles) gives the same sums bit for bit.  plan: the launch's pool plan (out)
template <class R>
hipError_t launch_trace_bands(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh, int bands,
                              double* part, size_t part_bytes, PoolPlan* plan, hipStream_t stream);
hipError_t launch_reduce_tiles(const ImageParams& im, double* sum, const double* part, int tiles, int chunks,
                               int tile0, int ntiles, hipStream_t stream, const ReduceGate* gate = nullptr);

// doubles of one batch's partials in a fused launch, and the items that complete it
size_t fused_batch_doubles(int cw, int ch, int batch, bool tri_bvh, int chunk);
uint32_t fused_batch_items(int cw, int ch, int batch, bool tri_bvh, int chunk);

// World.hit of n rays (n x 6 doubles, device) -> t, kind, index (device): rt_closest_hits
template <class R>
hipError_t launch_closest_hits(const SceneView<R>& sc, bool bvh, const double* rays, size_t n, double* t, int* kind,
                               int* idx, hipStream_t stream);

// default of rt_settings.sum_order = RT_SUM_POOL: the sample pool, unless RT_SAMPLE_POOL=0 is set in the
// environment (A/B runs of the lane-per-pixel kernel)
bool trace_uses_pool();
// the BVH-mode trace of this scene walks the uniform grid (ACC_GRID) rather than a tree
template <class R>
bool trace_walks_grid(const SceneView<R>& sc);
// scratch bytes the sample pool needs to trace `ns` samples of a cw x ch crop in one launch (0: one
// chunk, the partials go straight to the sums).  With less scratch (but at least one chunk's worth,
// tiles x kPartialBytesPerTile) launch_trace splits the samples over several launches.
size_t pool_partial_bytes(int cw, int ch, int ns, bool tri_bvh, int chunk = 0);

// dst[i] += src[i] (n elements, both on the stream's device): merging the shards of a multi-device render
template <class T>
hipError_t launch_add(T* dst, const T* src, size_t n, hipStream_t stream);

struct FinalizeParams {
    int n;
    int samples;
    int tone_map;
    double exposure, gamma;
};
// thresholds: a running frame of a progressive render (RGBA8 only) through preview_kernel, whose bytes
// come from the 255 gamma thresholds of launch_gamma_thresholds instead of a binary64 pow (the same
// bytes as finalize_kernel in 29 VGPRs, so it runs beside the trace waves; pt_trace.hip)
// The RGBA8 bytes of a gamma as a step function of the tone-mapped value (pt_trace.hip preview_kernel):
// t[k - 1] = the least binary64 tm whose byte is >= k, plus the values near the thresholds where the
// device pow is not monotone (exceptions: tm and its byte), found by scanning +-kGammaScan ulps of every
// threshold; overflow: more exceptions than kGammaExc (the table is then not used)
constexpr int kGammaExc = 1024, kGammaScan = 4096;
constexpr double kGammaMin = 0.25, kGammaMax = 4.0;   // gammas whose tables are used (preview_thresholds_ok)
struct GammaTable {
    double t[255];
    uint32_t n_exc, overflow;
    double exc_tm[kGammaExc];
    uint32_t exc_byte[kGammaExc];
};
hipError_t launch_finalize(const FinalizeParams& p, const double* sum, double* mean, float* post, uint8_t* rgba8,
                           hipStream_t stream, const GammaTable* thresholds = nullptr);
bool preview_thresholds_ok(double gamma);
// launch_reduce of a progressive batch and its running frame (preview_kernel's bytes through `table`, into
// rgba8) in one kernel: reduce_preview_kernel (pt_trace.hip).  When the gate skips the batch, neither runs
hipError_t launch_reduce_preview(const ImageParams& im, double* sum, const double* part, bool tri_bvh, hipStream_t stream,
                                 const ReduceGate* gate, const FinalizeParams& fp, const GammaTable* table, uint8_t* rgba8);
hipError_t launch_gamma_thresholds(double gamma, GammaTable* T, hipStream_t stream);
hipError_t launch_denoise(int w, int h, double w1, double w2, const float* in, float* out, uint8_t* rgba8,
                          hipStream_t stream);

}  // namespace rt
