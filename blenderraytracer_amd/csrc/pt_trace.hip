// pt_trace.hip — the path-tracing megakernel and its epilogue for gfx950 (MI355X).
//
// Default (sample pool, trace_pool_kernel): a wave owns an 8x8 pixel tile and one chunk of samples;
// the tile's (pixel, sample) items are dealt to its lanes as they finish, each finished sample's
// radiance is added to the tile's per-pixel partial sums in LDS, and the chunk partials are added to
// the per-pixel float64 sums in chunk order (reduce_kernel).  Per-sample radiance never leaves the CU.
// Lane-per-pixel (trace_kernel, RT_SAMPLE_POOL=0): one lane owns one pixel of the crop window and
// traces that pixel's samples [s_begin, s_end) in order (trace_pixel, pt_path.h) — the exact sample
// order of RayTracer.render, kept as the A/B and test reference.
// BVH mode: every lane walks its own path through the two-child BVH with a per-lane stack in LDS;
// brute-force mode: primitive records are walked in World.objects order by every lane in lockstep, so
// all record loads are wave-uniform scalar loads.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "pt_launch.h"
#include "pool_order.h"
#include "queue_slots.h"

namespace rt {

template <class R>
struct TraceArgs {
    SceneView<R> sc;            // first: start_sample reads the camera at its kernel-argument offset
    ImageParams im;             // (RT_CAM_RELOAD, pt_path.h), so every trace kernel takes TraceArgs
    Counters c;                 // as its first argument
};
static_assert(offsetof(TraceArgs<double>, sc) == 0 && offsetof(TraceArgs<float>, sc) == 0, "sc first");

// One wave (an 8x8 pixel tile) per workgroup: one-wave workgroups measured fastest (RTOW f64 4350 vs
// 4190 Msamples/s for 16x16 tiles, mesh50k 3342 vs 3094): finer work items shorten the frame's tail.
#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 6   // brute force: 80 VGPRs.  At 8 waves (64 VGPRs) the binary64 pool kernel
#endif                            // spills 300 B/lane: Cornell f64 5175 (8) / 6730 (4) / 6830 (6) Msamples/s,
                                  // f32 9274 (8) / 9680 (4) / 9978 (6)
#ifndef RT_BVH_WAVES_PER_SIMD
#define RT_BVH_WAVES_PER_SIMD 4   // binary64 BVH walk: 128 VGPRs (measured 3/4/5 waves: 5405/5462/5092)
#endif
#ifndef RT_BVH_WAVES_F32
#define RT_BVH_WAVES_F32 5        // binary32 BVH walk: 96 VGPRs (measured 4/5/6 waves: 6070/6628/6542)
#endif

#ifndef RT_SPHERES_WAVES_PER_SIMD
#define RT_SPHERES_WAVES_PER_SIMD 5   // binary64 sphere-only walk (ACC_BVH_SPHERES): 96 VGPRs, 13 spilled to
#endif                                // scratch in cold paths; RTOW 128 spp 4 / 5 waves: 7119 / 7335 Msamples/s
#ifndef RT_SPHERES_WAVES_F32
#define RT_SPHERES_WAVES_F32 6       // binary32 sphere-only walk: 80 VGPRs (5 / 6 waves: 8536 / 8800 RTOW f32)
#endif

// the binary64 stack is static (24 entries) unless RT_F64_DYN_STACK (A/B): then, as binary32's, dynamic
// LDS sized to the scene's deepest leaf, which 6 waves/SIMD would need.  Measured on the sphere-only
// kernel, RTOW 512 spp: static 5 waves 7962, dynamic 5 waves 7870, dynamic 6 waves (57 VGPRs spilled)
// 6909 Msamples/s
#ifndef RT_F64_DYN_STACK
#define RT_F64_DYN_STACK 0
#endif
template <class R, int ACC>
constexpr bool dyn_stack() { return sizeof(R) == 4 || (RT_F64_DYN_STACK != 0 && ACC == ACC_BVH_SPHERES); }

#ifndef RT_LDS_OCC_F64
#define RT_LDS_OCC_F64 4          // waves/SIMD of the LDS-node kernel (trace_pool_lds_kernel)
#endif
#ifndef RT_LDS_OCC_F32
#define RT_LDS_OCC_F32 6
#endif

#ifndef RT_GRID_WAVES_PER_SIMD
#define RT_GRID_WAVES_PER_SIMD 5
#endif
#ifndef RT_GRID_WAVES_F32
#define RT_GRID_WAVES_F32 6
#endif
// walks with a per-lane LDS stack (the ordered BVH walks)
template <int ACC>
constexpr bool uses_stack() {
    return ACC == ACC_BVH_STACK || ACC == ACC_BVH_SPHERES || ACC == ACC_BVH_SPHERES_LDS || ACC == ACC_BVH_TRI_LDS ||
           ACC == ACC_BVH_STACK_LEAN;
}

template <class R, int ACC>
constexpr int waves_per_simd() {
    if constexpr (ACC == ACC_GRID || ACC == ACC_GRID_LDS || ACC == ACC_GRID_LDS_LEAN)
        return sizeof(R) == 8 ? RT_GRID_WAVES_PER_SIMD : RT_GRID_WAVES_F32;
    if constexpr (ACC == ACC_BVH_SPHERES) return sizeof(R) == 8 ? RT_SPHERES_WAVES_PER_SIMD : RT_SPHERES_WAVES_F32;
    if constexpr (ACC == ACC_BVH_SPHERES_LDS) return sizeof(R) == 8 ? RT_LDS_OCC_F64 : RT_LDS_OCC_F32;
    if constexpr (ACC == ACC_BVH_TRI_LDS) return sizeof(R) == 8 ? RT_BVH_WAVES_PER_SIMD : RT_BVH_WAVES_F32;
    return ACC >= ACC_BVH ? (sizeof(R) == 8 ? RT_BVH_WAVES_PER_SIMD : RT_BVH_WAVES_F32) : RT_MIN_WAVES_PER_SIMD;
}

// Per-wave reduction of the lanes' work counters into Counters::totals (one 64-bit atomic each).
template <int ACC>
__device__ __forceinline__ void add_totals(const Counters& c, const PixelResult& r, const int lane) {
    if (!c.totals) return;
    const uint32_t parts[4] = {r.segments, r.work.nodes, r.work.spheres, r.work.tris};
    for (int k = 0; k < (ACC >= ACC_BVH ? 4 : 1); ++k) {
        unsigned long long v = parts[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) atomicAdd(c.totals + k, v);
    }
    if constexpr (RT_PROFILE != 0) {
        for (int k = 0; k < 3; ++k) {
            unsigned long long v = r.cyc[k];
            for (int off = 32; off > 0; off >>= 1) v = max(v, (unsigned long long)__shfl_xor(v, off));
            if (lane == 0) atomicAdd(c.totals + 4 + k, v);
        }
        const uint32_t trips[5] = {r.work.lane_trips, r.work.wave_trips, r.work.uni_trips, r.work.low8, r.work.low16};
        for (int k = 0; k < 5; ++k) {
            unsigned long long v = trips[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(c.totals + 7 + k, v);
        }
    }
}

// The render's cancel word (Counters::cancel, mapped host memory written by rt_cancel / the progress
// callback): read with system scope, so the read goes to host memory and not to a cached copy.
#ifndef RT_CANCEL_POLL
#define RT_CANCEL_POLL 1          // A/B: 0 = the kernels never read the cancel word (the gates still run)
#endif
// The one-wave pool kernel reads it as its workgroup (= one item) starts; the LDS pool kernel reads no
// cancel word at all (cancel_pool_launches moves its queue instead: a poll inside its item loop, even
// one read per 16 queue positions, cost config 3's 16 fused batches 3-5 % through the kernel's
// register allocation).
// copy: the wave's copy of the word; one line read by every wave measured 50 us per read (RTOW 16
// progressive batches: +4.5 % kernel time), the reads of one line being serialized.  Round 6: the copy in
// device memory (Counters::cancel_dev, agent scope: an L2 read) instead of the host word (system scope: a
// read over PCIe per workgroup, which bounded how fast a cancelled launch's remaining workgroups drain)
__device__ __forceinline__ bool cancel_requested(const Counters& c, unsigned copy) {
    return RT_CANCEL_POLL && c.cancel_dev &&
           __hip_atomic_load(const_cast<uint32_t*>(c.cancel_dev) + (copy % kDevCancelCopies) * kCancelStride,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c.cancel_gen;
}
// this batch leaves items untraced: its partials must not be reduced (one lane writes; a fused launch's
// batches are committed by their completion flags instead, ReduceGate::complete)
__device__ __forceinline__ void mark_aborted(const Counters& c) {
    __hip_atomic_store(c.aborted, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A chunk partial of a fused launch: stored through to memory (sc1: agent-scope store), since the
// reduce that reads it runs while this launch is still going, on whatever XCD
__device__ __forceinline__ void store_through(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The wave's item of a fused launch is done (the commit protocol of fused batches): the
// write-through hand-off of MI355X_MICROARCH.md ("Valid forms", the counter row; cdna_hip_programming.md
// §6 G16 R1, "sc1 (write-through) stores ... need no release fence"):
//  1. every lane: its partials stored write-through (store_through: global stores with sc1, which leave
//     the XCD's L2 and drop the line there), then `s_waitcnt vmcnt(0)` — the wave's stores have completed
//     at memory (inline asm, which the compiler can neither drop nor move stores across);
//  2. lane 0, after that wait: the batch's item count, a relaxed agent-scope RMW (performed at memory,
//     coherent across XCDs);
//  3. the lane whose increment completes the batch: the batch's flag in mapped host memory, a system-scope
//     release store (one per batch);
//  4. the host sees the flag and enqueues the batch's gate, which loads the flag with a system-scope
//     acquire (reduce_gate_kernel); the reduce follows the gate in stream order, in a dispatch of its own
//     (whose start invalidates the L1s it reads through), and reads the partials from memory.
// The one-wave kernels (this file compiled as pt_onewave.hip) take this form: a release fence per item is
// an L2 write-back (buffer_wbl2 sc1) + wait on gfx950, 712k of them per mesh50k frame — 2 % of that frame
// in progressive batches.  RT_COMMIT_FENCE=1, the LDS pool kernels' form: also an
// agent-scope release fence before the count (the write-through form gave config 3's LDS kernel a
// register allocation 2.3 % slower, measured interleaved) and an acquire fence before the flag.
#ifndef RT_COMMIT_FENCE
#ifdef RT_ONEWAVE_TU
#define RT_COMMIT_FENCE 0
#else
#define RT_COMMIT_FENCE 1
#endif
#endif
__device__ __forceinline__ void item_done(const Counters& c, int b, uint32_t batch_items, int ways, int lane) {
#if RT_COMMIT_FENCE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        const uint32_t k = __hip_atomic_fetch_add(c.batch_count + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k + 1 == batch_items) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(c.batch_flag + b * (ways > 1 ? ways : 1), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
#else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        const uint32_t k = __hip_atomic_fetch_add(c.batch_count + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k + 1 == batch_items)
            __hip_atomic_store(c.batch_flag + b * (ways > 1 ? ways : 1), 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#endif
}

// ---- lane-per-pixel kernel (RT_SAMPLE_POOL=0) ----
template <class R, bool COUNT, int ACC>
__global__ __launch_bounds__(64, (waves_per_simd<R, ACC>()))
void trace_kernel(const TraceArgs<R> args) {
    const ImageParams& im = args.im;
    BvhStack stk{nullptr, 0};
    if constexpr (uses_stack<ACC>()) {
        // per-lane traversal stacks, entry k of lane t at [k * 64 + t]: RT_BVH_STACK (binary64) or
        // sc.stack_entries (binary32: dynamic LDS sized by the launch to the scene's deepest leaf) x 4 B
        if constexpr (sizeof(R) == 8 && !dyn_stack<R, ACC>()) {
            __shared__ int bvh_stack[RT_BVH_STACK * 64];      // measured 1 % faster than the dynamic one
            stk.base = bvh_stack + threadIdx.x;
        } else {
            extern __shared__ int bvh_stack_dyn[];           // binary32 at 5 waves/SIMD: LDS is tight
            stk.base = bvh_stack_dyn + threadIdx.x;
        }
        stk.stride = 64;
    }
    const int lane = threadIdx.x;
    const Tile t = tile_of(im, blockIdx.x);
    const int cx = t.x0 + (lane & 7), cy = t.y0 + (lane >> 3);
    const bool valid = cx < im.cw && cy < im.ch;
    const size_t q = (size_t)cy * im.cw + cx;
    double acc[3] = {0, 0, 0};
    if (valid) { acc[0] = args.c.sum[3 * q]; acc[1] = args.c.sum[3 * q + 1]; acc[2] = args.c.sum[3 * q + 2]; }
    // invalid lanes trace nothing but stay for the wave reduction below
    const PixelResult r = trace_pixel<R, COUNT, ACC>(args.sc, im, cx, cy, valid ? im.s_end : im.s_begin, acc, stk);
    if (valid) {
        args.c.sum[3 * q] = acc[0]; args.c.sum[3 * q + 1] = acc[1]; args.c.sum[3 * q + 2] = acc[2];
        if (COUNT) {
            if (args.c.segs) args.c.segs[q] += r.segments;
            if (args.c.draws) args.c.draws[q] += r.draws;
        }
    }
    add_totals<ACC>(args.c, r, lane);
}

// ---- sample pool (the default trace kernel) ----
// A workgroup is one wave = one 8x8 tile of the crop x one chunk of up to `chunk` samples.  The tile's
// (pixel, sample) items are dealt to the lanes from a wave-uniform counter in sample-major order as
// lanes finish their samples, so a lane whose pixel is cheap (sky) goes on with the samples of its
// neighbours instead of idling until the wave's slowest pixel is done; the lanes still hold pixels of
// one 8x8 block (primary-ray coherence as in trace_kernel).
// Each finished sample's radiance is added (binary64) to its pixel's partial sum in LDS with a
// non-returning LDS atomic (ds_add_f64): the wave does not wait for it.  A wave's execution depends only
// on its items, so a pixel's samples are added in an order fixed by the scene, the tile and the chunk
// (the iteration in which each finishes; lanes finishing the same pixel in one iteration are combined
// by the LDS atomic unit in its fixed lane order) — bit-reproducible from run to run, independent of
// timing and of other waves (tests check it across processes).  Resolving same-pixel collisions in
// explicit lane-order rounds instead (ds_min owner election, or a per-pixel lane mask) costs an LDS
// round trip per iteration: -5 % RTOW f64, -10 % mesh50k, -15 % Cornell.
// At the end the wave writes its chunk partials (part[chunk][tile][3][64], one 512-B store per
// channel) and reduce_kernel adds them to the sums in chunk order; a launch with one chunk adds them
// directly.  Against the in-order lane-per-pixel kernel only the order of the binary64 additions
// differs (tests/test_gpu_parity.py::test_sample_pool_vs_lane_per_pixel: <= 1e-13 relative, every
// segment and draw count identical).
// RT_PARK (binary64 BVH walk): the path state the walk never reads — the throughput T, depth, the
// sample's segment count, its pixel m, the RNG key and draw count, the lane's segment total — is kept
// in LDS across closest_hit_acc instead of in VGPRs, and the walk's stack is sized to the scene's
// deepest leaf (dynamic LDS), so that the kernel fits RT_BVH_WAVES_PER_SIMD waves per SIMD.
#ifndef RT_PARK
#define RT_PARK 0
#endif
constexpr int kParkDoubles = 3, kParkInts = 6;
template <class R, int ACC>
constexpr bool parks() { return RT_PARK != 0 && sizeof(R) == 8 && uses_stack<ACC>(); }

// RT_DEFER_REGEN = K: a lane whose sample finished waits, without tracing, until K lanes of its wave wait
// (or none traces), and the waiting lanes then start their next samples together: the sample set-up
// (keys, the lens disk's rejection loop, the binary64 camera ray) runs for many lanes at once instead
// of for the few that finish in each iteration (RTOW +4.8 %).  A wave's execution still
// depends only on its items, so the sums stay bit-reproducible; K = 1 is the undeferred loop.
#ifndef RT_DEFER_REGEN
#define RT_DEFER_REGEN 16
#endif
// Scenes with triangles take a higher threshold in every kernel (mesh50k 256 spp, lean tree kernel: K = 8 /
// 16 / 24 / 32 / 40 / 48 / 56: 7,503 / 7,579 / 7,609 / 7,611 / 7,621 / 7,544 / 7,464 Msamples/s,
// interleaved; their walks are long, so fewer, fuller regenerations pay).  One threshold per scene, in
// every kernel, keeps the per-pixel summation order — and so BVH == brute force bit for bit — kernel-
// independent (a wave's schedule depends on its items, its segments and K only).  Re-measured with the exit
// skip (tri_exit_bound), kernel time: K = 24 / 32 / 40 / 48: 60.02 / 59.83 / 60.15 / 59.70 ms; 40 / 48 / 56:
// 59.85 / 59.50 / 60.00 ms (interleaved, two sessions, mesh50k 256 spp): 48.
#ifndef RT_DEFER_REGEN_TRI
#define RT_DEFER_REGEN_TRI 48
#endif
template <class R>
__device__ __forceinline__ int defer_regen(const SceneView<R>& sc) {
    return sc.num_tri_nodes > 0 ? RT_DEFER_REGEN_TRI : RT_DEFER_REGEN;
}

// CANCEL: the launch carries a cancel word (progressive renders, Counters::cancel); the instantiation
// without it holds no polling code (the poll's code alone cost 1.4 % on RTOW)
template <class R, bool COUNT, int ACC, bool CANCEL>
__global__ __launch_bounds__(64, (waves_per_simd<R, ACC>()))
void trace_pool_kernel(const TraceArgs<R> args, double* __restrict__ part, const int tiles, const int chunk) {
    const ImageParams& im = args.im;
    const SceneView<R>& sc = args.sc;
    constexpr bool PARK = parks<R, ACC>();
    BvhStack stk{nullptr, 0};
    double* park_d = nullptr;
    uint32_t* park_i = nullptr;
    if constexpr (PARK) {
        // dynamic LDS: [3 x 64 doubles][6 x 64 dwords][stack_entries x 64 ints]
        extern __shared__ double park_dyn[];
        park_d = park_dyn + threadIdx.x;
        park_i = reinterpret_cast<uint32_t*>(park_dyn + kParkDoubles * 64) + threadIdx.x;
        stk.base = reinterpret_cast<int*>(park_dyn + kParkDoubles * 64) + kParkInts * 64 + threadIdx.x;
        stk.stride = 64;
    } else if constexpr (uses_stack<ACC>()) {
        // per-lane traversal stacks, entry k of lane t at [k * 64 + t]: RT_BVH_STACK (binary64) or
        // sc.stack_entries (binary32: dynamic LDS sized by the launch to the scene's deepest leaf) x 4 B
        if constexpr (sizeof(R) == 8 && !dyn_stack<R, ACC>()) {
            __shared__ int bvh_stack[RT_BVH_STACK * 64];      // measured 1 % faster than the dynamic one
            stk.base = bvh_stack + threadIdx.x;
        } else {
            extern __shared__ int bvh_stack_dyn[];           // binary32 at 5 waves/SIMD: LDS is tight
            stk.base = bvh_stack_dyn + threadIdx.x;
        }
        stk.stride = 64;
    }
    __shared__ double acc[3 * 64];        // per-pixel partial sums of this chunk, [channel][m]
    const int lane = threadIdx.x;
    acc[lane] = 0;
    acc[64 + lane] = 0;
    acc[128 + lane] = 0;
    __syncthreads();
    if constexpr (CANCEL) {
        if (__builtin_amdgcn_readfirstlane((int)cancel_requested(args.c, blockIdx.x))) {
            // the workgroup is one item: it is left untraced (a fused launch's batch then never raises
            // its flag; a per-batch launch's gate reads `aborted`)
            if (lane == 0 && !args.c.batch_count) mark_aborted(args.c);
            return;
        }
    }
    const unsigned item = item_at(im, pool_position(blockIdx.x, gridDim.x), tiles);
    const int tile = item % tiles;
    const ChunkRange cr = chunk_range(im, (int)(item / tiles), chunk);
    const Tile tl = tile_of(im, tile);
    const int vw = tl.vw, nv = tl.nv;
    const int sb = cr.sb, se = cr.se;
    const uint32_t total = (uint32_t)nv * (uint32_t)max(0, se - sb);
    PixelResult res{0, 0, {0, 0, 0}, {0, 0, 0}};
    // the lane's current item: pixel m of the tile = (i, j) with key pkey at crop index q, sample s
    int i = 0, j = 0, s = 0, depth = 0;
    uint32_t m = 0, pkey = 0, isegs = 0;
    size_t q = 0;
    Rng<R> g;
    V3<R> o, d, T;
    auto begin_item = [&](const uint32_t k) {
        uint32_t sr;
        if (nv == 64) { m = k & 63; sr = k >> 6; }
        else { sr = k / (uint32_t)nv; m = k - sr * (uint32_t)nv; }
        const int px = tl.x0 + (int)(m % (uint32_t)vw), py = tl.y0 + (int)(m / (uint32_t)vw);
        const int row = im.y0 + py;
        i = im.x0 + px;
        j = im.height - 1 - row;
        pkey = pixel_key(im.seedm, (uint32_t)row * (uint32_t)im.width + (uint32_t)i);
        q = (size_t)py * im.cw + px;
        s = sb + (int)sr;
        T = mk<R>(1, 1, 1);
        depth = im.max_depth;
        isegs = 0;
        start_sample<R, false, feat_of<ACC>()>(sc, im, i, j, pkey, s, g, o, d);
    };
    uint32_t next = 64;                       // items [0, 64) are dealt to lanes 0..63 up front
    const int defer_k = defer_regen(sc);     // RT_DEFER_REGEN (wave-uniform)
    bool live = (uint32_t)lane < total;
    if (live) begin_item((uint32_t)lane);
    bool waiting = false;                     // the lane's sample is done, its next not yet started
    bool skip_tri = false;
    while (live) {                            // lanes only ever leave this loop, so every live lane
        const uint64_t t0 = RT_TICK();        // has seen every update of `next`
        if (!waiting) {
            if constexpr (PARK) {
                park_d[0] = (double)T.x; park_d[64] = (double)T.y; park_d[128] = (double)T.z;
                park_i[0] = (uint32_t)depth; park_i[64] = isegs; park_i[128] = m;
                park_i[192] = g.key; park_i[256] = g.k; park_i[320] = res.segments;
            }
            const Closest<R> c = closest_hit_acc<R, ACC>(sc, o, d, res.work, stk, skip_tri);
            if constexpr (PARK) {
                // the walk's stack stores may alias these slots as far as the compiler can tell: the
                // values are reloaded, not forwarded, so their registers are free during the walk
                T = mk<R>((R)park_d[0], (R)park_d[64], (R)park_d[128]);
                depth = (int)park_i[0]; isegs = park_i[64]; m = park_i[128];
                g.key = park_i[192]; g.k = park_i[256]; res.segments = park_i[320];
                if (COUNT) q = (size_t)(tl.y0 + (int)(m / (uint32_t)vw)) * im.cw + (tl.x0 + (int)(m % (uint32_t)vw));
            }
            const uint64_t t1 = RT_TICK();
            if (RT_PROFILE) res.cyc[0] += t1 - t0;
            ++res.segments;
            ++isegs;
            V3<R> L;
            waiting = shade_segment<R, feat_of<ACC>()>(sc, c, o, d, T, depth, g, L);
            // the next segment leaves the triangle just hit away from every triangle: no triangle walk
            // (tri_exit_bound, pt_core.h; binary64 only)
            if constexpr (sizeof(R) == 8 && (ACC == ACC_BVH || ACC == ACC_BVH_STACK || ACC == ACC_BVH_STACK_LEAN))
                skip_tri = !waiting && c.kind == HIT_TRI && leaves_tri_hull(sc, c.idx, o, d);
            if (RT_PROFILE) res.cyc[1] += RT_TICK() - t1;
            if (waiting) {
                if (COUNT) {
                    if (args.c.segs) atomicAdd(args.c.segs + q, isegs);
                    if (args.c.draws) atomicAdd(args.c.draws + q, g.k);
                }
                // add the finished sample's radiance to its pixel's partial: non-returning LDS atomics
                // (ds_add_f64), no wait.  Lanes that finish samples of the same pixel in one iteration
                // are combined by the LDS atomic unit in its fixed lane order.
                __hip_atomic_fetch_add(&acc[m], (double)L.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&acc[64 + m], (double)L.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&acc[128 + m], (double)L.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        const uint64_t t2 = RT_TICK();
        const uint64_t need = __ballot(waiting);
        if (need && (__popcll(need) >= defer_k || __ballot(!waiting) == 0)) {
            if (waiting) {
                const uint32_t k = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0));
                live = k < total;
                if (live) begin_item(k);
                waiting = false;
            }
            next += (uint32_t)__popcll(need);
        }
        if (RT_PROFILE) res.cyc[2] += RT_TICK() - t2;
    }
    __syncthreads();
    if (lane < nv) {
        if (part) {
            double* p = part + ((size_t)item * 3) * 64 + lane;           // item = chunk * tiles + tile
            if (args.c.batch_count) {
                store_through(p, acc[lane]);
                store_through(p + 64, acc[64 + lane]);
                store_through(p + 128, acc[128 + lane]);
            } else {
                p[0] = acc[lane];
                p[64] = acc[64 + lane];
                p[128] = acc[128 + lane];
            }
        } else {                                  // the launch's only chunk: this wave owns the pixels
            const size_t qq = (size_t)(tl.y0 + lane / vw) * im.cw + (tl.x0 + lane % vw);
            args.c.sum[3 * qq] += acc[lane];
            args.c.sum[3 * qq + 1] += acc[64 + lane];
            args.c.sum[3 * qq + 2] += acc[128 + lane];
        }
    }
    if (args.c.batch_count) {
        if (im.bands) {
            const int bb = band_of_tile(im, tile);
            item_done(args.c, bb, band_items(im, bb), 1, lane);
        } else {
            item_done(args.c, cr.b, (uint32_t)(im.batch_chunks * tiles), im.batch_ways, lane);
        }
    }
    add_totals<ACC>(args.c, res, lane);
}

// One (tile, chunk) item of the pool in a multi-wave workgroup (trace_pool_lds_kernel): item = chunk *
// tiles + tile, traced exactly as trace_pool_kernel traces its workgroup's item.  acc: the wave's
// 3 x 64 LDS partials (zero on entry, zero again on return); the barriers around them are wave-local.
// (trace_pool_kernel keeps its own copy of this loop: calling this function from it measured -1.6 %
// on RTOW binary64, from a different register allocation.)
template <class R, bool COUNT, int ACC>
__device__ __forceinline__ void pool_item(const TraceArgs<R>& args, double* __restrict__ part, const int tiles,
                                          const int chunk, const unsigned pos, double* acc, BvhStack stk,
                                          PixelResult& res, const int lane, const MatRec<R>* lmats = nullptr) {
    const ImageParams& im = args.im;
    const SceneView<R>& sc = args.sc;
    const unsigned item = item_at(im, pos, tiles);       // pos: the queue's position
    const int tile = item % tiles;
    const ChunkRange cr = chunk_range(im, (int)(item / tiles), chunk);
    const Tile tl = tile_of(im, tile);
    const int vw = tl.vw, nv = tl.nv;
    const int sb = cr.sb, se = cr.se;
    const uint32_t total = (uint32_t)nv * (uint32_t)max(0, se - sb);
    // the lane's current item: pixel m of the tile = (i, j) with key pkey at crop index q, sample s
    int i = 0, j = 0, s = 0, depth = 0;
    uint32_t m = 0, pkey = 0, isegs = 0;
    size_t q = 0;
    Rng<R> g;
    V3<R> o, d, T;
    auto begin_item = [&](const uint32_t k) {
        uint32_t sr;
        if (nv == 64) { m = k & 63; sr = k >> 6; }
        else { sr = k / (uint32_t)nv; m = k - sr * (uint32_t)nv; }
        const int px = tl.x0 + (int)(m % (uint32_t)vw), py = tl.y0 + (int)(m / (uint32_t)vw);
        const int row = im.y0 + py;
        i = im.x0 + px;
        j = im.height - 1 - row;
        pkey = pixel_key(im.seedm, (uint32_t)row * (uint32_t)im.width + (uint32_t)i);
        q = (size_t)py * im.cw + px;
        s = sb + (int)sr;
        T = mk<R>(1, 1, 1);
        depth = im.max_depth;
        isegs = 0;
        start_sample<R, sizeof(R) == 4 || (RT_CAM_RELOAD_LEAN64 != 0 && ACC == ACC_GRID_LDS_LEAN), feat_of<ACC>()>(sc, im, i, j, pkey, s, g, o, d);
    };
    uint32_t next = 64;                       // items [0, 64) are dealt to lanes 0..63 up front
    const int defer_k = defer_regen(sc);     // RT_DEFER_REGEN (wave-uniform)
    bool live = (uint32_t)lane < total;
    if (live) begin_item((uint32_t)lane);
    bool waiting = false;                     // as trace_pool_kernel (RT_DEFER_REGEN)
    int origin = -1;                          // RT_ORIGIN_LEAVE: the sphere the next segment starts on
    while (live) {                            // lanes only ever leave this loop, so every live lane
        const uint64_t t0 = RT_TICK();        // has seen every update of `next`
        if (!waiting) {
            const Closest<R> c = closest_hit_acc<R, ACC>(sc, o, d, res.work, stk, false, origin);
            const uint64_t t1 = RT_TICK();
            if (RT_PROFILE) res.cyc[0] += t1 - t0;
            ++res.segments;
            ++isegs;
            V3<R> L;
            waiting = shade_segment<R, feat_of<ACC>()>(sc, c, o, d, T, depth, g, L, lmats);
            if constexpr (RT_ORIGIN_LEAVE && sizeof(R) == 8 && ACC == ACC_GRID_LDS_LEAN)
                origin = !waiting && c.kind == HIT_SPHERE ? c.idx : -1;
            if (RT_PROFILE) res.cyc[1] += RT_TICK() - t1;
            if (waiting) {
                if (COUNT) {
                    if (args.c.segs) atomicAdd(args.c.segs + q, isegs);
                    if (args.c.draws) atomicAdd(args.c.draws + q, g.k);
                }
                __hip_atomic_fetch_add(&acc[m], (double)L.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&acc[64 + m], (double)L.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&acc[128 + m], (double)L.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        const uint64_t t2 = RT_TICK();
        const uint64_t need = __ballot(waiting);
        if (need && (__popcll(need) >= defer_k || __ballot(!waiting) == 0)) {
            if (waiting) {
                const uint32_t k = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0));
                live = k < total;
                if (live) begin_item(k);
                waiting = false;
            }
            next += (uint32_t)__popcll(need);
        }
        if (RT_PROFILE) res.cyc[2] += RT_TICK() - t2;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < nv) {
        if (part) {
            double* p = part + ((size_t)item * 3) * 64 + lane;           // item = chunk * tiles + tile
            if (args.c.batch_count) {
                store_through(p, acc[lane]);
                store_through(p + 64, acc[64 + lane]);
                store_through(p + 128, acc[128 + lane]);
            } else {
                p[0] = acc[lane];
                p[64] = acc[64 + lane];
                p[128] = acc[128 + lane];
            }
        } else {                                  // the launch's only chunk: this wave owns the pixels
            const size_t qq = (size_t)(tl.y0 + lane / vw) * im.cw + (tl.x0 + lane % vw);
            args.c.sum[3 * qq] += acc[lane];
            args.c.sum[3 * qq + 1] += acc[64 + lane];
            args.c.sum[3 * qq + 2] += acc[128 + lane];
        }
    }
    if (args.c.batch_count) {
        if (im.bands) {
            const int bb = band_of_tile(im, tile);
            item_done(args.c, bb, band_items(im, bb), 1, lane);
        } else {
            item_done(args.c, cr.b, (uint32_t)(im.batch_chunks * tiles), im.batch_ways, lane);
        }
    }
    acc[lane] = 0;                            // the wave's next item starts from zero partials
    acc[64 + lane] = 0;
    acc[128 + lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

#if !RT_ONEWAVE_TU   // the LDS pool kernels, the reduce and the host API: pt_trace.hip's own translation unit
// ---- sample pool with the sphere tree's nodes in LDS (ACC_BVH_SPHERES_LDS) ----
// The walk's divergent node reads (4 x 16 B per lane and step through the vector memory path, which
// is ~0.86 busy on RTOW) become LDS reads: a workgroup of lds_waves() waves copies the
// scene's two-child nodes into LDS once — child boxes (48 B, three 16-B reads at a 48-B stride, which
// spreads a 16-lane group's reads over 16 bank groups) and child references (8 B) in separate arrays —
// and its waves then take (tile, chunk) items from a device-wide queue until it is empty, so the
// workgroup's waves finish together and the copy is paid once per workgroup, not per item.  The items
// are the one-wave kernel's (item = chunk * tiles + tile, same partials layout), and each is traced
// exactly as there, so the sums are bit-identical to it.  The queue is one of kPoolQueues counter
// pairs {next item, waves exited}, held by one launch at a time (acquire_queue / hold_queue, queue_slots.h):
// the last wave to exit sets both back to 0.
// Waves per workgroup: a multiple of 4, so that every workgroup puts the same number of waves on
// each SIMD (10-wave workgroups at 5 waves/SIMD left one SIMD a wave short of the second workgroup:
// one workgroup per CU, RTOW -28 %)
#ifndef RT_LDS_WAVES_F64
#define RT_LDS_WAVES_F64 8        // 2 workgroups per CU at 4 waves/SIMD
#endif
#ifndef RT_LDS_WAVES_F32
#define RT_LDS_WAVES_F32 12       // 2 workgroups per CU at 6 waves/SIMD
#endif
// the grid's LDS kernel (ACC_GRID_LDS) holds no stacks: smaller workgroups, each with its own copy
#ifndef RT_GRID_LDS_WAVES_F64
#define RT_GRID_LDS_WAVES_F64 4   // 5 workgroups per CU at 5 waves/SIMD
#endif
#ifndef RT_GRID_LDS_WAVES_F32
#define RT_GRID_LDS_WAVES_F32 12  // 2 workgroups per CU at 6 waves/SIMD (8: 3 per CU, -0.7 %)
#endif
// the triangle tree's LDS kernel (ACC_BVH_TRI_LDS): one workgroup per CU at 4 waves/SIMD, so that the
// CU's one copy of the top levels is as large as its LDS allows beside the 16 waves' stacks and partials
// (binary32, 5 waves/SIMD: 4-wave workgroups, five copies per CU)
#ifndef RT_TRI_LDS_WAVES_F64
#define RT_TRI_LDS_WAVES_F64 16
#endif
#ifndef RT_TRI_LDS_WAVES_F32
#define RT_TRI_LDS_WAVES_F32 4
#endif
template <class R, int ACC = ACC_BVH_SPHERES_LDS>
constexpr int lds_waves() {
    if constexpr (ACC == ACC_GRID_LDS || ACC == ACC_GRID_LDS_LEAN) return sizeof(R) == 8 ? RT_GRID_LDS_WAVES_F64 : RT_GRID_LDS_WAVES_F32;
    if constexpr (ACC == ACC_BVH_TRI_LDS) return sizeof(R) == 8 ? RT_TRI_LDS_WAVES_F64 : RT_TRI_LDS_WAVES_F32;
    return sizeof(R) == 8 ? RT_LDS_WAVES_F64 : RT_LDS_WAVES_F32;
}
constexpr int kPoolQueues = 1024;
__device__ uint32_t g_pool_queue[2 * kPoolQueues];

// two-child nodes [0, n) into LDS: child boxes at box[3k .. 3k+2], references at kid[k]
__device__ __forceinline__ void copy_wide_lds(const Bvh2Node* src, int n, rt_u4* box, rt_u2* kid, int t, int threads) {
    for (int k = t; k < n; k += threads) {
        const rt_u4* g = reinterpret_cast<const rt_u4*>(src + k);
        const rt_u4 q3 = g[3];
        box[3 * k] = g[0];
        box[3 * k + 1] = g[1];
        box[3 * k + 2] = g[2];
        kid[k] = rt_u2{q3.x, q3.y};
    }
}

// ACC_GRID_LDS: the same workgroups and queue with the uniform grid's cell offsets and records
// (binary64: the 16-B binary32 filters; binary32: the whole 32-B records) in LDS instead of nodes: the
// filter rejections, most of a grid walk's record tests, no longer touch the vector memory path.
template <class R, bool COUNT, int ACC>
__global__ __launch_bounds__((64 * lds_waves<R, ACC>()), (waves_per_simd<R, ACC>()))
void trace_pool_lds_kernel(const TraceArgs<R> args, double* __restrict__ part, const int tiles, const int chunk,
                           const int items, const int qi) {
    constexpr int W = lds_waves<R, ACC>();
    const SceneView<R>& sc = args.sc;
    // dynamic LDS: [child boxes 48 B x n][child references 8 B x n][W stacks of entries x 64 ints], or
    // for the grid [records][cell offsets]
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_dyn[];
    __shared__ double acc_all[W * 3 * 64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    BvhStack stk{nullptr, 0};
    if constexpr (ACC == ACC_GRID_LDS || ACC == ACC_GRID_LDS_LEAN) {
        rt_u4* grec = reinterpret_cast<rt_u4*>(lds_dyn);
        int* gcell = reinterpret_cast<int*>(lds_dyn + grid_lds_rec_bytes(sc));
        copy_grid_lds(sc, grec, gcell, threadIdx.x, 64 * W);
        stk.gcell = gcell;
        stk.grec = grec;
    } else if constexpr (ACC == ACC_BVH_TRI_LDS) {
        // the triangle tree's breadth-first top levels (nodes [0, tri_lds_nodes)): the divergent node
        // reads of a walk's first levels become ds_read_b128s (deeper nodes, leaves and the sphere tree
        // stay in global memory)
        const int n = sc.tri_lds_nodes, entries = min(sc.stack_entries, RT_BVH_STACK);
        rt_u4* box = reinterpret_cast<rt_u4*>(lds_dyn);
        rt_u2* kid = reinterpret_cast<rt_u2*>(lds_dyn + 48 * n);
        int* stacks = reinterpret_cast<int*>(lds_dyn + 56 * n);
        copy_wide_lds(sc.tri_wide, n, box, kid, threadIdx.x, 64 * W);
        stk = BvhStack{stacks + wave * entries * 64 + lane, 64, box, kid};
        stk.ntop = n;
    } else {
        const int n = sc.num_sphere_wide, entries = min(sc.stack_entries, RT_BVH_STACK);
        rt_u4* box = reinterpret_cast<rt_u4*>(lds_dyn);
        rt_u2* kid = reinterpret_cast<rt_u2*>(lds_dyn + 48 * n);
        int* stacks = reinterpret_cast<int*>(lds_dyn + 56 * n);
        copy_wide_lds(sc.sphere_wide, n, box, kid, threadIdx.x, 64 * W);
        stk = BvhStack{stacks + wave * entries * 64 + lane, 64, box, kid};
    }
    double* acc = acc_all + wave * 3 * 64;
    acc[lane] = 0;
    acc[64 + lane] = 0;
    acc[128 + lane] = 0;
    const MatRec<R>* lmats = nullptr;
#if RT_MAT_LDS
    if constexpr (ACC == ACC_GRID_LDS || ACC == ACC_GRID_LDS_LEAN) {   // A/B: the material records after the grid's copy
        MatRec<R>* mm = reinterpret_cast<MatRec<R>*>(lds_dyn + ((grid_lds_bytes(sc) + 15) & ~(size_t)15));
        for (int k = threadIdx.x; k < sc.num_mats; k += 64 * W) mm[k] = sc.mats[k];
        lmats = mm;
    }
#endif
    __syncthreads();
    uint32_t* queue = g_pool_queue + 2 * qi;
    PixelResult res{0, 0, {0, 0, 0}, {0, 0, 0}};
    // no cancel word is read here: a cancel moves this launch's queue past its last item from outside
    // (cancel_pool_launches), and every wave's next take ends its loop
    for (;;) {
        uint32_t it = 0;
        if (lane == 0) it = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        it = (uint32_t)__builtin_amdgcn_readfirstlane((int)it);
        if (it >= (uint32_t)items) break;
        pool_item<R, COUNT, ACC>(args, part, tiles, chunk, it, acc, stk, res, lane, lmats);
    }
    add_totals<ACC>(args.c, res, lane);
    if (lane == 0) {
        const uint32_t e = __hip_atomic_fetch_add(queue + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e == gridDim.x * W - 1) {      // every other wave has made its last queue read
            __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// RT_CAM_RELOAD (pt_path.h start_sample) reads the camera words at offsetof(SceneView, cam_o) of the
// kernel-argument segment (RT_SC_RELOAD, pt_core.h closest_hit_acc, the whole SceneView likewise): that holds only while the LDS pool kernel's first parameter is TraceArgs<R>
// by value (whose first member is the SceneView, static_assert above).  A signature change fails here
// instead of reading the camera from the wrong bytes.
template <class F> struct FirstParam;
template <class A0, class... As> struct FirstParam<void (*)(A0, As...)> { using type = A0; };
static_assert(std::is_same<FirstParam<decltype(&trace_pool_lds_kernel<float, false, ACC_GRID_LDS>)>::type,
                           TraceArgs<float>>::value &&
              std::is_same<FirstParam<decltype(&trace_pool_lds_kernel<float, true, ACC_BVH_SPHERES_LDS>)>::type,
                           TraceArgs<float>>::value &&
              std::is_same<FirstParam<decltype(&trace_pool_lds_kernel<double, false, ACC_GRID_LDS_LEAN>)>::type,
                           TraceArgs<double>>::value &&
              std::is_same<FirstParam<decltype(&trace_pool_kernel<double, false, ACC_BVH_STACK_LEAN, false>)>::type,
                           TraceArgs<double>>::value,
              "the camera and grid reloads need TraceArgs as the LDS pool kernel's first (by-value) argument");

// sum[q] += part[c][tile][.][m] for c = 0 .. chunks-1 in chunk order (binary64); one thread per pixel,
// one one-wave workgroup per tile (its reads of one chunk are 3 x 512 contiguous bytes).  One-wave
// workgroups: while the next batch's trace waves hold the CUs (overlapped batches), a 256-thread
// workgroup waits for four free wave slots on one CU and was measured to take 7.8 ms instead of 0.1.
__global__ __launch_bounds__(64) void reduce_kernel(const ImageParams im, double* __restrict__ sum,
                                                    const double* __restrict__ part, const int tiles,
                                                    const int chunks, const uint32_t* __restrict__ skip,
                                                    const int tile0 = 0) {
    const int tile = tile0 + (int)blockIdx.x, m = threadIdx.x;
    if (tile >= tiles || (skip && *skip)) return;
    const Tile t = tile_of(im, tile);
    if (m >= t.nv) return;
    const size_t q = (size_t)(t.y0 + m / t.vw) * im.cw + (t.x0 + m % t.vw);
    double a0 = sum[3 * q], a1 = sum[3 * q + 1], a2 = sum[3 * q + 2];
    const double* p = part + (size_t)tile * 3 * 64 + m;
    const size_t stride = (size_t)tiles * 3 * 64;
    for (int c = 0; c < chunks; ++c, p += stride) {
        a0 += p[0];
        a1 += p[64];
        a2 += p[128];
    }
    sum[3 * q] = a0; sum[3 * q + 1] = a1; sum[3 * q + 2] = a2;
}

// ReduceGate (pt_launch.h): whether the batch's reduce runs; one lane does the host-memory traffic
__global__ __launch_bounds__(64) void reduce_gate_kernel(const ReduceGate g) {
    if (threadIdx.x != 0) return;
    const uint32_t a = __hip_atomic_load(const_cast<uint32_t*>(g.aborted), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t s = __hip_atomic_load(g.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // a fused batch's flag: the acquire end of item_done's hand-off (the partials the reduce reads)
    const uint32_t f = g.complete ? __hip_atomic_load(g.complete, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) : 1u;
    const uint32_t skip = (a | s) || !f ? 1u : 0u;
    *g.skip = skip;
    if (skip) __hip_atomic_store(g.stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(g.done, g.done_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

bool trace_uses_pool() {
    static const bool v = [] {             // thread-safe initialization (renders on several threads)
        const char* e = getenv("RT_SAMPLE_POOL");
        return !(e && e[0] == '0');
    }();
    return v;
}

// Samples per pool wave: ~2 sqrt(ns) (0.75 sqrt(ns) when the scene has a triangle BVH: its walks
// vary more in length, so shorter waves pay), for spheres doubled (up to ~4 sqrt(ns), <= 128) while
// the launch would have > 400k waves, halved (>= 4) until it has >= 64k waves (4x the chip's 16k wave slots).  Short waves shorten
// the frame's drain tail; long ones shorten each wave's own tail (its last items finish at different
// times) and write fewer chunk partials (each chunk is 24 B per pixel written and read back once).
// Measured (RTOW f64 Msamples/s): 1080p x 512 spp c45 / c90 7477 / 7436; x 256 c32 / c45 /
// c64 7363 / 7386 / 7295; x 128 c24 / c32 / c45 7330 / 7219 / 7156; x 64 c8 / c16 / c32 6720 / 7015 /
// 6947; 4K x 128 c23 / c45 7331 / 7393; mesh50k 256 spp c12 / c16 / c24 / c32 6786 / 6673 / 6687 /
// 6391; Cornell 512^2 x 64 spp (4096 tiles) 4.  RT_POOL_CHUNK overrides (A/B runs).
static int pool_chunk(int ns, int tiles, bool tri_bvh) {
    static const int v = [] {
        const char* e = getenv("RT_POOL_CHUNK");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    if (v) return v;
    int c = std::min(128, std::max(4, (int)((tri_bvh ? 0.75 : 2.0) * std::sqrt((double)ns) + 0.5)));
    const int cmax = tri_bvh ? c : std::min(128, std::max(4, (int)(4.0 * std::sqrt((double)ns) + 0.5)));
    while (c < cmax && (long long)tiles * ((ns + c - 1) / c) > 400000) c = std::min(cmax, c * 2);
    while (c > 4 && (long long)tiles * ((ns + c - 1) / c) < 65536) c = std::max(4, c / 2);
    return c;
}

#endif  // !RT_ONEWAVE_TU

// dynamic LDS of a trace launch: the ordered walk's per-lane stacks (the scene's deepest leaf entries)
template <int ACC, class R>
static size_t stack_lds_bytes(const SceneView<R>& sc) {
    return uses_stack<ACC>() && dyn_stack<R, ACC>() ? (size_t)std::min(sc.stack_entries, RT_BVH_STACK) * 64 * sizeof(int) : 0;
}
// ... of the pool kernel (RT_PARK: the parked path state + the stack, binary64)
template <int ACC, class R>
static size_t pool_lds_bytes(const SceneView<R>& sc) {
    if constexpr (parks<R, ACC>())
        return (size_t)64 * (kParkDoubles * sizeof(double) + kParkInts * 4 + std::min(sc.stack_entries, RT_BVH_STACK) * 4);
    return stack_lds_bytes<ACC>(sc);
}

static int crop_tiles(int cw, int ch) { return ((cw + 7) / 8) * ((ch + 7) / 8); }

// The one-wave pool kernel (trace_pool_kernel) and the lane-per-pixel kernel (trace_kernel) are
// compiled in a translation unit of their own, pt_onewave.hip (this file with RT_ONEWAVE_TU), with
// LLVM's AMDGPU register-pressure trackers (build.py: mesh50k +1.0 %, Cornell +1.4 %; the same flag
// costs the LDS kernels 3.6 %).  Their kernels are instantiated and launched only there.
template <class R, int ACC>
hipError_t launch_onewave_pool(const TraceArgs<R>& a, bool count, double* part, int tiles, int chunks, int chunk,
                               hipStream_t stream);
template <class R, int ACC>
hipError_t launch_lane_kernel(const TraceArgs<R>& a, bool count, hipStream_t stream);

#if RT_ONEWAVE_TU
template <class R, int ACC>
hipError_t launch_onewave_pool(const TraceArgs<R>& a, bool count, double* part, int tiles, int chunks, int chunk,
                               hipStream_t stream) {
    const size_t lds = pool_lds_bytes<ACC>(a.sc);
#define RT_POOL_LAUNCH(C, X) hipLaunchKernelGGL((trace_pool_kernel<R, C, ACC, X>), dim3(tiles * chunks), dim3(64), lds, stream, \
                                             a, part, tiles, chunk)
    if (a.c.cancel) { if (count) RT_POOL_LAUNCH(true, true); else RT_POOL_LAUNCH(false, true); }
    else if (count) RT_POOL_LAUNCH(true, false);
    else RT_POOL_LAUNCH(false, false);
#undef RT_POOL_LAUNCH
    return hipGetLastError();
}
template <class R, int ACC>
hipError_t launch_lane_kernel(const TraceArgs<R>& a, bool count, hipStream_t stream) {
    const int tiles = crop_tiles(a.im.cw, a.im.ch);
    const size_t lds = stack_lds_bytes<ACC>(a.sc);
    if (count) hipLaunchKernelGGL((trace_kernel<R, true, ACC>), dim3(tiles), dim3(64), lds, stream, a);
    else hipLaunchKernelGGL((trace_kernel<R, false, ACC>), dim3(tiles), dim3(64), lds, stream, a);
    return hipGetLastError();
}
#define RT_ONEWAVE_INST(R, ACC)                                                                                  \
    template hipError_t launch_onewave_pool<R, ACC>(const TraceArgs<R>&, bool, double*, int, int, int, hipStream_t); \
    template hipError_t launch_lane_kernel<R, ACC>(const TraceArgs<R>&, bool, hipStream_t);
RT_ONEWAVE_INST(double, ACC_BRUTE)
RT_ONEWAVE_INST(double, ACC_BVH)
RT_ONEWAVE_INST(double, ACC_BVH_STACK)
RT_ONEWAVE_INST(double, ACC_BVH_SPHERES)
RT_ONEWAVE_INST(double, ACC_GRID)
RT_ONEWAVE_INST(double, ACC_BVH_STACK_LEAN)
RT_ONEWAVE_INST(double, ACC_BRUTE_LEAN)
RT_ONEWAVE_INST(float, ACC_BRUTE)
RT_ONEWAVE_INST(float, ACC_BVH)
RT_ONEWAVE_INST(float, ACC_BVH_STACK)
RT_ONEWAVE_INST(float, ACC_BVH_SPHERES)
RT_ONEWAVE_INST(float, ACC_GRID)
RT_ONEWAVE_INST(float, ACC_BVH_STACK_LEAN)
RT_ONEWAVE_INST(float, ACC_BRUTE_LEAN)
#undef RT_ONEWAVE_INST
#else   // !RT_ONEWAVE_TU: the rest of the file

size_t pool_partial_bytes(int cw, int ch, int ns, bool tri_bvh, int chunk_override) {
    if (cw <= 0 || ch <= 0 || ns <= 0) return 0;
    const int tiles = crop_tiles(cw, ch), chunk = chunk_override > 0 ? chunk_override : pool_chunk(ns, tiles, tri_bvh);
    const size_t chunks = (size_t)((ns + chunk - 1) / chunk);
    return chunks > 1 ? chunks * tiles * kPartialBytesPerTile : 0;
}

// Which sphere-only launches read the nodes from LDS: binary32 (RTOW 256 spp, 6 waves/SIMD: 9752 vs
// 9504 Msamples/s); binary64 only when asked (RT_LDS_NODES=2): RTOW's 481 nodes (27 KB) + 5 workgroups'
// stacks and partials exceed 160 KiB at 5 waves/SIMD, and at 4 the LDS kernel (7497) is slower than the
// one-wave kernel at 5 (7744; at 4: 7291).  RT_LDS_NODES=0: never (A/B).
#ifndef RT_LDS_NODES
#define RT_LDS_NODES 1
#endif
// Which grid launches read the grid from LDS (trace_pool_lds_kernel<.., ACC_GRID_LDS>): RT_LDS_GRID=0
// never (A/B), 1 (default) whenever the copy fits
#ifndef RT_LDS_GRID
#define RT_LDS_GRID 1
#endif
// RT_MAT_LDS (A/B): the grid LDS kernel also stages the material records in LDS (the budget check then
// counts them: fewer workgroups per CU when they do not fit beside the grid)
#ifndef RT_MAT_LDS
#define RT_MAT_LDS 0
#endif
template <class R>
static size_t lds_grid_bytes(const SceneView<R>& sc) {
    static const int v = [] {
        const char* e = getenv("RT_LDS_GRID");
        return e ? atoi(e) : RT_LDS_GRID;
    }();
    if (v < 1 || sc.num_grid_cells <= 0) return 0;
    constexpr int W = lds_waves<R, ACC_GRID_LDS>();
    const size_t b = ((grid_lds_bytes(sc) + 15) & ~(size_t)15) + (RT_MAT_LDS ? sizeof(MatRec<R>) * (size_t)sc.num_mats : 0);
    // RT_MAT_LDS: one workgroup per CU fewer (4 instead of 5 binary64 grid workgroups)
    const size_t budget = 160 * 1024 / (4 * waves_per_simd<R, ACC_GRID_LDS>() / W - (RT_MAT_LDS ? 1 : 0));
    return b + (size_t)W * 3 * 64 * 8 + 256 <= budget ? b : 0;
}

// LDS of trace_pool_lds_kernel (dynamic part), 0 if not used for this scene or if its sphere tree does
// not fit: the kernel's workgroups per CU share its 160 KiB
template <class R>
static size_t lds_nodes_bytes(const SceneView<R>& sc) {
    static const int v = [] {
        const char* e = getenv("RT_LDS_NODES");
        return e ? atoi(e) : RT_LDS_NODES;
    }();
    if (v < (sizeof(R) == 8 ? 2 : 1) || sc.num_sphere_wide <= 0) return 0;
    constexpr int W = lds_waves<R>();
    const size_t b = (size_t)56 * sc.num_sphere_wide + (size_t)W * std::min(sc.stack_entries, RT_BVH_STACK) * 64 * 4;
    const size_t budget = 160 * 1024 / (4 * waves_per_simd<R, ACC_BVH_SPHERES_LDS>() / W);
    return b + (size_t)W * 3 * 64 * 8 + 256 <= budget ? b : 0;
}

// Which launches of scenes with a triangle tree run trace_pool_lds_kernel<.., ACC_BVH_TRI_LDS> (the top
// levels of the triangle tree in LDS): RT_LDS_TRI = 0 (default) never, 1 binary64, 2 both precisions.
// Measured (round 6, mesh50k 1080p x 128 spp f64, interleaved x2, identical images): the one-wave kernel
// 6915 / 6845 Msamples/s; the persistent kernel with 1019 / 255 / 64 top nodes in LDS 6360-6369 /
// 6319-6323 / 6238-6272, in 8-wave workgroups (507 nodes, two copies per CU) 6283-6336: the LDS nodes buy
// +1.8 % over the same kernel without them, the persistent form loses 9 % against hardware-dispatched
// one-wave workgroups (round 5's persistent one-wave kernel with per-XCD queues: -10 %) — DESIGN.md §4
#ifndef RT_LDS_TRI
#define RT_LDS_TRI 0
#endif
// the triangle-tree nodes a launch stages (0: the one-wave kernel): as many of the breadth-first prefix
// (RT_TRI_TOP_NODES, or RT_TRI_LDS_NODES from the environment for A/B runs) as fit the CU's LDS beside
// the workgroups' stacks and partials, at least 64
template <class R>
static int lds_tri_nodes(const SceneView<R>& sc) {
    static const int v = [] {
        const char* e = getenv("RT_LDS_TRI");
        return e ? atoi(e) : RT_LDS_TRI;
    }();
    static const int cap = [] {
        const char* e = getenv("RT_TRI_LDS_NODES");
        return e ? std::max(0, std::min(atoi(e), RT_TRI_TOP_NODES)) : RT_TRI_TOP_NODES;
    }();
    if (v < (sizeof(R) == 8 ? 1 : 2) || sc.num_tri_wide <= 0) return 0;
    constexpr int W = lds_waves<R, ACC_BVH_TRI_LDS>();
    const long long budget = 160 * 1024 / (4 * waves_per_simd<R, ACC_BVH_TRI_LDS>() / W);
    const long long fixed = (long long)W * std::min(sc.stack_entries, RT_BVH_STACK) * 64 * 4 + (long long)W * 3 * 64 * 8 + 256;
    const long long n = std::min<long long>({(long long)sc.num_tri_wide, (long long)cap, (budget - fixed) / 56});
    return n >= 64 ? (int)n : 0;
}
template <class R>
static size_t lds_tri_bytes(const SceneView<R>& sc, int nodes) {
    return (size_t)56 * nodes + (size_t)lds_waves<R, ACC_BVH_TRI_LDS>() * std::min(sc.stack_entries, RT_BVH_STACK) * 64 * 4;
}

// ---- ownership of the LDS pool launches' queues (queue_slots.h) ----
// Per device, kPoolQueues counter pairs (g_pool_queue, device memory); a launch holds its pair from
// acquire_queue() until the pair's event — recorded on the launch's stream after the launch
// (hold_queue), and again after a cancel's clear kernel — has completed.  Launches in flight together
// (streams, scenes, precisions, threads) therefore never share a pair.  Every call is under
// g_launch_mu, which also makes cancel_pool_launches' check (the launch still holds its pair) and act
// (the move, the clear, the later release) one step.
namespace {
std::mutex g_launch_mu;
QueueSlots<hipEvent_t>* g_slots[64];      // per device, created on first use (under g_launch_mu)

QueueSlots<hipEvent_t>& device_slots(int dev) {
    QueueSlots<hipEvent_t>*& s = g_slots[dev & 63];
    if (!s) s = new QueueSlots<hipEvent_t>(kPoolQueues);   // lives as long as the process
    return *s;
}
// a slot's release event has completed (never recorded: complete; a device error: nothing will
// complete later either, the launch that failed reports it)
bool release_done(hipEvent_t ev) {
    if (!ev) return true;
    const hipError_t q = hipEventQuery(ev);
    if (q == hipErrorNotReady) return false;
    if (q != hipSuccess) (void)hipGetLastError();
    return true;
}
}  // namespace

// a queue pair of the current device for one LDS launch: waits (20-us sleeps) while every pair is held,
// which takes kPoolQueues launches in flight on one device
static hipError_t acquire_queue(int* dev, int* qi) {
    hipError_t e = hipGetDevice(dev);
    if (e != hipSuccess) return e;
    for (;;) {
        {
            std::lock_guard<std::mutex> g(g_launch_mu);
            QueueSlots<hipEvent_t>& s = device_slots(*dev);
            const int k = s.acquire(release_done);
            if (k >= 0) {
                if (!s.token(k)) e = hipEventCreateWithFlags(&s.token(k), hipEventDisableTiming);
                if (e != hipSuccess) {
                    s.token(k) = nullptr;
                    s.abandon(k);
                    return e;
                }
                *qi = k;
                return hipSuccess;
            }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}
// after the launch on `stream` (launched: false when it failed to enqueue): the pair is held until the
// launch has ended
static hipError_t hold_queue(int dev, int qi, hipStream_t stream, bool launched) {
    std::lock_guard<std::mutex> g(g_launch_mu);
    QueueSlots<hipEvent_t>& s = device_slots(dev);
    if (!launched) {
        s.abandon(qi);
        return hipSuccess;
    }
    const hipError_t e = hipEventRecord(s.token(qi), stream);
    if (e != hipSuccess) {
        // not recorded: the event's last record (complete, or never recorded) would free the pair
        // while the launch may run, so the pair is waited for here instead
        (void)hipStreamSynchronize(stream);
        s.abandon(qi);
        return e;
    }
    s.hold(qi, s.token(qi));
    return hipSuccess;
}

// ---- cancelling LDS pool launches in flight (pt_launch.h: cancel_pool_launches) ----
// The queue of launch qi moved to `items`: takes from then on return >= items.  aborted is stored first
// (system scope, before the move's release), so the batch's gate, which runs after the launch ends and
// so after a wave has taken a moved position, reads it set.
__global__ __launch_bounds__(64) void queue_cancel_kernel(const int qi, const uint32_t items, uint32_t* aborted) {
    if (threadIdx.x != 0) return;
    if (aborted) __hip_atomic_store(aborted, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
    __hip_atomic_fetch_max(g_pool_queue + 2 * qi, items, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a render's device-memory cancel word (Counters::cancel_dev): every copy := gen
__global__ __launch_bounds__(64) void cancel_word_kernel(uint32_t* word, const uint32_t gen) {
    if (threadIdx.x < kDevCancelCopies)
        __hip_atomic_store(word + threadIdx.x * kCancelStride, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// after the launch (and the move) ended: the queue pair back to 0 for its next holder
__global__ __launch_bounds__(64) void queue_clear_kernel(const int qi) {
    if (threadIdx.x < 2) __hip_atomic_store(g_pool_queue + 2 * qi + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

namespace {
struct PoolLaunch {
    const uint32_t* cancel;
    uint32_t* aborted;
    int device, qi;
    unsigned gen;                         // the pair's generation (QueueSlots::generation) for this launch
    uint32_t items;
    hipStream_t stream;
};
std::vector<PoolLaunch> g_launches;       // launches that may still run (pruned as they are found done)
hipStream_t g_cancel_stream[64];          // per device, created on first use (under g_launch_mu)
struct CancelWord {
    const uint32_t* cancel;
    int device;
    uint32_t* word;
    uint32_t gen;
};
std::vector<CancelWord> g_words;          // registered device cancel words (until forget_pool_launches)

hipError_t cancel_stream(int device, hipStream_t* out) {   // under g_launch_mu, device current
    hipStream_t& cs = g_cancel_stream[device & 63];
    hipError_t e = hipSuccess;
    if (!cs) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        e = hipStreamCreateWithPriority(&cs, hipStreamNonBlocking, hi);
    }
    *out = cs;
    return e;
}

// drop the records for which keep() is false
template <class F>
void prune_launches(F keep) {
    size_t w = 0;
    for (size_t k = 0; k < g_launches.size(); ++k)
        if (keep(g_launches[k])) g_launches[w++] = g_launches[k];
    g_launches.resize(w);
}
// the launch has ended: its pair's release event completed (then the pair may have been handed to
// another launch since, which the generation shows).  Under g_launch_mu.
bool launch_done(const PoolLaunch& l) {
    QueueSlots<hipEvent_t>& s = device_slots(l.device);
    return s.generation(l.qi) != l.gen || !s.held(l.qi) || release_done(s.token(l.qi));
}
}  // namespace

// after the launch was enqueued (and its pair held, hold_queue) on `stream` of device `dev`.  Records
// whose launch has ended are dropped here and in cancel_pool_launches: a record is only acted on while
// its launch still holds its pair (checked under the lock that hands pairs out)
static hipError_t register_pool_launch(const Counters& c, int dev, int qi, uint32_t items, hipStream_t stream) {
    std::lock_guard<std::mutex> g(g_launch_mu);
    prune_launches([](const PoolLaunch& l) { return !launch_done(l); });
    g_launches.push_back(PoolLaunch{c.cancel, c.aborted, dev, qi, device_slots(dev).generation(qi), items, stream});
    return hipSuccess;
}

hipError_t cancel_pool_launches(const uint32_t* cancel) {
    if (!cancel) return hipSuccess;
    std::lock_guard<std::mutex> g(g_launch_mu);
    int cur = -1;
    hipError_t err = hipSuccess;
    prune_launches([&](const PoolLaunch& l) {
        if (l.cancel != cancel) return !launch_done(l);
        if (launch_done(l)) return false;
        if (cur < 0 && hipGetDevice(&cur) != hipSuccess) cur = 0;
        hipError_t e = hipSetDevice(l.device);
        hipStream_t cs = nullptr;
        if (e == hipSuccess) e = cancel_stream(l.device, &cs);
        hipEvent_t ev = nullptr;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(queue_cancel_kernel, dim3(1), dim3(64), 0, cs, l.qi, l.items, l.aborted);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ev, cs);
        if (e == hipSuccess) e = hipStreamWaitEvent(l.stream, ev, 0);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(queue_clear_kernel, dim3(1), dim3(64), 0, l.stream, l.qi);
            e = hipGetLastError();
        }
        // the pair stays held until the clear has run (it waits for the move): no other launch can take
        // it while the move may still land on it
        QueueSlots<hipEvent_t>& slots = device_slots(l.device);
        if (e == hipSuccess) e = hipEventRecord(slots.token(l.qi), l.stream);
        if (e == hipSuccess) slots.extend(l.qi, slots.token(l.qi));
        else (void)hipStreamSynchronize(l.stream);   // not recorded: the pair is released only once idle
        if (ev) (void)hipEventDestroy(ev);
        if (e != hipSuccess && err == hipSuccess) err = e;
        return false;                     // cancelled: the record goes
    });
    for (const CancelWord& w : g_words) { // the one-wave kernels' device words
        if (w.cancel != cancel) continue;
        if (cur < 0 && hipGetDevice(&cur) != hipSuccess) cur = 0;
        hipError_t e = hipSetDevice(w.device);
        hipStream_t cs = nullptr;
        if (e == hipSuccess) e = cancel_stream(w.device, &cs);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(cancel_word_kernel, dim3(1), dim3(64), 0, cs, w.word, w.gen);
            e = hipGetLastError();
        }
        if (e != hipSuccess && err == hipSuccess) err = e;
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    return err;
}

void forget_pool_launches(const uint32_t* cancel) {
    std::lock_guard<std::mutex> g(g_launch_mu);
    prune_launches([&](const PoolLaunch& l) { return l.cancel != cancel && !launch_done(l); });
    size_t w = 0;
    for (size_t k = 0; k < g_words.size(); ++k)
        if (g_words[k].cancel != cancel) g_words[w++] = g_words[k];
    g_words.resize(w);
}

void register_cancel_word(const uint32_t* cancel, int device, uint32_t* word, uint32_t gen) {
    std::lock_guard<std::mutex> g(g_launch_mu);
    g_words.push_back(CancelWord{cancel, device, word, gen});
    // the device's cancel stream now, not in the first cancel (its creation took ~7 ms there)
    if (!g_cancel_stream[device & 63]) {
        int cur = 0;
        hipStream_t cs = nullptr;
        if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(device) == hipSuccess) {
            (void)cancel_stream(device, &cs);
            (void)hipSetDevice(cur);
        }
    }
}

static int device_cus() {
    static std::atomic<int> cus[64];       // 0: not yet read (racing readers store the same value)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = cus[dev].load(std::memory_order_relaxed);
    if (!n) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

// one trace_pool_lds_kernel launch with its own work queue (lb: its dynamic LDS)
template <class R, int LACC>
static hipError_t launch_lds_pool(const TraceArgs<R>& a, bool count, double* part, int tiles, int chunks, int chunk,
                                  size_t lb, hipStream_t stream) {
    int dev = 0, qi = 0;
    if (const hipError_t e = acquire_queue(&dev, &qi)) return e;
    const long long items = (long long)tiles * chunks;
    constexpr int W = lds_waves<R, LACC>();
    const int resident = device_cus() * 4 * waves_per_simd<R, LACC>() / W;
    const int grid = (int)std::min<long long>(resident, (items + W - 1) / W);
    if (count) hipLaunchKernelGGL((trace_pool_lds_kernel<R, true, LACC>), dim3(grid), dim3(64 * W), lb, stream,
                                  a, part, tiles, chunk, (int)items, qi);
    else hipLaunchKernelGGL((trace_pool_lds_kernel<R, false, LACC>), dim3(grid), dim3(64 * W), lb, stream,
                            a, part, tiles, chunk, (int)items, qi);
    const hipError_t e = hipGetLastError();
    const hipError_t eh = hold_queue(dev, qi, stream, e == hipSuccess);
    if (e != hipSuccess) return e;
    if (eh != hipSuccess) return eh;
    if (!a.c.cancel) return hipSuccess;
    return register_pool_launch(a.c, dev, qi, (uint32_t)items, stream);
}

// The lean kernels (feat_of, pt_core.h) serve launches whose scene has the sky gradient, the perspective
// camera and supersampling AA, and the lean kernel's primitives: the grid's (ACC_GRID_LDS_LEAN) spheres
// alone, the triangle BVH walk's (ACC_BVH_STACK_LEAN) and World order's (ACC_BRUTE_LEAN) no boxes (World
// order: no triangles either).  RT_LEAN=0: never (A/B); 1 (default): all three; 2: the grid's only
#ifndef RT_LEAN
#define RT_LEAN 1
#endif
template <class R>
static bool scene_lean(const SceneView<R>& sc, const ImageParams& im, int feat) {
    static const int v = [] {
        const char* e = getenv("RT_LEAN");
        return e ? atoi(e) : RT_LEAN;
    }();
    if (v == 0 || (v == 2 && feat != 0)) return false;
    return (sc.num_planes == 0 || (feat & F_PLANES)) && (sc.num_boxes == 0 || (feat & F_BOXES)) &&
           (sc.num_tri_nodes == 0 || (feat & F_TRIS)) && sc.background == 0 && !sc.cam_ortho && im.aa_mode == 0;
}

template <class R, int ACC>
static hipError_t launch_pool_kernel(const TraceArgs<R>& a0, bool count, double* part, int tiles, int chunks,
                                     int chunk, hipStream_t stream) {
    if constexpr (ACC == ACC_BRUTE) {
        if (scene_lean(a0.sc, a0.im, feat_of<ACC_BRUTE_LEAN>()))
            return launch_onewave_pool<R, ACC_BRUTE_LEAN>(a0, count, part, tiles, chunks, chunk, stream);
    } else if constexpr (ACC == ACC_GRID) {
        if (const size_t lb = lds_grid_bytes(a0.sc)) {
            if (scene_lean(a0.sc, a0.im, feat_of<ACC_GRID_LDS_LEAN>()))
                return launch_lds_pool<R, ACC_GRID_LDS_LEAN>(a0, count, part, tiles, chunks, chunk, lb, stream);
            return launch_lds_pool<R, ACC_GRID_LDS>(a0, count, part, tiles, chunks, chunk, lb, stream);
        }
    } else if constexpr (ACC == ACC_BVH_SPHERES) {
        if (const size_t lb = lds_nodes_bytes(a0.sc))
            return launch_lds_pool<R, ACC_BVH_SPHERES_LDS>(a0, count, part, tiles, chunks, chunk, lb, stream);
    } else if constexpr (ACC == ACC_BVH_STACK) {
        TraceArgs<R> a = a0;
        a.sc.tri_lds_nodes = lds_tri_nodes(a.sc);
        if (a.sc.tri_lds_nodes)
            return launch_lds_pool<R, ACC_BVH_TRI_LDS>(a, count, part, tiles, chunks, chunk,
                                                       lds_tri_bytes(a.sc, a.sc.tri_lds_nodes), stream);
        if (scene_lean(a0.sc, a0.im, feat_of<ACC_BVH_STACK_LEAN>()))
            return launch_onewave_pool<R, ACC_BVH_STACK_LEAN>(a0, count, part, tiles, chunks, chunk, stream);
    }
    return launch_onewave_pool<R, ACC>(a0, count, part, tiles, chunks, chunk, stream);
}

template <class R, int ACC>
static hipError_t launch_pool(const TraceArgs<R>& a0, bool count, hipStream_t stream) {
    const ImageParams& im = a0.im;
    const int ns_all = im.s_end - im.s_begin;
    // the chunk choice depends on the scene, not on the walk, so BVH and brute force add the samples
    // in the same order (bit-identical sums)
    const bool tri_bvh = a0.sc.num_tri_nodes > 0;
    const int tiles = crop_tiles(im.cw, im.ch), chunk = im.pool_chunk > 0 ? im.pool_chunk : pool_chunk(ns_all, tiles, tri_bvh);
    const int chunks_all = (ns_all + chunk - 1) / chunk;
    // chunk partials that fit the scratch buffer; a frame that needs more is split into launches
    const size_t per_chunk = (size_t)tiles * kPartialBytesPerTile;
    int chunks_fit = chunks_all;
    if (chunks_all > 1) {
        chunks_fit = (int)std::min<size_t>((size_t)chunks_all, a0.c.part ? a0.c.part_bytes / per_chunk : 0);
        if (chunks_fit < 1) return hipErrorInvalidValue;
    }
    const int ns_max = chunks_fit * chunk;
    for (int b = im.s_begin; b < im.s_end; b += ns_max) {
        TraceArgs<R> a = a0;
        a.im.s_begin = b;
        a.im.s_end = std::min(im.s_end, b + ns_max);
        const int ns = a.im.s_end - b, chunks = (ns + chunk - 1) / chunk;
        if ((long long)tiles * chunks > 0x7FFFFFFFLL) return hipErrorInvalidConfiguration;
        double* part = chunks > 1 ? a0.c.part : nullptr;
        if (const hipError_t e = launch_pool_kernel<R, ACC>(a, count, part, tiles, chunks, chunk, stream)) return e;
        if (part)
            hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)tiles), dim3(64), 0, stream, a.im, a.c.sum,
                               (const double*)part, tiles, chunks, (const uint32_t*)nullptr);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// RT_BVH_WALK=skip (A/B runs): the stackless preorder walk; default: the ordered two-child walk, in its
// sphere-only form for scenes without triangles (RT_BVH_WALK=two: always the general form)
template <class R>
static int bvh_walk_mode(const SceneView<R>& sc) {
    static const int v = [] {
        const char* e = getenv("RT_BVH_WALK");
        // A/B: skip = stackless walk, two = the general ordered walk, tree = the sphere tree even where
        // the grid was chosen, grid = the grid wherever one was built
        return e && !strncmp(e, "skip", 4) ? ACC_BVH : e && !strncmp(e, "two", 3) ? ACC_BVH_STACK
             : e && !strncmp(e, "grid", 4) ? ACC_GRID : e && !strncmp(e, "tree", 4) ? -2 : ACC_BVH_SPHERES;
    }();
    if (sc.num_tri_nodes > 0) return v == ACC_BVH ? ACC_BVH : ACC_BVH_STACK;
    const bool grid = sc.num_grid_cells > 0 && (v == ACC_GRID || (v == ACC_BVH_SPHERES && sc.use_grid));
    return grid ? ACC_GRID : v == -2 || v == ACC_GRID ? ACC_BVH_SPHERES : v;
}

template <class R>
bool trace_walks_grid(const SceneView<R>& sc) { return bvh_walk_mode(sc) == ACC_GRID; }
template bool trace_walks_grid<double>(const SceneView<double>&);
template bool trace_walks_grid<float>(const SceneView<float>&);

template <class R, int ACC>
static hipError_t launch_acc(const TraceArgs<R>& a, bool count, bool pool, hipStream_t stream) {
    if (pool) return launch_pool<R, ACC>(a, count, stream);
    return launch_lane_kernel<R, ACC>(a, count, stream);
}

template <class R>
hipError_t launch_trace(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh, bool pool,
                        hipStream_t stream) {
    if (im.cw <= 0 || im.ch <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    TraceArgs<R> a{sc, im, c};
    const bool count = c.segs || c.draws;
    if (!bvh) return launch_acc<R, ACC_BRUTE>(a, count, pool, stream);
    const int mode = bvh_walk_mode(sc);
    if (mode == ACC_BVH) return launch_acc<R, ACC_BVH>(a, count, pool, stream);
    if (mode == ACC_BVH_SPHERES) return launch_acc<R, ACC_BVH_SPHERES>(a, count, pool, stream);
    if (mode == ACC_GRID) return launch_acc<R, ACC_GRID>(a, count, pool, stream);
    return launch_acc<R, ACC_BVH_STACK>(a, count, pool, stream);
}

template hipError_t launch_trace<double>(const SceneView<double>&, const ImageParams&, const Counters&, bool, bool, hipStream_t);
template hipError_t launch_trace<float>(const SceneView<float>&, const ImageParams&, const Counters&, bool, bool, hipStream_t);

PoolPlan pool_plan(int cw, int ch, int ns, bool tri_bvh, int chunk) {
    PoolPlan p{0, 0, 0, 0};
    if (cw <= 0 || ch <= 0 || ns <= 0) return p;
    p.tiles = crop_tiles(cw, ch);
    p.chunk = chunk > 0 ? chunk : pool_chunk(ns, p.tiles, tri_bvh);
    p.chunks = (ns + p.chunk - 1) / p.chunk;
    p.part_bytes = (size_t)p.chunks * p.tiles * kPartialBytesPerTile;
    return p;
}

// The pool kernel alone, every chunk (even a single one) into `part`: the sums are not touched, so
// several such launches (batches) may run at once on different streams; launch_reduce adds them.
template <class R, int ACC>
static hipError_t launch_partials_acc(const TraceArgs<R>& a, bool count, const PoolPlan& p, double* part,
                                      hipStream_t stream) {
    if ((long long)p.tiles * p.chunks > 0x7FFFFFFFLL) return hipErrorInvalidConfiguration;
    return launch_pool_kernel<R, ACC>(a, count, part, p.tiles, p.chunks, p.chunk, stream);
}

template <class R>
hipError_t launch_trace_partials(const SceneView<R>& sc, const ImageParams& im, const Counters& c, bool bvh,
                                 double* part, size_t part_bytes, hipStream_t stream) {
    if (im.cw <= 0 || im.ch <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    const PoolPlan p = pool_plan(im.cw, im.ch, im.s_end - im.s_begin, sc.num_tri_nodes > 0, im.pool_chunk);
    if (!part || part_bytes < p.part_bytes) return hipErrorInvalidValue;
    TraceArgs<R> a{sc, im, c};
    const bool count = c.segs || c.draws;
    if (!bvh) return launch_partials_acc<R, ACC_BRUTE>(a, count, p, part, stream);
    const int mode = bvh_walk_mode(sc);
    if (mode == ACC_BVH) return launch_partials_acc<R, ACC_BVH>(a, count, p, part, stream);
    if (mode == ACC_BVH_SPHERES) return launch_partials_acc<R, ACC_BVH_SPHERES>(a, count, p, part, stream);
    if (mode == ACC_GRID) return launch_partials_acc<R, ACC_GRID>(a, count, p, part, stream);
    return launch_partials_acc<R, ACC_BVH_STACK>(a, count, p, part, stream);
}

template hipError_t launch_trace_partials<double>(const SceneView<double>&, const ImageParams&, const Counters&, bool,
                                                  double*, size_t, hipStream_t);
template hipError_t launch_trace_partials<float>(const SceneView<float>&, const ImageParams&, const Counters&, bool,
                                                 double*, size_t, hipStream_t);

size_t fused_batch_doubles(int cw, int ch, int batch, bool tri_bvh, int chunk) {
    return pool_plan(cw, ch, batch, tri_bvh, chunk).part_bytes / sizeof(double);
}
uint32_t fused_batch_items(int cw, int ch, int batch, bool tri_bvh, int chunk) {
    const PoolPlan p = pool_plan(cw, ch, batch, tri_bvh, chunk);
    return (uint32_t)((size_t)p.tiles * p.chunks);
}

template <class R>
hipError_t launch_trace_batches(const SceneView<R>& sc, const ImageParams& im0, const Counters& c, bool bvh, int batch,
                                double* part, size_t part_bytes, hipStream_t stream) {
    if (im0.cw <= 0 || im0.ch <= 0 || im0.s_end <= im0.s_begin || batch <= 0) return hipSuccess;
    const bool tri = sc.num_tri_nodes > 0;
    const PoolPlan p = pool_plan(im0.cw, im0.ch, batch, tri, im0.pool_chunk);   // one batch's chunks
    const int stride = batch * (im0.batch_ways > 1 ? im0.batch_ways : 1);
    const int nb = (im0.s_end - im0.s_begin + stride - 1) / stride;
    if (!part || !c.batch_count || !c.batch_flag || part_bytes < (size_t)nb * p.part_bytes) return hipErrorInvalidValue;
    if ((long long)p.tiles * p.chunks * nb > 0x7FFFFFFFLL) return hipErrorInvalidConfiguration;
    ImageParams im = im0;
    im.pool_chunk = p.chunk;
    im.batch_samples = batch;
    im.batch_chunks = p.chunks;
    const PoolPlan all{p.tiles, p.chunk, p.chunks * nb, (size_t)nb * p.part_bytes};
    TraceArgs<R> a{sc, im, c};
    const bool count = c.segs || c.draws;
    if (!bvh) return launch_partials_acc<R, ACC_BRUTE>(a, count, all, part, stream);
    const int mode = bvh_walk_mode(sc);
    if (mode == ACC_BVH) return launch_partials_acc<R, ACC_BVH>(a, count, all, part, stream);
    if (mode == ACC_BVH_SPHERES) return launch_partials_acc<R, ACC_BVH_SPHERES>(a, count, all, part, stream);
    if (mode == ACC_GRID) return launch_partials_acc<R, ACC_GRID>(a, count, all, part, stream);
    return launch_partials_acc<R, ACC_BVH_STACK>(a, count, all, part, stream);
}

template hipError_t launch_trace_batches<double>(const SceneView<double>&, const ImageParams&, const Counters&, bool, int,
                                                 double*, size_t, hipStream_t);
template hipError_t launch_trace_batches<float>(const SceneView<float>&, const ImageParams&, const Counters&, bool, int,
                                                double*, size_t, hipStream_t);

// the partials of tiles [tile0, tile0 + ntiles) of a banded launch (launch_trace_bands)
hipError_t launch_reduce_tiles(const ImageParams& im, double* sum, const double* part, int tiles, int chunks,
                               int tile0, int ntiles, hipStream_t stream, const ReduceGate* gate) {
    if (ntiles <= 0) return hipSuccess;
    if (gate) hipLaunchKernelGGL(reduce_gate_kernel, dim3(1), dim3(64), 0, stream, *gate);
    hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)ntiles), dim3(64), 0, stream, im, sum, part, tiles, chunks,
                       (const uint32_t*)(gate ? gate->skip : nullptr), tile0);
    return hipGetLastError();
}

template <class R>
hipError_t launch_trace_bands(const SceneView<R>& sc, const ImageParams& im0, const Counters& c, bool bvh, int bands,
                              double* part, size_t part_bytes, PoolPlan* plan, hipStream_t stream) {
    if (im0.cw <= 0 || im0.ch <= 0 || im0.s_end <= im0.s_begin || bands <= 0) return hipSuccess;
    const PoolPlan p = pool_plan(im0.cw, im0.ch, im0.s_end - im0.s_begin, sc.num_tri_nodes > 0, im0.pool_chunk);
    if (plan) *plan = p;
    if (!part || !c.batch_count || !c.batch_flag || part_bytes < p.part_bytes || bands > (im0.ch + 7) / 8)
        return hipErrorInvalidValue;
    if ((long long)p.tiles * p.chunks > 0x7FFFFFFFLL) return hipErrorInvalidConfiguration;
    ImageParams im = im0;
    im.pool_chunk = p.chunk;
    im.bands = bands;
    im.band_chunks = p.chunks;
    TraceArgs<R> a{sc, im, c};
    const bool count = c.segs || c.draws;
    if (!bvh) return launch_partials_acc<R, ACC_BRUTE>(a, count, p, part, stream);
    const int mode = bvh_walk_mode(sc);
    if (mode == ACC_BVH) return launch_partials_acc<R, ACC_BVH>(a, count, p, part, stream);
    if (mode == ACC_BVH_SPHERES) return launch_partials_acc<R, ACC_BVH_SPHERES>(a, count, p, part, stream);
    if (mode == ACC_GRID) return launch_partials_acc<R, ACC_GRID>(a, count, p, part, stream);
    return launch_partials_acc<R, ACC_BVH_STACK>(a, count, p, part, stream);
}
template hipError_t launch_trace_bands<double>(const SceneView<double>&, const ImageParams&, const Counters&, bool, int,
                                               double*, size_t, PoolPlan*, hipStream_t);
template hipError_t launch_trace_bands<float>(const SceneView<float>&, const ImageParams&, const Counters&, bool, int,
                                              double*, size_t, PoolPlan*, hipStream_t);

hipError_t launch_reduce(const ImageParams& im, double* sum, const double* part, bool tri_bvh, hipStream_t stream,
                         const ReduceGate* gate) {
    if (im.cw <= 0 || im.ch <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    const PoolPlan p = pool_plan(im.cw, im.ch, im.s_end - im.s_begin, tri_bvh, im.pool_chunk);
    if (gate) hipLaunchKernelGGL(reduce_gate_kernel, dim3(1), dim3(64), 0, stream, *gate);
    hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)p.tiles), dim3(64), 0, stream, im, sum, part, p.tiles, p.chunks,
                       (const uint32_t*)(gate ? gate->skip : nullptr));
    return hipGetLastError();
}

// ---- World.hit for given rays (rt_closest_hits: the BVH proof on device arithmetic) ----
template <class R, int ACC>
__global__ __launch_bounds__(64) void closest_hits_kernel(const SceneView<R> sc, const double* __restrict__ rays,
                                                          const size_t n, double* __restrict__ t_out,
                                                          int* __restrict__ kind_out, int* __restrict__ idx_out) {
    __shared__ int stack[RT_BVH_STACK * 64];
    const BvhStack stk{stack + threadIdx.x, 64};
    const size_t r = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= n) return;
    const double* q = rays + 6 * r;
    const V3<R> o = mk<R>((R)q[0], (R)q[1], (R)q[2]), d = mk<R>((R)q[3], (R)q[4], (R)q[5]);
    Work w{0, 0, 0, 0, 0, 0};
    const Closest<R> c = closest_hit_acc<R, ACC>(sc, o, d, w, stk);
    t_out[r] = c.kind == HIT_NONE ? (double)INFINITY : (double)c.t;
    kind_out[r] = c.kind;
    idx_out[r] = c.kind == HIT_NONE ? -1 : c.idx;
}

// ... through the LDS copy of the nodes (the walk of trace_pool_lds_kernel)
template <class R>
__global__ __launch_bounds__(64) void closest_hits_lds_kernel(const SceneView<R> sc, const double* __restrict__ rays,
                                                              const size_t n, double* __restrict__ t_out,
                                                              int* __restrict__ kind_out, int* __restrict__ idx_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_dyn[];   // [boxes][references][stack]
    const int nn = sc.num_sphere_wide;
    rt_u4* box = reinterpret_cast<rt_u4*>(lds_dyn);
    rt_u2* kid = reinterpret_cast<rt_u2*>(lds_dyn + 48 * nn);
    copy_wide_lds(sc.sphere_wide, nn, box, kid, threadIdx.x, 64);
    __syncthreads();
    const BvhStack stk{reinterpret_cast<int*>(lds_dyn + 56 * nn) + threadIdx.x, 64, box, kid};
    const size_t r = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= n) return;
    const double* q = rays + 6 * r;
    const V3<R> o = mk<R>((R)q[0], (R)q[1], (R)q[2]), d = mk<R>((R)q[3], (R)q[4], (R)q[5]);
    Work w{0, 0, 0, 0, 0, 0};
    const Closest<R> c = closest_hit_acc<R, ACC_BVH_SPHERES_LDS>(sc, o, d, w, stk);
    t_out[r] = c.kind == HIT_NONE ? (double)INFINITY : (double)c.t;
    kind_out[r] = c.kind;
    idx_out[r] = c.kind == HIT_NONE ? -1 : c.idx;
}

// ... through the LDS copy of the grid (the walk of trace_pool_lds_kernel<.., ACC_GRID_LDS>)
template <class R>
__global__ __launch_bounds__(64) void closest_hits_grid_lds_kernel(const SceneView<R> sc, const double* __restrict__ rays,
                                                                   const size_t n, double* __restrict__ t_out,
                                                                   int* __restrict__ kind_out, int* __restrict__ idx_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_dyn[];   // [records][cell offsets]
    BvhStack stk{nullptr, 0};
    rt_u4* grec = reinterpret_cast<rt_u4*>(lds_dyn);
    int* gcell = reinterpret_cast<int*>(lds_dyn + grid_lds_rec_bytes(sc));
    copy_grid_lds(sc, grec, gcell, threadIdx.x, 64);
    __syncthreads();
    stk.gcell = gcell;
    stk.grec = grec;
    const size_t r = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= n) return;
    const double* q = rays + 6 * r;
    const V3<R> o = mk<R>((R)q[0], (R)q[1], (R)q[2]), d = mk<R>((R)q[3], (R)q[4], (R)q[5]);
    Work w{0, 0, 0, 0, 0, 0};
    const Closest<R> c = closest_hit_acc<R, ACC_GRID_LDS>(sc, o, d, w, stk);
    t_out[r] = c.kind == HIT_NONE ? (double)INFINITY : (double)c.t;
    kind_out[r] = c.kind;
    idx_out[r] = c.kind == HIT_NONE ? -1 : c.idx;
}

// ... through the LDS copy of the triangle tree's top levels (trace_pool_lds_kernel<.., ACC_BVH_TRI_LDS>'s
// walk; sc.tri_lds_nodes set by the launch)
template <class R>
__global__ __launch_bounds__(64) void closest_hits_tri_lds_kernel(const SceneView<R> sc, const double* __restrict__ rays,
                                                                  const size_t n, double* __restrict__ t_out,
                                                                  int* __restrict__ kind_out, int* __restrict__ idx_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_dyn[];   // [boxes][references][stack]
    const int nn = sc.tri_lds_nodes;
    rt_u4* box = reinterpret_cast<rt_u4*>(lds_dyn);
    rt_u2* kid = reinterpret_cast<rt_u2*>(lds_dyn + 48 * nn);
    copy_wide_lds(sc.tri_wide, nn, box, kid, threadIdx.x, 64);
    __syncthreads();
    BvhStack stk{reinterpret_cast<int*>(lds_dyn + 56 * nn) + threadIdx.x, 64, box, kid};
    stk.ntop = nn;
    const size_t r = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (r >= n) return;
    const double* q = rays + 6 * r;
    const V3<R> o = mk<R>((R)q[0], (R)q[1], (R)q[2]), d = mk<R>((R)q[3], (R)q[4], (R)q[5]);
    Work w{0, 0, 0, 0, 0, 0};
    const Closest<R> c = closest_hit_acc<R, ACC_BVH_TRI_LDS>(sc, o, d, w, stk);
    t_out[r] = c.kind == HIT_NONE ? (double)INFINITY : (double)c.t;
    kind_out[r] = c.kind;
    idx_out[r] = c.kind == HIT_NONE ? -1 : c.idx;
}

template <class R>
hipError_t launch_closest_hits(const SceneView<R>& sc, bool bvh, const double* rays, size_t n, double* t, int* kind,
                               int* idx, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64));
    const bool spheres = bvh && bvh_walk_mode(sc) == ACC_BVH_SPHERES;   // the walk the trace kernel runs
    if (bvh && bvh_walk_mode(sc) == ACC_BVH_STACK && lds_tri_nodes(sc)) {
        SceneView<R> v = sc;
        v.tri_lds_nodes = lds_tri_nodes(sc);
        const size_t lb = (size_t)56 * v.tri_lds_nodes + (size_t)std::min(sc.stack_entries, RT_BVH_STACK) * 64 * 4;
        hipLaunchKernelGGL((closest_hits_tri_lds_kernel<R>), grid, dim3(64), lb, stream, v, rays, n, t, kind, idx);
    } else if (spheres && lds_nodes_bytes(sc)) {
        const size_t lb = (size_t)56 * sc.num_sphere_wide + (size_t)std::min(sc.stack_entries, RT_BVH_STACK) * 64 * 4;
        hipLaunchKernelGGL((closest_hits_lds_kernel<R>), grid, dim3(64), lb, stream, sc, rays, n, t, kind, idx);
    } else if (spheres)
        hipLaunchKernelGGL((closest_hits_kernel<R, ACC_BVH_SPHERES>), grid, dim3(64), 0, stream, sc, rays, n, t, kind, idx);
    else if (bvh && bvh_walk_mode(sc) == ACC_GRID && lds_grid_bytes(sc))
        hipLaunchKernelGGL((closest_hits_grid_lds_kernel<R>), grid, dim3(64), lds_grid_bytes(sc), stream, sc, rays, n, t, kind, idx);
    else if (bvh && bvh_walk_mode(sc) == ACC_GRID)
        hipLaunchKernelGGL((closest_hits_kernel<R, ACC_GRID>), grid, dim3(64), 0, stream, sc, rays, n, t, kind, idx);
    else if (bvh) hipLaunchKernelGGL((closest_hits_kernel<R, ACC_BVH_STACK>), grid, dim3(64), 0, stream, sc, rays, n, t, kind, idx);
    else hipLaunchKernelGGL((closest_hits_kernel<R, ACC_BRUTE>), grid, dim3(64), 0, stream, sc, rays, n, t, kind, idx);
    return hipGetLastError();
}
template hipError_t launch_closest_hits<double>(const SceneView<double>&, bool, const double*, size_t, double*, int*, int*,
                                                hipStream_t);
template hipError_t launch_closest_hits<float>(const SceneView<float>&, bool, const double*, size_t, double*, int*, int*,
                                               hipStream_t);

// ---- multi-device sample split: dst += src elementwise (the shards' sums / counters, in shard order) ----
template <class T>
__global__ __launch_bounds__(256) void add_kernel(T* __restrict__ dst, const T* __restrict__ src, const size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

template <class T>
hipError_t launch_add(T* dst, const T* src, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(add_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dst, src, n);
    return hipGetLastError();
}
template hipError_t launch_add<double>(double*, const double*, size_t, hipStream_t);
template hipError_t launch_add<uint32_t>(uint32_t*, const uint32_t*, size_t, hipStream_t);

// ---- epilogue: mean, toneMap, gammaCorrect, RGBA8 (ray-tracer.js:208-252, post-processor.js:9-42) ----
__device__ __forceinline__ uint8_t to_u8(double c) {
    double v = js_min<double>(255.0, js_max<double>(0.0, floor(c * 255.0)));
    return v != v ? (uint8_t)0 : (uint8_t)v;                  // Uint8ClampedArray stores NaN as 0
}

// one-wave workgroups, like reduce_kernel: the preview frames run beside trace waves
// one channel of the epilogue: the mean times exposure, tone map, gamma (ray-tracer.js:216-235)
__device__ __forceinline__ double post_channel(const FinalizeParams& p, double c, double inv_gamma) {
    const double x = c * p.exposure;
    double tm;
    if (p.tone_map == 1) tm = js_max<double>(0.0, (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14));
    else if (p.tone_map == 2) tm = x;
    else tm = x / (1.0 + x);
    return jsm::pow(js_max<double>(0.0, tm), inv_gamma);      // post-processor.js:38, V8's Math.pow (js_math.h)
}

__global__ __launch_bounds__(64) void finalize_kernel(const FinalizeParams p, const double* __restrict__ sum,
                                                       double* __restrict__ mean, float* __restrict__ post,
                                                       uint8_t* __restrict__ rgba8) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    double c[3], g[3];
    const double inv_gamma = 1.0 / p.gamma;
    for (int k = 0; k < 3; ++k) c[k] = sum[3 * q + k] / (double)p.samples;
    if (mean) { mean[3 * q] = c[0]; mean[3 * q + 1] = c[1]; mean[3 * q + 2] = c[2]; }
    for (int k = 0; k < 3; ++k) g[k] = post_channel(p, c[k], inv_gamma);
    if (post) *reinterpret_cast<float4*>(post + 4 * q) = make_float4((float)g[0], (float)g[1], (float)g[2], 1.0f);
    if (rgba8) {
        uchar4 o = make_uchar4(to_u8(g[0]), to_u8(g[1]), to_u8(g[2]), 255);
        *reinterpret_cast<uchar4*>(rgba8 + 4 * q) = o;
    }
}

// The running frame of a progressive render (RGBA8 only) in at most 32 VGPRs: while batches trace, the
// trace waves hold 480 of a SIMD's 512 VGPRs (5 waves x 96), and finalize_kernel's 80-VGPR waves wait
// for trace waves to exit (measured 0.2 - 7.5 ms per preview, delaying the next batches' reduces on the
// same stream; a fused launch's waves never exit).  The binary64 pow alone needs 64 VGPRs, so the
// preview does without it: the byte finalize_kernel stores, floor(255 pow(max(0, tm), 1/gamma)) clamped,
// is a step function of the tone-mapped value tm, non-decreasing wherever the pow is monotone, so
// it equals the number of thresholds T_k <= tm, T_k (k = 1..255) the least binary64 tm whose byte is >= k
// (a binary search over the binary64 bit patterns with the same pow, gamma_thresholds_kernel).
// Where the pow is not monotone the count is wrong, and such values can only lie next to a threshold (a pow error of an ulp moves the
// byte only where 255 pow(tm) is within ulps of an integer): gamma_exceptions_kernel evaluates the byte on
// the +-kGammaScan ulps around every threshold and records every value whose byte differs from the count;
// the preview checks those exceptions (none or a few).  The preview computes tm exactly as
// finalize_kernel (binary64, same operations): the same bytes (tests/test_gpu_parity.py::
// test_progressive_preview_and_cancel, ::test_preview_thresholds_match_finalize).  NaN tm: byte 0, as to_u8.
__device__ __forceinline__ uint32_t gamma_byte(double tm, double inv_gamma) {
    return to_u8(jsm::pow(js_max<double>(0.0, tm), inv_gamma));
}
__device__ __forceinline__ uint32_t gamma_count(const double* __restrict__ t, double tm) {
    uint32_t lo = 0, n = 255;            // the number of thresholds <= tm (t ascending; a NaN tm passes none)
    while (n > 0) {
        const uint32_t h = n >> 1;
        if (t[lo + h] <= tm) { lo += h + 1; n -= h + 1; }
        else n = h;
    }
    return lo;
}
__global__ __launch_bounds__(256) void gamma_thresholds_kernel(const double inv_gamma, GammaTable* __restrict__ g) {
    const uint32_t k = threadIdx.x + 1;
    if (threadIdx.x == 0) { g->n_exc = 0; g->overflow = 0; }
    if (k > 255) return;
    // smallest non-negative binary64 tm (by bit pattern, the same order) with byte(tm) >= k:
    // byte(+0) = 0 < k, byte(+inf) = 255 >= k
    uint64_t lo = 0, hi = 0x7FF0000000000000ull;
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (gamma_byte(__longlong_as_double((long long)mid), inv_gamma) >= k) hi = mid;
        else lo = mid;
    }
    g->t[k - 1] = __longlong_as_double((long long)hi);
}
// block k - 1 scans +-kGammaScan ulps around threshold k (32 values per thread)
__global__ __launch_bounds__(256) void gamma_exceptions_kernel(const double inv_gamma, GammaTable* __restrict__ g) {
    const int64_t center = __double_as_longlong(g->t[blockIdx.x]);
    for (int j = 0; j < 2 * kGammaScan / 256; ++j) {
        const int64_t bits = center - kGammaScan + (int64_t)threadIdx.x * (2 * kGammaScan / 256) + j;
        if (bits < 0 || bits >= (int64_t)0x7FF0000000000000ll) continue;
        const double tm = __longlong_as_double(bits);
        const uint32_t b = gamma_byte(tm, inv_gamma);
        if (b == gamma_count(g->t, tm)) continue;
        const uint32_t e = atomicAdd(&g->n_exc, 1u);
        if (e < (uint32_t)kGammaExc) { g->exc_tm[e] = tm; g->exc_byte[e] = b; }
        else g->overflow = 1;
    }
}

__global__ __launch_bounds__(64) void preview_kernel(const FinalizeParams p, const double* __restrict__ sum,
                                                     const GammaTable* __restrict__ g, uint8_t* __restrict__ rgba8) {
    const uint32_t ne = min(g->n_exc, (uint32_t)kGammaExc);
    // grid-stride (RT_PREVIEW_WGS caps the workgroups; default one per 64 pixels)
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < p.n; q += gridDim.x * blockDim.x) {
    uint32_t o = 255u << 24;
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
        const double x = sum[3 * q + k] / (double)p.samples * p.exposure;
        double tm;
        if (p.tone_map == 1) tm = js_max<double>(0.0, (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14));
        else if (p.tone_map == 2) tm = x;
        else tm = x / (1.0 + x);
        uint32_t b = gamma_count(g->t, tm);
        for (uint32_t e = 0; e < ne; ++e)        // the values next to a threshold where pow is not monotone
            if (g->exc_tm[e] == tm) b = g->exc_byte[e];
        o |= b << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(rgba8 + 4 * q) = o;
    }
}

// A progressive batch's reduce and its running frame in one pass (RT_FUSED_PREVIEW): each thread adds its
// pixel's chunk partials to the sums exactly as reduce_kernel does, then computes the pixel's RGBA8 byte
// from the new sums exactly as preview_kernel does (the same binary64 values: identical bytes).  One
// one-wave workgroup per tile instead of two kernels' (the trace's one-wave workgroups of triangle scenes
// leave no VGPRs beside them, so every side workgroup takes a trace wave's slot), and the sums are not
// read a second time.  26 VGPRs, like the two kernels it replaces (reduce 16, preview 20).
__global__ __launch_bounds__(64, 8) void reduce_preview_kernel(const ImageParams im, double* __restrict__ sum,
                                                                const double* __restrict__ part, const int tiles,
                                                                const int chunks, const uint32_t* __restrict__ skip,
                                                                const FinalizeParams p, const GammaTable* __restrict__ g,
                                                                uint8_t* __restrict__ rgba8) {
    const int tile = blockIdx.x, m = threadIdx.x;
    if (tile >= tiles || (skip && *skip)) return;
    const Tile t = tile_of(im, tile);
    if (m >= t.nv) return;
    const size_t q = (size_t)(t.y0 + m / t.vw) * im.cw + (t.x0 + m % t.vw);
    double a[3] = {sum[3 * q], sum[3 * q + 1], sum[3 * q + 2]};
    const double* pp = part + (size_t)tile * 3 * 64 + m;
    const size_t stride = (size_t)tiles * 3 * 64;
    for (int c = 0; c < chunks; ++c, pp += stride) {
        a[0] += pp[0];
        a[1] += pp[64];
        a[2] += pp[128];
    }
    sum[3 * q] = a[0]; sum[3 * q + 1] = a[1]; sum[3 * q + 2] = a[2];
    const uint32_t ne = min(g->n_exc, (uint32_t)kGammaExc);
    uint32_t o = 255u << 24;
#pragma unroll 1
    for (int k = 0; k < 3; ++k) {
        const double x = a[k] / (double)p.samples * p.exposure;
        double tm;
        if (p.tone_map == 1) tm = js_max<double>(0.0, (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14));
        else if (p.tone_map == 2) tm = x;
        else tm = x / (1.0 + x);
        uint32_t b = gamma_count(g->t, tm);
        for (uint32_t e = 0; e < ne; ++e)
            if (g->exc_tm[e] == tm) b = g->exc_byte[e];
        o |= b << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(rgba8 + 4 * q) = o;
}

hipError_t launch_reduce_preview(const ImageParams& im, double* sum, const double* part, bool tri_bvh, hipStream_t stream,
                                 const ReduceGate* gate, const FinalizeParams& fp, const GammaTable* table, uint8_t* rgba8) {
    if (im.cw <= 0 || im.ch <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    const PoolPlan pl = pool_plan(im.cw, im.ch, im.s_end - im.s_begin, tri_bvh, im.pool_chunk);
    if (gate) hipLaunchKernelGGL(reduce_gate_kernel, dim3(1), dim3(64), 0, stream, *gate);
    hipLaunchKernelGGL(reduce_preview_kernel, dim3((unsigned)pl.tiles), dim3(64), 0, stream, im, sum, part, pl.tiles,
                       pl.chunks, (const uint32_t*)(gate ? gate->skip : nullptr), fp, table, rgba8);
    return hipGetLastError();
}

// thresholds of gamma_byte for this gamma: only for gammas in [kGammaMin, kGammaMax] (pt_launch.h), the
// range where the +-kGammaScan-ulp exception scan is verified to find every value at which the device
// pow is not monotone (tests/test_gpu_parity.py::test_preview_thresholds_match_finalize checks
// +-3000 ulps around every threshold at both ends and inside).  The width of such a region grows with
// gamma, so outside the range — and when 1/gamma is not a finite positive number, where the byte is not a
// non-decreasing function of tm at all — RGBA8-only epilogues and previews take finalize_kernel.
bool preview_thresholds_ok(double gamma) {
    const double ig = 1.0 / gamma;
    return ig > 0.0 && ig < INFINITY && gamma >= kGammaMin && gamma <= kGammaMax;
}
hipError_t launch_gamma_thresholds(double gamma, GammaTable* T, hipStream_t stream) {
    hipLaunchKernelGGL(gamma_thresholds_kernel, dim3(1), dim3(256), 0, stream, 1.0 / gamma, T);
    hipLaunchKernelGGL(gamma_exceptions_kernel, dim3(255), dim3(256), 0, stream, 1.0 / gamma, T);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeParams& p, const double* sum, double* mean, float* post, uint8_t* rgba8,
                           hipStream_t stream, const GammaTable* thresholds) {
    if (p.n <= 0) return hipSuccess;
    static const int cap = [] {               // A/B: at most this many preview workgroups (0: no cap)
        const char* e = getenv("RT_PREVIEW_WGS");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    if (thresholds && !mean && !post && rgba8)
        hipLaunchKernelGGL(preview_kernel, dim3(cap ? std::min((p.n + 63) / 64, cap) : (p.n + 63) / 64), dim3(64), 0,
                           stream, p, sum, thresholds, rgba8);
    else
        hipLaunchKernelGGL(finalize_kernel, dim3((p.n + 63) / 64), dim3(64), 0, stream, p, sum, mean, post, rgba8);
    return hipGetLastError();
}

// ---- PostProcessor.denoise (post-processor.js:45-77) + the RGBA8 pass of ray-tracer.js:269-275 ----
// 3x3 Gaussian over the Float32 post-gamma frame with clamp-to-edge; accumulation in binary64 in the
// reference's order (ky outer, kx inner); result stored as Float32, RGBA8 made from that Float32.
__global__ __launch_bounds__(256) void denoise_kernel(const int w, const int h, const double w1, const double w2,
                                                      const float* __restrict__ in, float* __restrict__ out,
                                                      uint8_t* __restrict__ rgba8) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= w * h) return;
    const int y = q / w, x = q - y * w;
    double r = 0, g = 0, b = 0, weight = 0;
    for (int ky = -1; ky <= 1; ++ky) {
        for (int kx = -1; kx <= 1; ++kx) {
            const int nx = max(0, min(w - 1, x + kx)), ny = max(0, min(h - 1, y + ky));
            const float4 v = *reinterpret_cast<const float4*>(in + 4 * ((size_t)ny * w + nx));
            const int d2 = kx * kx + ky * ky;
            const double wt = d2 == 0 ? 1.0 : (d2 == 1 ? w1 : w2);
            r += (double)v.x * wt;
            g += (double)v.y * wt;
            b += (double)v.z * wt;
            weight += wt;
        }
    }
    const float a = in[4 * (size_t)q + 3];
    const float4 o = make_float4((float)(r / weight), (float)(g / weight), (float)(b / weight), a);
    if (out) *reinterpret_cast<float4*>(out + 4 * (size_t)q) = o;
    if (rgba8) *reinterpret_cast<uchar4*>(rgba8 + 4 * (size_t)q) =
        make_uchar4(to_u8((double)o.x), to_u8((double)o.y), to_u8((double)o.z), 255);
}

hipError_t launch_denoise(int w, int h, double w1, double w2, const float* in, float* out, uint8_t* rgba8,
                          hipStream_t stream) {
    const int n = w * h;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(denoise_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, w, h, w1, w2, in, out, rgba8);
    return hipGetLastError();
}

#endif  // !RT_ONEWAVE_TU

}  // namespace rt
