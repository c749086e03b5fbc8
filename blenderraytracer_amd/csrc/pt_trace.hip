// pt_trace.hip — the path-tracing megakernel and its epilogue for gfx950 (MI355X).
//
// Default (sample pool, trace_pool_kernel): a wave owns an 8x8 pixel tile and one chunk of samples;
// the tile's (pixel, sample) items are dealt to its lanes as they finish, per-sample radiance goes to
// an HBM buffer and accumulate_kernel adds it to the per-pixel sums in sample order.
// Lane-per-pixel (trace_kernel, RT_SAMPLE_POOL=0): one lane owns one pixel of the crop window and
// traces that pixel's samples [s_begin, s_end) in order (trace_pixel, pt_path.h).
// Either way each wave covers an 8x8 pixel block, so neighbouring rays share a wave.  BVH mode:
// every lane walks its own path through the two-child BVH with a per-lane stack in LDS; brute-force
// mode: primitive records are walked in World.objects order by every lane in lockstep, so all record
// loads are wave-uniform scalar loads.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "pt_launch.h"

namespace rt {

template <class R>
struct TraceArgs {
    SceneView<R> sc;
    ImageParams im;
    Counters c;
};

// Workgroup = RT_WG_WAVES waves, each an 8x8 pixel block; tiles of 8x8 (1 wave), 16x8 (2) or 16x16 (4).
// One-wave workgroups measured fastest (RTOW f64 4350 vs 4190 Msamples/s, mesh50k 3342 vs 3094): 4x
// more, smaller work items shorten the tail of a frame whose pixels cost very different amounts.
#ifndef RT_WG_WAVES
#define RT_WG_WAVES 1
#endif
constexpr int kWgThreads = 64 * RT_WG_WAVES;
constexpr int kTileW = RT_WG_WAVES >= 2 ? 16 : 8;
constexpr int kTileH = RT_WG_WAVES == 4 ? 16 : 8;

#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 6   // brute force: 80 VGPRs.  At 8 waves (64 VGPRs) the binary64 pool kernel
#endif                            // spills 300 B/lane: Cornell f64 5175 (8) / 6730 (4) / 6830 (6) Msamples/s,
                                  // f32 9274 (8) / 9680 (4) / 9978 (6)

#ifndef RT_BVH_WAVES_PER_SIMD
#define RT_BVH_WAVES_PER_SIMD 4   // binary64 BVH walk: 128 VGPRs (measured 3/4/5 waves: 3861/4065/3287)
#endif
#ifndef RT_BVH_WAVES_F32
#define RT_BVH_WAVES_F32 5        // binary32 BVH walk: 96 VGPRs (measured 3/4/5 waves: 5362/5230/5506)
#endif

// RT_PIXEL_QUEUE=1 (A/B builds): a grid of one resident workgroup per wave slot whose lanes take
// pixels from a global queue (trace_pixels_queue, pt_path.h) instead of one lane per pixel
#ifndef RT_PIXEL_QUEUE
#define RT_PIXEL_QUEUE 0
#endif

template <class R, int ACC>
constexpr int waves_per_simd() {
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
        const uint32_t trips[3] = {r.work.lane_trips, r.work.wave_trips, r.work.uni_trips};
        for (int k = 0; k < 3; ++k) {
            unsigned long long v = trips[k];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(c.totals + 7 + k, v);
        }
    }
}

template <class R, bool COUNT, int ACC>
__global__ __launch_bounds__(kWgThreads, (waves_per_simd<R, ACC>()))
void trace_kernel(const TraceArgs<R> args) {
    const ImageParams& im = args.im;
    LdsSpheres lds{nullptr};
    BvhStack stk{nullptr, 0};
    if constexpr (ACC >= ACC_BVH_STACK) {
        // per-lane traversal stacks, entry k of thread t at [k * kWgThreads + t] (96 / 144 B per lane)
        __shared__ int bvh_stack[(ACC == ACC_BVH4 ? RT_BVH4_STACK : RT_BVH_STACK) * kWgThreads];
        stk.base = bvh_stack + threadIdx.x;
        stk.stride = kWgThreads;
    }
    if constexpr (ACC == ACC_LDS) {
        // stage the binary32 sphere filter records of the whole scene in LDS (one copy per workgroup)
        extern __shared__ SphereFilter lds_spheres[];
        for (int t = threadIdx.x; t < args.sc.num_spheres; t += blockDim.x) lds_spheres[t] = args.sc.sphere_filter[t];
        __syncthreads();
        lds = LdsSpheres{lds_spheres};
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#if RT_PIXEL_QUEUE
    (void)wave;
    unsigned long long* const head = args.c.queue;
    auto fetch = [head]() -> uint32_t {             // wave-aggregated: one atomic per fetching wave
        const uint64_t mask = __ballot(1);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
        uint32_t base = 0;
        if (rank == 0) base = (uint32_t)atomicAdd(head, (unsigned long long)__popcll(mask));
        return (uint32_t)__builtin_amdgcn_readfirstlane(base) + rank;
    };
    const PixelResult r = trace_pixels_queue<R, COUNT, ACC>(args.sc, im, fetch, args.c.sum, COUNT ? args.c.segs : nullptr,
                                                            COUNT ? args.c.draws : nullptr, lds, stk);
#else
    const int tiles_x = (im.cw + kTileW - 1) / kTileW;
    // raster tile order: workgroups are dealt round-robin to the 8 XCDs, so every XCD gets an even mix
    // of cheap (sky) and expensive tiles.  Measured worse: reversed raster (-6 %), scattered (-6 %)
    // and XCD-contiguous bands (-34 %: per-XCD load imbalance) — DESIGN.md.
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int cx = tx * kTileW + (wave % (kTileW / 8)) * 8 + (lane & 7);     // 8x8 pixels per wave
    const int cy = ty * kTileH + (wave / (kTileW / 8)) * 8 + (lane >> 3);
    const bool valid = cx < im.cw && cy < im.ch;
    const size_t q = (size_t)cy * im.cw + cx;
    double acc[3] = {0, 0, 0};
    if (valid) { acc[0] = args.c.sum[3 * q]; acc[1] = args.c.sum[3 * q + 1]; acc[2] = args.c.sum[3 * q + 2]; }
    // invalid lanes trace nothing but stay for the wave reduction below
    const PixelResult r = trace_pixel<R, COUNT, ACC>(args.sc, im, cx, cy, valid ? im.s_end : im.s_begin, acc, lds, stk);
    if (valid) {
        args.c.sum[3 * q] = acc[0]; args.c.sum[3 * q + 1] = acc[1]; args.c.sum[3 * q + 2] = acc[2];
        if (COUNT) {
            if (args.c.segs) args.c.segs[q] += r.segments;
            if (args.c.draws) args.c.draws[q] += r.draws;
        }
    }
#endif
    add_totals<ACC>(args.c, r, lane);
}

// ---- sample pool (the default trace kernel) ----
// A workgroup is one wave = one 8x8 tile of the crop x one chunk of up to `chunk` samples.  The tile's
// (pixel, sample) items are dealt to the lanes from a wave-uniform counter in sample-major order as
// lanes finish their samples, so a lane whose pixel is cheap (sky) goes on with the samples of its
// neighbours instead of idling until the wave's slowest pixel is done; the lanes still hold pixels of
// one 8x8 block (primary-ray coherence as in trace_kernel).  Each sample's radiance goes to
// rad[tile][s - s_begin][m][0..2] (m = pixel of the tile: a wave writes one contiguous region, whole
// cache lines); accumulate_kernel then adds them to the per-pixel sums in sample order:
// the same binary64 additions in the same order as trace_pixel, so the sums are bit-identical to
// trace_kernel's (tests/test_gpu_parity.py::test_sample_pool_bit_identical).
template <class R, bool COUNT, int ACC>
__global__ __launch_bounds__(64, (waves_per_simd<R, ACC>()))
void trace_pool_kernel(const TraceArgs<R> args, R* __restrict__ rad, const int tiles, const int chunk, const int rev) {
    const ImageParams& im = args.im;
    const SceneView<R>& sc = args.sc;
    BvhStack stk{nullptr, 0};
    if constexpr (ACC >= ACC_BVH_STACK) {
        __shared__ int bvh_stack[(ACC == ACC_BVH4 ? RT_BVH4_STACK : RT_BVH_STACK) * 64];
        stk.base = bvh_stack + threadIdx.x;
        stk.stride = 64;
    }
    const LdsSpheres lds{nullptr};
    const int lane = threadIdx.x;
    const int ci = blockIdx.x / tiles, tile = (rev & 1) ? tiles - 1 - (int)(blockIdx.x % tiles) : blockIdx.x % tiles;
    const int tiles_x = (im.cw + 7) / 8;
    const int tx0 = (tile % tiles_x) * 8, ty0 = (tile / tiles_x) * 8;
    const int vw = min(8, im.cw - tx0), nv = vw * min(8, im.ch - ty0);   // valid pixels of the tile
    const int sb = im.s_begin + ci * chunk, se = min(im.s_end, sb + chunk);
    const uint32_t total = (uint32_t)nv * (uint32_t)max(0, se - sb);
    const int ns = im.s_end - im.s_begin;     // samples of this launch
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
        const int px = tx0 + (int)(m % (uint32_t)vw), py = ty0 + (int)(m / (uint32_t)vw);
        const int row = im.y0 + py;
        i = im.x0 + px;
        j = im.height - 1 - row;
        pkey = pixel_key(im.seedm, (uint32_t)row * (uint32_t)im.width + (uint32_t)i);
        q = (size_t)py * im.cw + px;
        s = sb + (int)sr;
        T = mk<R>(1, 1, 1);
        depth = im.max_depth;
        isegs = 0;
        start_sample(sc, im, i, j, pkey, s, g, o, d);
    };
    uint32_t next = 64;                       // items [0, 64) are dealt to lanes 0..63 up front
    bool live = (uint32_t)lane < total;
    if (live) begin_item((uint32_t)lane);
    while (live) {                            // lanes only ever leave this loop, so every live lane
        const uint64_t t0 = RT_TICK();        // has seen every update of `next`
        const Closest<R> c = closest_hit_acc<R, ACC>(sc, o, d, lds, res.work, stk);
        const uint64_t t1 = RT_TICK();
        if (RT_PROFILE) res.cyc[0] += t1 - t0;
        ++res.segments;
        ++isegs;
        V3<R> L;
        const bool done = shade_segment(sc, c, o, d, T, depth, g, L);
        const uint64_t t2 = RT_TICK();
        if (RT_PROFILE) res.cyc[1] += t2 - t1;
        if (done) {
            R* p = rad + (((size_t)tile * ns + (size_t)(s - im.s_begin)) * 64 + m) * 3;
            p[0] = L.x; p[1] = L.y; p[2] = L.z;
            if (COUNT) {
                if (args.c.segs) atomicAdd(args.c.segs + q, isegs);
                if (args.c.draws) atomicAdd(args.c.draws + q, g.k);
            }
        }
        const uint64_t need = __ballot(done);
        if (done) {
            const uint32_t k = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0));
            live = k < total;
            if (live) begin_item(k);
        }
        next += (uint32_t)__popcll(need);
        if (RT_PROFILE) res.cyc[2] += RT_TICK() - t2;
    }
    add_totals<ACC>(args.c, res, lane);
}

// sum[q] += rad[tile][s][m] for s = 0 .. ns-1 in order (binary64, as trace_pixel adds its samples);
// one thread per pixel, a wave per tile (its reads of one sample are 64 x 3 contiguous values)
template <class R>
__global__ __launch_bounds__(256) void accumulate_kernel(const ImageParams im, double* __restrict__ sum,
                                                         const R* __restrict__ rad, const int tiles, const int ns) {
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6), m = threadIdx.x & 63;
    if (tile >= tiles) return;
    const int tiles_x = (im.cw + 7) / 8;
    const int tx0 = (tile % tiles_x) * 8, ty0 = (tile / tiles_x) * 8;
    const int vw = min(8, im.cw - tx0), nv = vw * min(8, im.ch - ty0);
    if (m >= nv) return;
    const size_t q = (size_t)(ty0 + m / vw) * im.cw + (tx0 + m % vw);
    double a0 = sum[3 * q], a1 = sum[3 * q + 1], a2 = sum[3 * q + 2];
    const R* p = rad + ((size_t)tile * ns * 64 + m) * 3;
    RT_UNROLL(8)
    for (int s = 0; s < ns; ++s, p += 64 * 3) {
        a0 += (double)p[0];
        a1 += (double)p[1];
        a2 += (double)p[2];
    }
    sum[3 * q] = a0; sum[3 * q + 1] = a1; sum[3 * q + 2] = a2;
}

bool trace_uses_pool() {
    static int v = -1;
    if (v == -1) {
        const char* e = getenv("RT_SAMPLE_POOL");
        v = !(e && e[0] == '0') && !RT_PIXEL_QUEUE;
    }
    return v == 1;
}

// A/B tile order (RT_POOL_ORDER=rev: last tile first within each chunk)
static int pool_rev() {
    static int v = -1;
    if (v == -1) {
        const char* e = getenv("RT_POOL_ORDER");
        v = e && e[0] == 'r';
    }
    return v;
}

// Samples per pool wave: ~1.5 sqrt(ns) (0.75 sqrt(ns) when the scene has a triangle BVH: its walks
// vary more in length, so shorter waves pay), halved (>= 4) until the launch has >= 64k waves (4x the
// chip's 16k wave slots).  Short waves shorten the frame's drain tail; long ones shorten each wave's
// own tail (its last items finish at different times).  Measured best chunks, 1080p: RTOW 512 spp
// 24-34, 64 spp 16; mesh50k 256 spp 12, 32 spp 8; Cornell 512^2 x 64 spp (4096 tiles) 4.
// RT_POOL_CHUNK overrides (A/B runs).
static int pool_chunk(int ns, int tiles, bool tri_bvh) {
    static int v = -1;
    if (v == -1) {
        const char* e = getenv("RT_POOL_CHUNK");
        v = e ? std::max(1, atoi(e)) : 0;
    }
    if (v) return v;
    int c = std::min(64, std::max(4, (int)((tri_bvh ? 0.75 : 1.5) * std::sqrt((double)ns) + 0.5)));
    while (c > 4 && (long long)tiles * ((ns + c - 1) / c) < 65536) c = std::max(4, c / 2);
    return c;
}

template <class R, int ACC>
static hipError_t launch_pool(const TraceArgs<R>& a0, bool count, hipStream_t stream) {
    const ImageParams& im = a0.im;
    const size_t per_sample = pool_sample_bytes(im.cw, im.ch, sizeof(R));
    const size_t fit = a0.c.pool ? a0.c.pool_bytes / per_sample : 0;
    if (fit < 1) return hipErrorInvalidValue;
    const int ns_max = (int)std::min<size_t>(fit, (size_t)(im.s_end - im.s_begin));
    const int tiles = ((im.cw + 7) / 8) * ((im.ch + 7) / 8), chunk = pool_chunk(ns_max, tiles, ACC >= ACC_BVH && a0.sc.num_tri_nodes > 0);
    R* rad = static_cast<R*>(a0.c.pool);
    for (int b = im.s_begin; b < im.s_end; b += ns_max) {
        TraceArgs<R> a = a0;
        a.im.s_begin = b;
        a.im.s_end = std::min(im.s_end, b + ns_max);
        const int ns = a.im.s_end - b, chunks = (ns + chunk - 1) / chunk;
        if ((long long)tiles * chunks > 0x7FFFFFFFLL) return hipErrorInvalidConfiguration;
        if (count) hipLaunchKernelGGL((trace_pool_kernel<R, true, ACC>), dim3(tiles * chunks), dim3(64), 0, stream, a, rad, tiles, chunk, pool_rev());
        else hipLaunchKernelGGL((trace_pool_kernel<R, false, ACC>), dim3(tiles * chunks), dim3(64), 0, stream, a, rad, tiles, chunk, pool_rev());
        hipLaunchKernelGGL(accumulate_kernel<R>, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, stream, a.im, a.c.sum,
                           (const R*)rad, tiles, ns);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// RT_SPHERE_PATH=lds stages the 16-B sphere filter records in LDS per workgroup instead of reading them
// with scalar loads (measured equal on RTOW); default: scalar loads.
static int sphere_path_override() {
    static int v = -2;
    if (v == -2) {
        const char* e = getenv("RT_SPHERE_PATH");
        v = !e ? -1 : (e[0] == 'l' ? 1 : 0);
    }
    return v;
}

// RT_BVH_WALK (A/B runs): "skip" = the stackless preorder walk, "four" = the four-child walk (when the
// scene's stack bound allows it); default: the two-child walk (measured: four-child -3 % on RTOW,
// +1..8 % on mesh50k)
static int bvh_walk_mode(int four_ok) {
    static int v = -1;
    if (v == -1) {
        const char* e = getenv("RT_BVH_WALK");
        v = !e ? ACC_BVH_STACK : (!strncmp(e, "skip", 4) ? ACC_BVH : (!strncmp(e, "four", 4) ? ACC_BVH4 : ACC_BVH_STACK));
    }
    return v == ACC_BVH4 && !four_ok ? ACC_BVH_STACK : v;
}

static int device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return cus;
}

template <class R, int ACC>
static hipError_t launch_acc(const TraceArgs<R>& a, int tiles, size_t lds_bytes, bool count, hipStream_t stream) {
    if (ACC != ACC_LDS && trace_uses_pool()) return launch_pool<R, ACC>(a, count, stream);
    if (RT_PIXEL_QUEUE) {
        // one workgroup per resident wave slot (4 SIMDs per CU), never more than the queue's blocks
        const int slots = device_cus() * 4 * waves_per_simd<R, ACC>() / RT_WG_WAVES;
        tiles = (int)std::min<uint32_t>((uint32_t)slots, (queue_length(a.im) / 64 + RT_WG_WAVES - 1) / RT_WG_WAVES);
    }
    if (count) hipLaunchKernelGGL((trace_kernel<R, true, ACC>), dim3(tiles), dim3(kWgThreads), lds_bytes, stream, a);
    else hipLaunchKernelGGL((trace_kernel<R, false, ACC>), dim3(tiles), dim3(kWgThreads), lds_bytes, stream, a);
    return hipGetLastError();
}

template <class R>
hipError_t launch_trace(const SceneView<R>& sc, const ImageParams& im, const Counters& c, int walk,
                        hipStream_t stream) {
    if (im.cw <= 0 || im.ch <= 0 || im.s_end <= im.s_begin) return hipSuccess;
    const int tiles = ((im.cw + kTileW - 1) / kTileW) * ((im.ch + kTileH - 1) / kTileH);
    TraceArgs<R> a{sc, im, c};
    const bool count = c.segs || c.draws;
    if (RT_PIXEL_QUEUE) {
        if (!c.queue) return hipErrorInvalidValue;
        const hipError_t e = hipMemsetAsync(c.queue, 0, sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    if (walk != ACC_BRUTE) {
        const int mode = bvh_walk_mode(walk == ACC_BVH4);
        if (mode == ACC_BVH) return launch_acc<R, ACC_BVH>(a, tiles, 0, count, stream);
        if (mode == ACC_BVH4) return launch_acc<R, ACC_BVH4>(a, tiles, 0, count, stream);
        return launch_acc<R, ACC_BVH_STACK>(a, tiles, 0, count, stream);
    }
    const size_t lds_bytes = (size_t)sc.num_spheres * sizeof(SphereFilter);
    const bool lds = sizeof(R) == 8 && sc.num_spheres > 0 && lds_bytes <= 48 * 1024 && sphere_path_override() == 1;
    if constexpr (sizeof(R) == 8) {
        if (lds) return launch_acc<R, ACC_LDS>(a, tiles, lds_bytes, count, stream);
    }
    return launch_acc<R, ACC_BRUTE>(a, tiles, 0, count, stream);
}

template hipError_t launch_trace<double>(const SceneView<double>&, const ImageParams&, const Counters&, int, hipStream_t);
template hipError_t launch_trace<float>(const SceneView<float>&, const ImageParams&, const Counters&, int, hipStream_t);

// ---- epilogue: mean, toneMap, gammaCorrect, RGBA8 (ray-tracer.js:208-252, post-processor.js:9-42) ----
__device__ __forceinline__ uint8_t to_u8(double c) {
    double v = js_min<double>(255.0, js_max<double>(0.0, floor(c * 255.0)));
    return v != v ? (uint8_t)0 : (uint8_t)v;                  // Uint8ClampedArray stores NaN as 0
}

__global__ __launch_bounds__(256) void finalize_kernel(const FinalizeParams p, const double* __restrict__ sum,
                                                       double* __restrict__ mean, float* __restrict__ post,
                                                       uint8_t* __restrict__ rgba8) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= p.n) return;
    double c[3], g[3];
    const double inv_gamma = 1.0 / p.gamma;
    for (int k = 0; k < 3; ++k) c[k] = sum[3 * q + k] / (double)p.samples;
    if (mean) { mean[3 * q] = c[0]; mean[3 * q + 1] = c[1]; mean[3 * q + 2] = c[2]; }
    for (int k = 0; k < 3; ++k) {
        double x = c[k] * p.exposure, tm;
        if (p.tone_map == 1) tm = js_max<double>(0.0, (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14));
        else if (p.tone_map == 2) tm = x;
        else tm = x / (1.0 + x);
        g[k] = pow(js_max<double>(0.0, tm), inv_gamma);
    }
    if (post) *reinterpret_cast<float4*>(post + 4 * q) = make_float4((float)g[0], (float)g[1], (float)g[2], 1.0f);
    if (rgba8) {
        uchar4 o = make_uchar4(to_u8(g[0]), to_u8(g[1]), to_u8(g[2]), 255);
        *reinterpret_cast<uchar4*>(rgba8 + 4 * q) = o;
    }
}

hipError_t launch_finalize(const FinalizeParams& p, const double* sum, double* mean, float* post, uint8_t* rgba8,
                           hipStream_t stream) {
    if (p.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_kernel, dim3((p.n + 255) / 256), dim3(256), 0, stream, p, sum, mean, post, rgba8);
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

}  // namespace rt
