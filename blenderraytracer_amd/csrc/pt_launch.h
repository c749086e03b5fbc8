// pt_launch.h — host-visible launch interface of the path-tracing kernels (pt_trace.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_path.h"

namespace rt {

// Counters::totals slots: 0 segments, 1 BVH nodes, 2 sphere tests, 3 triangle tests; RT_PROFILE builds:
// 4..6 cycles (closest hit, shading, regeneration), 7 / 8 walk iterations per lane / per wave, 9 wave
// iterations whose active lanes all sit at one inner node; slot kQueueSlot: the pixel-queue head
constexpr int kTotalSlots = 12;
constexpr int kQueueSlot = 11;

struct Counters {
    double* sum;               // n*3 running per-pixel radiance sums (read-modify-write)
    uint32_t* segs;            // optional n per-pixel world.hit counts
    uint32_t* draws;           // optional n per-pixel RNG draws
    unsigned long long* totals;   // optional [segments, BVH nodes, sphere tests, triangle tests]
    unsigned long long* queue = nullptr;   // pixel-queue head (RT_PIXEL_QUEUE builds), zeroed per launch
    void* pool = nullptr;      // sample-pool radiance buffer (trace_uses_pool()): per-sample radiance
    size_t pool_bytes = 0;     // of up to pool_bytes / pool_sample_bytes(cw, ch, sizeof(R)) samples per launch
};

template <class R>
// walk: ACC_BRUTE (World order), ACC_BVH_STACK (two-child BVH walk) or ACC_BVH4 (four-child walk)
hipError_t launch_trace(const SceneView<R>& sc, const ImageParams& im, const Counters& c, int walk, hipStream_t stream);

// true: launch_trace runs the sample-pool kernel, which needs Counters::pool (at least one sample of
// the crop: pool_sample_bytes); RT_SAMPLE_POOL=0 in the environment selects the lane-per-pixel
// kernel (A/B runs, tests)
bool trace_uses_pool();
// bytes the pool holds per sample of a cw x ch crop: 64 pixels per 8x8 tile (edge tiles padded)
inline size_t pool_sample_bytes(int cw, int ch, size_t real_bytes) {
    return (size_t)((cw + 7) / 8) * (size_t)((ch + 7) / 8) * 64 * 3 * real_bytes;
}

struct FinalizeParams {
    int n;
    int samples;
    int tone_map;
    double exposure, gamma;
};
hipError_t launch_finalize(const FinalizeParams& p, const double* sum, double* mean, float* post, uint8_t* rgba8,
                           hipStream_t stream);
hipError_t launch_denoise(int w, int h, double w1, double w2, const float* in, float* out, uint8_t* rgba8,
                          hipStream_t stream);

}  // namespace rt
