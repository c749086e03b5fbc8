// pt_path.h — the per-lane body of the megakernel: one pixel, samples [s_begin, s_end).
//
// The recursion of rayColor (js/ray-tracer.js:102-123) is flattened into one loop whose body is
// exactly one world.hit: when a path terminates (miss, emissive, absorption, depth cap) the lane
// adds its radiance to the pixel sum and immediately regenerates the camera ray of its next sample
// (path regeneration), so the lanes of a wave stay busy until their pixel is done.
// Radiance is carried as a forward throughput product T (att_0*att_1*...)*E instead of the
// recursion's att_0*(att_1*(...*E)): the same factors, rounded in a different order (<= a few ulp);
// every path DECISION is unaffected.
#pragma once
#include "pt_core.h"

namespace rt {

struct ImageParams {
    int width, height;         // full image (pixel keys)
    int x0, y0, cw, ch;        // crop window (top-down rows)
    int samples;               // sampleCount (divisor of the mean)
    int s_begin, s_end;        // sample range of this launch
    int max_depth;
    int aa_mode;
    uint32_t seedm;            // seed_mix(seed)
    int pool_chunk;            // samples per sample-pool wave (0: pool_chunk's rule for this launch's samples)
    // fused batches (launch_trace_batches): the launch traces batches of batch_samples samples from
    // s_begin, batch_chunks chunks each, batch-major (chunk index c of the launch = batch c / batch_chunks);
    // 0: one batch
    int batch_samples, batch_chunks;
    // the whole-batch multi-device split (rt_capi.cpp): the launch's batches are every batch_ways-th batch
    // of the render (batch b starts batch_ways * batch_samples samples after batch b - 1, and raises the
    // flag batch_flag[b * batch_ways]); 0 or 1: consecutive batches
    int batch_ways;
    // pixel bands (rt_trace_device_bands, pool_order.h band_item): the launch's items band-major over `bands`
    // horizontal bands of whole tile rows, band_chunks chunks each; band b's items counted in
    // Counters::batch_count[b], its flag raised when all are done; 0: no bands
    int bands, band_chunks;
};

// Stochastic AA offsets (ray-tracer.js:136-141): sqrt, cos and sin in binary64 are long code that
// the default supersampling never runs, so they stay out of line (RT_COLD, pt_core.h).  Arguments and
// result by value: no local's address escapes into the call.
template <class R> struct AaUv { R u, v; };
template <class R>
RT_COLD_HD AaUv<R> stochastic_uv(uint32_t key, int i, int j, int width, int height) {
    Rng<R> g{key, 0};
    R r1 = g.next(), r2 = g.next();
    R ox = sqrt(r1) * js_cos<R>((R)2 * (R)3.141592653589793 * r2);       // ray-tracer.js:130-131, V8's Math.cos / sin
    R oy = sqrt(r1) * js_sin<R>((R)2 * (R)3.141592653589793 * r2);
    return AaUv<R>{((R)i + (R)0.5 + ox * (R)0.5) / (R)width, ((R)j + (R)0.5 + oy * (R)0.5) / (R)height};
}

#ifndef RT_OPAQUE_WH
#define RT_OPAQUE_WH 0
#endif
// The camera ray (camera.js:38-51) from the camera's 22 words at cp (SceneView: cam_o, cam_llc, cam_h,
// cam_v, cam_u, cam_vv, cam_w, lens_radius, contiguous)
template <class R, class P, int FEAT = F_ALL>
RT_HD void camera_ray(const SceneView<R>& sc, R u, R v, Rng<R>& g, V3<R>& o, V3<R>& d, P cp) {
    const V3<R> co = mk<R>(cp[0], cp[1], cp[2]);
    const V3<R> llc = mk<R>(cp[3], cp[4], cp[5]);
    const V3<R> hor = mk<R>(cp[6], cp[7], cp[8]);
    const V3<R> ver = mk<R>(cp[9], cp[10], cp[11]);
    const V3<R> cu = mk<R>(cp[12], cp[13], cp[14]);
    const V3<R> cv = mk<R>(cp[15], cp[16], cp[17]);
    V3<R> rd = random_in_unit_disk(g) * (R)cp[21];
    if ((FEAT & F_CAMALL) != 0 && sc.cam_ortho) {
        o = (co + cu * rd.x) + cv * rd.y;
        d = normalize((((llc + hor * u) + ver * v) - o) + mk<R>(cp[18], cp[19], cp[20]) * (R)-1);
    } else {
        o = co + (cu * rd.x + cv * rd.y);
        d = ((llc + hor * u) + ver * v) - o;
    }
}

// RELOAD (RT_CAM_RELOAD: the binary32 LDS pool kernel): the camera words read from the kernel-argument
// segment at every sample start (scalar loads through a pointer the compiler cannot hoist) instead of
// kept live in SGPRs across the segment loop, where the kernel's SGPR spills are reloaded by VALU
// v_readlane instructions: RTOW f32 +1.6 % (SGPR spills 61 -> 49).  In binary64 the freed SGPRs went to
// spills inside the walk instead (round 5: RTOW -0.3 %, mesh50k -9 %, Cornell -16 %; round 6's lean
// one-wave kernels: mesh50k -10 %), so binary32 and, with pt_core.h RT_SC_RELOAD, the binary64 lean
// grid kernel only.
#ifndef RT_CAM_RELOAD
#define RT_CAM_RELOAD 1
#endif
#ifndef RT_CAM_RELOAD_LEAN64
#define RT_CAM_RELOAD_LEAN64 1    // the binary64 lean grid kernel reloads too (round 6, with RT_SC_RELOAD)
#endif
// FEAT without F_CAMALL (the lean kernels): supersampling AA and the perspective camera only
template <class R, bool RELOAD = false, int FEAT = F_ALL>
RT_HD void start_sample(const SceneView<R>& sc, const ImageParams& im, int i, int j, uint32_t pkey, int s, Rng<R>& g,
                        V3<R>& o, V3<R>& d) {
    RT_HCOUNT(HC_SAMPLES, 1);
    g.key = sample_key(pkey, (uint32_t)s);
    g.k = 0;
    R u, v;                                                                   // ray-tracer.js:125-149
#if RT_OPAQUE_WH && defined(__HIP_DEVICE_COMPILE__)
    // (R)width / (R)height converted here from the kernel-argument SGPRs at every sample start instead of
    // hoisted out of the pool loop by the compiler (they then live in scratch): A/B
    int iw = im.width, ih = im.height;
    asm volatile("" : "+s"(iw), "+s"(ih));
    const R width = (R)iw, height = (R)ih;
#else
    const R width = (R)im.width, height = (R)im.height;
#endif
    if ((FEAT & F_CAMALL) == 0) {
        u = ((R)i + g.next()) / width;
        v = ((R)j + g.next()) / height;
    } else if (im.aa_mode == 1) {
        const AaUv<R> uv = stochastic_uv<R>(g.key, i, j, im.width, im.height);
        u = uv.u;
        v = uv.v;
        g.k = 2;
    } else if (im.aa_mode == 0) {
        u = ((R)i + g.next()) / width;
        v = ((R)j + g.next()) / height;
    } else {
        u = ((R)i + (R)0.5) / width;
        v = ((R)j + (R)0.5) / height;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (RELOAD && RT_CAM_RELOAD != 0) {
        // sc is the kernel's first argument's first member (the trace kernels take TraceArgs first,
        // pt_trace.hip): its camera words sit at offsetof(SceneView, cam_o) in the kernel-argument
        // segment.  (Taking &sc.cam_o instead makes the argument escape into a private copy.)
        typedef const __attribute__((address_space(4))) R* CamPtr;
        typedef const __attribute__((address_space(4))) char* ArgPtr;
        CamPtr cp = (CamPtr)((ArgPtr)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(SceneView<R>, cam_o));
        asm volatile("" : "+s"(cp));
        camera_ray<R, CamPtr, FEAT>(sc, u, v, g, o, d, cp);
        return;
    }
#endif
    camera_ray<R, const R*, FEAT>(sc, u, v, g, o, d, &sc.cam_o[0]);
}

// x^5 for Schlick's approximation (materials.js:79-83, Math.pow(1 - cosine, 5)), correctly rounded —
// the fast path of schlick_reflects.  The reference's own Math.pow (V8 in Node 12, restated exactly in
// js_math.h) is not correctly rounded: it differs from RN(x^5) by 1 ulp in ~9.6 % of arguments
// (tests/test_js_host.py::test_pow5_vs_v8_math_pow).  The path only uses the value in
// `reflectance > Math.random()`, whose draws are multiples of 2^-24; schlick_reflects takes V8's own pow
// wherever the reflectance lies within 2^-40 of the draw, so the decision is V8's.  The device pow
// (ocml, <= 1 ulp) costs ~100 binary64 instructions.  Here x^2, x^4, x^5 are carried
// as unevaluated sums hi + lo (error-free products by FMA): the pair approximates x^5 to ~2^-100
// relative, so the single final rounding gives RN(x^5) unless x^5 lies within 2^-100 of a rounding
// midpoint.  10 binary64 ops; exact for x = 0 and x = 1.  Checked against exact rationals
// (tests/test_hostcheck.py::test_pow5_correctly_rounded) and against Node's own Math.pow(x, 5) on the
// same arguments (tests/test_js_host.py::test_pow5_vs_v8_math_pow, which reports the mismatch rate).
// Only for 0 <= x <= 2 (no overflow/underflow concerns: x is 0 or >= 2^-53).
template <class R>
RT_HD R pow5_rn(R x) {
    const R p = x * x, pe = fma(x, x, -p);                 // x^2 = p + pe exactly
    const R q = p * p, qe = fma(p, p, -q) + (R)2 * (p * pe); // x^4 ~ q + qe
    const R r = q * x, re = fma(q, x, -r) + qe * x;          // x^5 ~ r + re
    return r + re;
}

// V8's Math.pow(x, 5) itself (js_math.h): the rare exact path of schlick_reflects — inlined (config 3
// and Cornell unchanged; out of line, the call's register saves cost Cornell 4.4 %) or, in the lean
// triangle-tree kernel, out of line (inlined cost config 5 0.6 %, out of line nothing)
RT_HD double js_pow5_exact(double x) { return jsm::pow(x, 5.0); }
static RT_COLD_HD double js_pow5_exact_ool(double x) { return jsm::pow(x, 5.0); }

// Dielectric.scatter (materials.js:51-83) by value (RT_COLD_DIEL: out of line, so its registers leave the
// trace kernel's allocation — A/B): the new direction and the RNG's draw count
template <class R> struct DielOut { V3<R> nd; uint32_t k; };
#ifndef RT_COLD_DIEL
#define RT_COLD_DIEL 0
#endif
#if RT_COLD_DIEL && defined(__HIP_DEVICE_COMPILE__)
#define RT_DIEL_HD __host__ __device__ __attribute__((noinline))
#else
#define RT_DIEL_HD RT_HD
#endif
// Schlick's decision `reflectance(cosine, ratio) > Math.random()` (materials.js:64, 79-83) for the draw u.
// In binary64 the reference decides with V8's Math.pow (js_math.h), which lies within 1 ulp of the
// correctly rounded pow5_rn on every argument tested (9.6 % differ).  A difference can move the
// reflectance across the draw only when the two lie within a few ulps; within 2^-40 relative (4096 ulps)
// the reflectance is recomputed with V8's own pow — out of line, taken about once per 10^5 tests — so
// the decision is the reference's bit for bit (tests/test_js_host.py::test_schlick_decisions_are_v8s).
// OOL: the exact path out of line (js_pow5_exact_ool)
template <class R, bool OOL = false>
RT_HD bool schlick_reflects(R r0, R cos_t, R u) {
    R refl = r0 + ((R)1 - r0) * pow5_rn((R)1 - cos_t);
    if constexpr (sizeof(R) == 8)
        if (fabs(refl - u) <= refl * (R)0x1p-40)
            refl = r0 + ((R)1 - r0) * (OOL ? js_pow5_exact_ool((R)1 - cos_t) : js_pow5_exact((R)1 - cos_t));
    return refl > u;
}

template <class R, bool OOL = false>
RT_DIEL_HD DielOut<R> dielectric_scatter(R inv_ior, R ior, R r0f, R r0b, bool front, V3<R> n, V3<R> unit, uint32_t key,
                                         uint32_t k) {
    Rng<R> g{key, k};
    V3<R> nd;
    // 1 / ior and both faces' r0 come precomputed (scene_pack.h, the same roundings): two divisions fewer
    R ratio = front ? inv_ior : ior;
    R cos_t = js_min<R>(dot(unit * (R)-1, n), (R)1);
    R sin_t = sqrt((R)1 - cos_t * cos_t);
    bool reflect_it = ratio * sin_t > (R)1;
    if (!reflect_it) {                                                        // random drawn only if it can refract
        RT_HCOUNT(HC_DIELECTRIC_SCHLICK, 1);
        reflect_it = schlick_reflects<R, OOL>(front ? r0f : r0b, cos_t, g.next());
    }
    if (reflect_it) {
        nd = reflect(unit, n);
    } else {
        R ct = js_min<R>(dot(unit * (R)-1, n), (R)1);
        V3<R> perp = (unit + n * ct) * ratio;
        V3<R> par = n * (-sqrt(fabs((R)1 - dot(perp, perp))));
        nd = perp + par;
    }
    return DielOut<R>{nd, g.k};
}

// Scatter at a non-emissive hit (materials.js:20-83).  Returns false when Metal absorbs.
// The three materials share their common steps so that a wave holding several of them runs each step
// once (a branch runs for the union of its lanes): Lambertian and Metal draw one randomInUnitSphere
// and nothing else (Metal's reflect draws nothing), so that rejection loop runs before the material
// branch (RTOW +3.8 %), and the one normalize each material needs — Lambertian the unit-sphere point
// `p`, Metal and Dielectric the ray direction — arrives as `unit`, computed by shade_segment together
// with the missed rays' (skyGradient's) normalize (+1.6 %).
template <class R, bool OOL = false>
RT_HD bool scatter(const MatRec<R>& m, const Hit<R>& h, V3<R> unit, V3<R> p, Rng<R>& g, V3<R>& nd, V3<R>& att) {
    if (m.type <= 1) {
        att = mk(m.c[0], m.c[1], m.c[2]);
        if (m.type == 0) {                                                    // Lambertian :20-25
            RT_HCOUNT(HC_LAMBERT, 1);
            nd = h.n + unit;
            return true;
        }
        RT_HCOUNT(HC_METAL, 1);
        nd = reflect(unit, h.n) + p * m.p;                                    // Metal :36-41 (roughness)
        return dot(nd, h.n) > (R)0;
    }
    RT_HCOUNT(HC_DIELECTRIC, 1);
#ifdef RT_PROBE_NODIEL                                                        // timing probe only (inexact)
    nd = reflect(unit, h.n);
    att = mk<R>(1, 1, 1);
    return true;
#endif
    // Dielectric :51-83 (ior)
    const DielOut<R> r = dielectric_scatter<R, OOL>(m.c[0], m.p, m.c[1], m.c[2], h.front, h.n, unit, g.key, g.k);
    nd = r.nd;
    g.k = r.k;
    att = mk<R>(1, 1, 1);
    return true;
}

// RT_PROFILE=1 (A/B builds only): shader-clock cycles per lane spent in closest hit, shading and
// sample regeneration, reduced per wave (max) into Counters::totals[4..6]
#ifndef RT_PROFILE
#define RT_PROFILE 0
#endif
#if RT_PROFILE && defined(__HIP_DEVICE_COMPILE__)
#define RT_TICK() ((uint64_t)clock64())
#else
#define RT_TICK() ((uint64_t)0)
#endif

struct PixelResult { uint32_t segments, draws; Work work; uint64_t cyc[3]; };

// Shade the segment whose closest hit is c (rayColor's body after world.hit, ray-tracer.js:106-122):
// emission / scatter / background.  Returns true when the sample's path ended; its radiance L is
// then in `L`, otherwise (o, d, T, depth) describe the next segment.
template <class R, int FEAT = F_ALL>
RT_HD bool shade_segment(const SceneView<R>& sc, const Closest<R>& c, V3<R>& o, V3<R>& d, V3<R>& T, int& depth,
                         Rng<R>& g, V3<R>& L, const MatRec<R>* mats = nullptr) {
    bool done = true;
    L = mk<R>(0, 0, 0);
    const bool hit = c.kind != HIT_NONE;
    Hit<R> h{};
    MatRec<R> m{};
    V3<R> p = mk<R>(0, 0, 0);
    if (hit) {
        h = hit_record<R, FEAT>(sc, o, d, c);
        m = mats ? mats[h.mat] : sc.mats[h.mat];            // mats: an LDS copy (RT_MAT_LDS A/B)
        if (m.type <= 1) p = random_in_unit_sphere(g);                       // Lambertian / Metal's only draws
    }
    // one normalize for every lane (see scatter): Lambertian's p, else the ray direction (Metal,
    // Dielectric, and a missed ray's skyGradient)
    const V3<R> unit = normalize(hit && m.type == 0 ? p : d);
    if (hit) {
        if (m.type == 3) {                                                    // Emissive (materials.js:87-96)
            RT_HCOUNT(HC_EMISSIVE, 1);
            L = mk(T.x * m.c[0], T.y * m.c[1], T.z * m.c[2]);                 // emission
        } else {
            V3<R> nd, att;
            if (scatter<R, (FEAT & F_TRIS) != 0 && FEAT != F_ALL>(m, h, unit, p, g, nd, att)) {
                T = mk(T.x * att.x, T.y * att.y, T.z * att.z);
                o = h.p;
                d = nd;
                done = --depth <= 0;                                          // rayColor(.., 0) returns 0
            }
        }
    } else {
        RT_HCOUNT(HC_MISS, 1);
        const V3<R> bg = background<R, FEAT>(sc, d, unit);                    // world.background(ray)
        L = mk(T.x * bg.x, T.y * bg.y, T.z * bg.z);
    }
    return done;
}

// Trace samples [im.s_begin, s_end) of crop pixel (cx, cy), adding radiance into sum[0..2].
// In binary64 with maxBounces <= RT_REC_DEPTH, a sample's radiance is evaluated in the order of the
// reference's recursion (ray-tracer.js:102-121: emitted + attenuation * rayColor(scattered)): the
// attenuations are kept and multiplied onto the path's end value from the last bounce back, a0 * (a1 *
// (... * X)), where the sample pool carries the throughput forward, ((a0 * a1) * ...) * X.  emitted is
// zero for every material that scatters (an Emissive hit ends the path), so this is the recursion's
// value bit for bit; with the samples added in sample order (this function) the means are the
// reference's.  Deeper renders carry the throughput forward.
#ifndef RT_REC_DEPTH
#define RT_REC_DEPTH 16
#endif
template <class R, bool COUNT, int ACC = ACC_BRUTE>
RT_HD PixelResult trace_pixel(const SceneView<R>& sc, const ImageParams& im, int cx, int cy, int s_end, double* sum,
                              BvhStack stk = BvhStack{nullptr, 0}) {
    const int i = im.x0 + cx, row = im.y0 + cy, j = im.height - 1 - row;
    const uint32_t pkey = pixel_key(im.seedm, (uint32_t)row * (uint32_t)im.width + (uint32_t)i);
    PixelResult res{0, 0, {0, 0, 0}, {0, 0, 0}};
    int s = im.s_begin;
    double sx = sum[0], sy = sum[1], sz = sum[2];
    Rng<R> g;
    V3<R> o, d, T = mk<R>(1, 1, 1);
    int depth = im.max_depth;
    const bool rec = sizeof(R) == 8 && im.max_depth <= RT_REC_DEPTH;
    V3<R> att[RT_REC_DEPTH];                   // rec: the sample's attenuations, bounce by bounce
    int nb = 0;
    bool skip_tri = false;                     // tri_exit_bound (pt_core.h)
    if (s < s_end) start_sample(sc, im, i, j, pkey, s, g, o, d);
    while (s < s_end) {
        const uint64_t t0 = RT_TICK();
        const Closest<R> c = closest_hit_acc<R, ACC>(sc, o, d, res.work, stk, skip_tri);
        const uint64_t t1 = RT_TICK();
        if (RT_PROFILE) res.cyc[0] += t1 - t0;
        ++res.segments;
        V3<R> L;
        if (rec) T = mk<R>(1, 1, 1);           // then T = 1 * attenuation and L = 1 * X: exact
        const bool done = shade_segment(sc, c, o, d, T, depth, g, L);
        if constexpr (sizeof(R) == 8 && (ACC == ACC_BVH || ACC == ACC_BVH_STACK || ACC == ACC_BVH_STACK_LEAN))
            skip_tri = !done && c.kind == HIT_TRI && leaves_tri_hull(sc, c.idx, o, d);
        const uint64_t t2 = RT_TICK();
        if (RT_PROFILE) res.cyc[1] += t2 - t1;
        if (rec && !done) att[nb++] = T;
        if (done) {
            if (rec) {
                for (int k = nb - 1; k >= 0; --k) L = mk(att[k].x * L.x, att[k].y * L.y, att[k].z * L.z);
                nb = 0;
            }
            sx += (double)L.x; sy += (double)L.y; sz += (double)L.z;
            if (COUNT) res.draws += g.k;
            ++s;
            T = mk<R>(1, 1, 1);
            depth = im.max_depth;
            if (s < s_end) start_sample(sc, im, i, j, pkey, s, g, o, d);
        }
        if (RT_PROFILE) res.cyc[2] += RT_TICK() - t2;
    }
    sum[0] = sx; sum[1] = sy; sum[2] = sz;
    return res;
}

}  // namespace rt
