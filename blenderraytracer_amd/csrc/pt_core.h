// pt_core.h — device-side building blocks of the path-tracing megakernel (gfx950).
//
// Everything is templated on the arithmetic type R:
//   R = double : the reference's own arithmetic (JS numbers), compiled with -ffp-contract=off so
//                every + - * / sqrt is one correctly rounded binary64 op in the JS evaluation order.
//                Ray paths then follow the reference decision for decision (tests/test_gpu_parity.py).
//   R = float  : fast mode; same algorithm in binary32.
// Reference citations are js/<file>:<line> in Shinzef/BlenderRayTracer.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "js_math.h"

// Path code is __host__ __device__ so that tests/hostcheck can run the kernel's exact per-lane
// logic on the CPU (test infrastructure only; librt_hip.so has no host execution path).
#define RT_HD __host__ __device__ __forceinline__
// Code the hot loop rarely or never runs (hdri / procedural backgrounds, stochastic AA) is kept out of
// line on the device, so it does not take part in the trace kernel's register allocation.
#ifndef RT_COLD_BG
#define RT_COLD_BG 1               // RTOW +1.2 %, mesh50k +0.8 %, Cornell -1.5 %
#endif
#if RT_COLD_BG && defined(__HIP_DEVICE_COMPILE__)
#define RT_COLD __attribute__((noinline))
#else
#define RT_COLD
#endif
#define RT_COLD_HD __host__ __device__ RT_COLD

namespace rt {

// Math.pow / exp / sin / cos as the reference's V8 computes them (js_math.h) in binary64; the binary32
// fast mode keeps the device's own
template <class R> RT_HD R js_pow(R x, R y) {
    if constexpr (sizeof(R) == 8) return jsm::pow(x, y);
    else return pow(x, y);
}
template <class R> RT_HD R js_exp(R x) {
    if constexpr (sizeof(R) == 8) return jsm::exp(x);
    else return exp(x);
}
template <class R> RT_HD R js_sin(R x) {
    if constexpr (sizeof(R) == 8) return jsm::sin(x);
    else return sin(x);
}
template <class R> RT_HD R js_cos(R x) {
    if constexpr (sizeof(R) == 8) return jsm::cos(x);
    else return cos(x);
}

// Host-only event counts for the instruction-floor model: compiled into the host check
// built with -DRT_HOST_COUNTERS (scripts/floor_counts.py) and nowhere else.
#if defined(RT_HOST_COUNTERS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long rt_host_count[16];
#define RT_HCOUNT(k, n) (rt_host_count[k] += (n))
#else
#define RT_HCOUNT(k, n) ((void)0)
#endif
enum HostCount { HC_F64_TESTS = 0, HC_DISC_OK, HC_SECOND_ROOT, HC_ACCEPT, HC_LAMBERT, HC_METAL, HC_DIELECTRIC,
                 HC_EMISSIVE, HC_MISS, HC_SAMPLES, HC_SPHERE_DRAW_ROUNDS, HC_DISK_DRAW_ROUNDS, HC_FILTER_TESTS,
                 HC_DIELECTRIC_SCHLICK, HC_TRI_FILTERS, HC_TRI_TESTS };

// ---- keyed RNG ------------------------------------------------------------------
RT_HD uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
RT_HD uint32_t pixel_key(uint32_t seedm, uint32_t pixel) { return lowbias32(seedm ^ pixel); }
RT_HD uint32_t sample_key(uint32_t pkey, uint32_t sample) {
    return lowbias32(pkey ^ lowbias32(sample + 0x1B873593U));
}

template <class R>
struct Rng {
    uint32_t key, k;
    RT_HD uint32_t next_u24() {                       // next() == next_u24() * 2^-24
        uint32_t h = lowbias32(key ^ (k * 0x9E3779B9U));
        ++k;
        return h >> 8;
    }
    RT_HD R next() { return (R)next_u24() * (R)(1.0 / 16777216.0); }   // exact in f32 and f64
};

// ---- JS semantics helpers ----------------------------------------------------------------------
template <class R> RT_HD R js_max(R a, R b) {   // Math.max: NaN-propagating
    return (a != a || b != b) ? (R)NAN : (a > b ? a : b);
}
template <class R> RT_HD R js_min(R a, R b) {
    return (a != a || b != b) ? (R)NAN : (a < b ? a : b);
}

template <class R> struct V3 { R x, y, z; };
template <class R> RT_HD V3<R> mk(R x, R y, R z) { return V3<R>{x, y, z}; }
template <class R> RT_HD V3<R> operator+(V3<R> a, V3<R> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class R> RT_HD V3<R> operator-(V3<R> a, V3<R> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class R> RT_HD V3<R> operator*(V3<R> a, R s) { return {a.x * s, a.y * s, a.z * s}; }
template <class R> RT_HD V3<R> vdiv(V3<R> a, R s) { return {a.x / s, a.y / s, a.z / s}; }
template <class R> RT_HD R dot(V3<R> a, V3<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <class R> RT_HD V3<R> cross(V3<R> a, V3<R> b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// RT_DIV_RCP: a vector divided by one scalar s through y = RN(1/s) instead of three IEEE divisions.
// Markstein's theorem: if q is a faithful rounding of x/s (within 1 ulp) and y = RN(1/s), then with the
// exact remainder e = x - q s (one FMA) RN(q + e y) = RN(x / s), when nothing under- or overflows.
// q0 = RN(x y) is NOT always faithful (it can be 1.5 ulp off: y's error times x, plus q0's rounding), so
// binary64 — the reference's arithmetic — takes one correction more: q1 = RN(q0 + RN(x - q0 s) y) is within
// 1/2 ulp + 2^-100 ulp of x/s, hence faithful, and the second correction RN(q1 + (x - q1 s) y) is the
// correctly rounded quotient by the theorem (5 binary64 ops instead of a ~22-slot division).  Binary32
// (the non-conforming fast mode) keeps the single correction, bit-identical to the division on every
// significand of x for 2,000+ divisors (tests/test_root_div.py).  Guarded so that every intermediate is a
// normal number: 2^-500 <= |x| <= 2^500 and 2^-400 <= |s| <= 2^400, so |x / s| lies in [2^-900, 2^900]
// (binary32: 2^-60 .. 2^60, 2^-40 .. 2^40); outside — zero components included — the plain divisions run.
// The sphere normal's (p - c) / r uses RN(1/r) precomputed per sphere (no division left), normalize one
// division for y.  Single correction in both precisions: RTOW f64 +0.9 %, f32 +1.2 % (DESIGN.md §4;
// round 1's form, a runtime reciprocal and refinement, measured -3.5 %).
#ifndef RT_DIV_RCP
#define RT_DIV_RCP 1
#endif
#ifndef RT_DIV_F64_TWICE
#define RT_DIV_F64_TWICE 1        // 0 (A/B): round 4's single correction in binary64 too
#endif
// Binary64 measured (RTOW 256 spp f64, interleaved x2): two corrections 10197, IEEE divisions 10260, round
// 4's single correction 10299 Msamples/s — so binary64 takes the IEEE divisions (RT_DIV_RCP_F64 = 0:
// exact by definition; 1: the provable two-correction form above, A/B)
#ifndef RT_DIV_RCP_F64
#define RT_DIV_RCP_F64 0
#endif
template <class R> constexpr bool div_rcp_on() { return RT_DIV_RCP && (sizeof(R) == 4 || RT_DIV_RCP_F64); }
template <class R> RT_HD R div_rcp_1(R x, R s, R y) {           // guarded by the caller
    const R q0 = x * y;
    const R q1 = fma(fma(-q0, s, x), y, q0);
    if constexpr (sizeof(R) == 4 || RT_DIV_F64_TWICE == 0) return q1;
    return fma(fma(-q1, s, x), y, q1);
}
template <class R> RT_HD bool div_rcp_range(R x) {
    const R ax = fabs(x);
    return ax >= (R)(sizeof(R) == 8 ? 0x1p-500 : 0x1p-60) && ax <= (R)(sizeof(R) == 8 ? 0x1p500 : 0x1p60);
}
// smallest / largest |a.k| (device: IEEE minimum / maximum, NaN-propagating — a NaN fails every guard
// compare; host: fmin / fmax, where a NaN component goes through div_rcp_1 and stays NaN)
template <class R> RT_HD R min3abs(V3<R> a) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_minimum(fabs(a.x), __builtin_elementwise_minimum(fabs(a.y), fabs(a.z)));
#else
    return fmin(fabs(a.x), fmin(fabs(a.y), fabs(a.z)));
#endif
}
template <class R> RT_HD R max3abs(V3<R> a) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_maximum(fabs(a.x), __builtin_elementwise_maximum(fabs(a.y), fabs(a.z)));
#else
    return fmax(fabs(a.x), fmax(fabs(a.y), fabs(a.z)));
#endif
}
template <class R> RT_HD V3<R> vdiv_rcp(V3<R> a, R s, R y) {
    const R smin = sizeof(R) == 8 ? (R)0x1p-400 : (R)0x1p-40, smax = sizeof(R) == 8 ? (R)0x1p400 : (R)0x1p40;
    const R xmin = sizeof(R) == 8 ? (R)0x1p-500 : (R)0x1p-60, xmax = sizeof(R) == 8 ? (R)0x1p500 : (R)0x1p60;
    const R as = fabs(s);
    // every component in div_rcp_range, as one min3 and one max3 (RTOW f32: six compares fewer)
    if (div_rcp_on<R>() && min3abs(a) >= xmin && max3abs(a) <= xmax && as >= smin && as <= smax)
        return {div_rcp_1(a.x, s, y), div_rcp_1(a.y, s, y), div_rcp_1(a.z, s, y)};
    return vdiv(a, s);
}
// normalize's a / l, l = RN(sqrt(RN(RN(ax^2 + ay^2) + az^2))): every |a.k| <= l (1 + 2^-22) (three
// roundings of the sum, one of the sqrt; an overflowing square makes l infinite), so the quotients lie
// within the guard's range once l does and the smallest |a.k| does — one min3 and three compares
// instead of vdiv_rcp's nine (RT_UNIT_GUARD=0, A/B: vdiv_rcp's guard)
#ifndef RT_UNIT_GUARD
#define RT_UNIT_GUARD 1
#endif
template <class R> RT_HD V3<R> vdiv_rcp_unit(V3<R> a, R l, R y) {
    if (!RT_UNIT_GUARD) return vdiv_rcp(a, l, y);
    const R smin = sizeof(R) == 8 ? (R)0x1p-400 : (R)0x1p-40, smax = sizeof(R) == 8 ? (R)0x1p400 : (R)0x1p40;
    const R xmin = sizeof(R) == 8 ? (R)0x1p-500 : (R)0x1p-60;
    if (div_rcp_on<R>() && min3abs(a) >= xmin && l >= smin && l <= smax)
        return {div_rcp_1(a.x, l, y), div_rcp_1(a.y, l, y), div_rcp_1(a.z, l, y)};
    return vdiv(a, l);
}
template <class R> RT_HD V3<R> normalize(V3<R> a) {          // math.js:18
    R l = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
#if RT_DIV_RCP
    return l > (R)0 ? vdiv_rcp_unit(a, l, (R)1 / l) : mk<R>(0, 0, 0);
#else
    return l > (R)0 ? vdiv(a, l) : mk<R>(0, 0, 0);
#endif
}
template <class R> RT_HD V3<R> reflect(V3<R> a, V3<R> n) {   // math.js:19
    return a - n * ((R)2 * dot(a, n));
}

// ---- scene records in HBM (built by rt_scene_create) ---------------------------------------------
enum RunKind : int { RUN_SPHERES = 0, RUN_PLANES = 1, RUN_BOXES = 2, RUN_TRIANGLES = 3, RUN_MESH = 4 };
struct Run { int kind, begin, end, mat; };   // consecutive world objects of one kind (mat: mesh material)

template <class R> struct SphereRec { R cx, cy, cz, r2; };            // r2 = radius*radius (geometry.js:19)
// binary32 pre-filter record of a sphere (f64 mode only): centre rounded to f32 and the radius^2
// inflated by the error bound, r2p = r^2 + 2^-17 (2|c|^2 + r^2), rounded up; see sphere_filter_bound.
struct SphereFilter { float cx, cy, cz, r2p; };
// the filter's margin 2^RT_FILTER_MARGIN Q (sphere_filter_bound)
#ifndef RT_FILTER_MARGIN
#define RT_FILTER_MARGIN (-17)
#endif
constexpr double filter_margin() {   // 2^RT_FILTER_MARGIN, exact
    double v = 1.0;
    for (int k = 0; k > RT_FILTER_MARGIN; --k) v *= 0.5;
    return v;
}
template <class R> struct PlaneRec { R px, py, pz, nx, ny, nz; };
template <class R> struct BoxRec { R mnx, mny, mnz, mxx, mxy, mxz; };
template <class R> struct TriRec { R v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z, nx, ny, nz; };  // e1=v1-v0, e2=v2-v0
// A material in 40 B (binary64): c = albedo (Lambertian, Metal), emission = color * intensity
// (Emissive) or, for a Dielectric, {1 / index, Schlick r0 of the front face, of the back face}; p =
// roughness (Metal) or refraction index (Dielectric) — a hit reads one record per segment
template <class R> struct MatRec { int type, pad; R c[3]; R p; };
// BVH leaf records in leaf order: everything one primitive test and its acceptance need (the
// binary32 filter, the R-precision geometry, World index, World.objects index, material) in one
// contiguous record, so a leaf issues all its loads at once instead of a chain of dependent ones.
template <class R> struct SphereLeaf { SphereFilter f; SphereRec<R> s; int id, obj, mat, pad; };   // 64 B
template <> struct SphereLeaf<float> { SphereRec<float> s; int id, obj, mat, pad; };                 // 32 B
// a triangle leaf carries only what the test reads (the winner's normal is read from TriRec by hit_record)
template <class R> struct TriGeom { R v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z; };
// (the material is read from SceneView::tri_mat when a triangle is accepted: 80 / 48 B instead of 96 / 64,
// mesh50k f32 +1.6 %, f64 ±0)
template <class R> struct alignas(16) TriLeaf { TriGeom<R> t; int id, obj; };                           // 80 / 48 B
// binary32 pre-filter record of a triangle (binary64 mode only; leaf order, beside TriLeaf<double>):
// v0, e1, e2 rounded to binary32 and n = e2 x e1 (computed in binary64, rounded); n is NaN for a triangle
// outside the filter's range (tri_filter_bound: then it is never rejected).  48 B
struct alignas(16) TriFilter { float v0[3], e1[3], e2[3], n[3]; };

// BVH node (32 B), nodes in depth-first preorder: an internal node's first child is the next node,
// `skip` is the index just past its subtree.  fc = (first << 4) | count for a leaf of `count` <= 15
// primitives at leaf-order positions [first, first+count), 0 for an internal node.
struct BvhNode { float lo[3]; int skip; float hi[3]; int fc; };
// The same tree as 64-B two-child nodes for the ordered stack walk: box k = {lo, hi} of child k,
// child[k] >= 0 an inner node, < 0 the leaf ~fc.  Depth <= RT_BVH_STACK (scene_pack.h).
// Bounds interleaved by child (lo[axis][child]) so both children's planes of an axis form one float2:
// the slab test is 6 packed FMAs (v_pk_fma_f32) per node.
struct Bvh2Node { float lo[3][2]; float hi[3][2]; int child[2]; int pad[2]; };
#ifndef RT_BVH_STACK
#define RT_BVH_STACK 24           // 6 KB of LDS per one-wave workgroup; trees up to ~16.7M primitives
#endif

template <class R>
struct SceneView {
    const Run* runs;
    int num_runs;
    int num_prims;                 // primitives tested per segment (brute force)
    const SphereRec<R>* spheres;
    const SphereFilter* sphere_filter;   // f64 mode: binary32 pre-filter records (same order)
    int num_spheres;
    const R* sphere_r;             // radius (normal = (p - c) / r, geometry.js:34)
    const R* sphere_inv_r;         // RN(1 / radius) in R (RT_DIV_RCP)
    const PlaneRec<R>* planes;
    const BoxRec<R>* boxes;
    const TriRec<R>* tris;
    const int* sphere_mat;
    const int* plane_mat;
    const int* box_mat;
    const int* tri_mat;            // per triangle (mesh triangles carry the mesh's material)
    const MatRec<R>* mats;
    int num_mats;
    const int* perm;               // World.cloudNoise.p[512]
    // acceleration structure (closest_hit_bvh): planes and boxes are tested brute force with their
    // World.objects index, spheres and triangles through one BVH each over leaf-order copies
    int num_planes, num_boxes;
    const int* plane_obj;
    const int* box_obj;
    const BvhNode* sphere_nodes;
    int num_sphere_nodes;
    const SphereLeaf<R>* bvh_sphere_leaf;
    const BvhNode* tri_nodes;
    int num_tri_nodes;
    const TriLeaf<R>* bvh_tri_leaf;
    const TriFilter* tri_filter;   // binary64: the triangle leaves' binary32 pre-filter records (same order)
    const Bvh2Node* sphere_wide;   // two-child nodes of the two trees (preorder)
    const Bvh2Node* tri_wide;
    int num_sphere_wide, num_tri_wide;
    int tri_lds_nodes;             // ACC_BVH_TRI_LDS: the triangle tree's nodes [0, tri_lds_nodes) are read
                                   // from the workgroup's LDS copy (set per launch, pt_trace.hip)
    int stack_entries;             // deepest leaf of the two trees (>= 1): the ordered walk's stack bound
    const SphereLeaf<R>* big_spheres;   // dominant spheres kept out of the sphere tree (scene_pack.h)
    int num_big_spheres;
    // uniform grid over the sphere tree's spheres (ACC_GRID, scene_pack.h build_grid): cell c = (x, y, z)
    // -> x + n0 (y + n1 z) holds grid_leaf[grid_cell[c] .. grid_cell[c + 1])
    const int* grid_cell;
    const SphereLeaf<R>* grid_leaf;
    int grid_n[3];
    float grid_lo[3], grid_hi[3], grid_cs[3];   // cells [lo + k cs, lo + (k+1) cs); hi: the padded box
    float grid_ics[3];             // 1 / grid_cs rounded to binary32: the walk's entry cell
    float grid_far;                // rays with |origin|_inf beyond this take the sphere-list fallback
    int num_grid_cells;            // 0: no grid
    int num_grid_recs;             // grid_cell[num_grid_cells]: registrations (records in grid_leaf)
    int use_grid;                  // choose_walk (scene_pack.h): the trace kernel walks the grid
    // tri_exit_bound (binary64): per triangle id {C+, C-}, upper bounds of n.x and -n.x over every vertex
    // of every triangle (+inf: not computed / no use), and the bound's scene constants
    const double* tri_exit;
    double exit_k0, exit_k1, exit_k2, exit_l1, exit_l2;
    // camera (camera.js:8-36 vectors, computed on the host in binary64)
    R cam_o[3], cam_llc[3], cam_h[3], cam_v[3], cam_u[3], cam_vv[3], cam_w[3];   // contiguous with
    R lens_radius;                                                                 // lens_radius: start_sample
    int cam_ortho;
    int background;
    R sky_intensity;
    R solid[3];
};

enum HitKind : int { HIT_NONE = -1, HIT_SPHERE = 0, HIT_PLANE = 1, HIT_BOX = 2, HIT_TRI = 3 };

// tri_exit_bound.  A ray leaving triangle A's plane on the side away from every triangle of the scene
// cannot hit a triangle, so its segment skips the triangle walk (a convex mesh's reflected rays: config 5).
// N = +-n (n: A's stored normal, |n|_2 within 1e-6 of 1, else C = +inf), C >= N.w over the exact vertices w
// in {v0, v0 + e1, v0 + e2} of every triangle (scene_pack.h build_tri_exit), g = N.d >= 0, a = N.o.  Take
// eps = 2^-53, Me >= every |e1|inf, |e2|inf, Mv >= every |v0|inf, md = |d|inf, mo = |o|inf, Ms = mo + Mv.
// The binary64 test (triangle_candidate) decides through A = d.(e2 x e1)..., X, Y, Z (tri_filter_bound),
// computed within EA = 64 eps md Me^2, EX = EY = 64 eps md Me Ms, EZ = 64 eps Me^2 Ms of the exact values.
// Suppose it accepts a triangle f at t64 >= 0.001 with L1: 1e4 (EX + 1.01 EA) <= 0.004 and L2: EZ <= 1e-9.
//  - |A64| >= 1e-4, so |A| > 0 and |A - A64| / |A64| <= 1e4 EA <= 0.004;
//  - the exact u = X / A, v = Y / A lie within du = 2.1 eps + 1e4 (EX + 1.01 EA) of u64, v64 (in [0, 1]),
//    so the weights (1 - u - v, u, v) of the exact ray point x(t) = v0 + u e1 + v e2 are >= -delta,
//    delta = eps + 2 du, and N.x(t) <= C + 2 delta |N|_1 2 Me <= C + 7 delta Me;
//  - the exact t = Z / A >= (0.001 (1 - 2.1 eps) - 1e4 EZ) / (1 + 1e4 EA) >= 0.000986 > T0 = 0.00095;
//  - but N.x(t) = a + t g >= a + T0 g.
// So no triangle is accepted when a - C + T0 g > 7 delta Me + the evaluation errors of a, g and the sum
// (<= eps (10.6 mo + 5.3 Mv + 5.3 Me + 0.01 md)): the check below is twice that total,
//   B = K0 + K1 md (mo + K2) + 24 eps (mo + md),  K0 = 2 eps (42 Me + 12 Mv),  K1 = 2 eps 8.96e6 Me^2,
//   K2 = Mv + 1.01 Me,
// and L1, L2 as md (mo + K2) <= exit_l1, mo <= exit_l2.  NaN anywhere fails a comparison: no skip.
// tests/test_tri_exit.py: grazing and adversarial exits checked against the binary64 test of every triangle.
#ifndef RT_TRI_EXIT
#define RT_TRI_EXIT 1
#endif
template <class R>
RT_HD bool leaves_tri_hull(const SceneView<R>& sc, int id, V3<R> o, V3<R> d) {
    if constexpr (sizeof(R) != 8 || RT_TRI_EXIT == 0) return false;
    else {
#if !defined(__HIP_DEVICE_COMPILE__)
        if (!sc.tri_exit) return false;         // a host view built without the bounds (the device's always has them)
#endif
        const TriRec<R>& tr = sc.tris[id];
        const double gp = tr.nx * d.x + tr.ny * d.y + tr.nz * d.z;
        const double an = tr.nx * o.x + tr.ny * o.y + tr.nz * o.z;
        const bool pos = gp > 0.0;
        const double C = sc.tri_exit[2 * id + (pos ? 0 : 1)];
        const double g = pos ? gp : -gp, a = pos ? an : -an;
        const double mo = fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z)));
        const double md = fmax(fabs(d.x), fmax(fabs(d.y), fabs(d.z)));
        const double mm = md * (mo + sc.exit_k2);
        const double bnd = sc.exit_k0 + sc.exit_k1 * mm + 0x1.8p-49 * (mo + md);      // 24 eps = 3 * 2^-50
        return mm <= sc.exit_l1 && mo <= sc.exit_l2 && (a - C) + 0.00095 * g > bnd;
    }
}

template <class R>
struct Closest { R t; int kind, idx, mat, obj; };   // obj: World.objects index (BVH mode only)

#ifndef RT_SPHERE_UNROLL
#define RT_SPHERE_UNROLL 16
#endif
#define RT_PRAGMA(x) _Pragma(#x)
#define RT_UNROLL(n) RT_PRAGMA(unroll n)

// RT_ORIGIN_LEAVE: in the binary64 lean grid kernel (config 3) the sphere a segment starts on — the one just
// hit — takes the exact leave rule (sphere_leaves: both roots below tmin, decided without the sqrt and the
// root divisions), the other spheres the plain test: only the origin sphere is one the ray can be leaving.
// Interleaved x2, RTOW 512 spp f64: 94.6-94.7 vs 94.8-95.1 ms (+0.3 %), identical images (the rule applied
// to every sphere: -0.8 %)
#ifndef RT_ORIGIN_LEAVE
#define RT_ORIGIN_LEAVE 1
#endif
#ifndef RT_LEAVE_ALL
#define RT_LEAVE_ALL 0
#endif
#ifndef RT_LEAVE_INSIDE
#define RT_LEAVE_INSIDE 1         // binary64 only (binary32 measured -0.7 %); 2 (A/B): both; 0 (A/B): round 4's away rule only
#endif
template <class R> RT_HD bool sphere_leaves(R hb, R c, R a, R tmin) {
    if (!RT_LEAVE_INSIDE || (sizeof(R) == 4 && RT_LEAVE_INSIDE == 1)) return hb >= (R)0 && c >= (R)0;
    return hb >= (R)0 &&
           (c >= (R)0 || (-c < hb * (tmin * (R)0.25) && hb * (R)(sizeof(R) == 8 ? 0x1p-45 : 0x1p-18) < a * (tmin * (R)0.25)));
}

// Sphere.hit (geometry.js:15-45) folded into World.hit's strict-< acceptance, in R arithmetic.
template <class R>
RT_HD void sphere_test_f64(const SceneView<R>& sc, V3<R> o, V3<R> d, R a, R tmin, int i, Closest<R>& b) {
    const SphereRec<R> s = sc.spheres[i];
    R ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
    R hb = ocx * d.x + ocy * d.y + ocz * d.z;
    R c = (ocx * ocx + ocy * ocy + ocz * ocz) - s.r2;
    if (RT_LEAVE_ALL && sphere_leaves<R>(hb, c, a, tmin)) return;   // both roots below tmin (pt_core.h `leave`)
    R disc = hb * hb - a * c;
    if (disc < (R)0) return;
    R sq = sqrt(disc);
    R root = (-hb - sq) / a;
    if (root < tmin || b.t < root) {
        root = (-hb + sq) / a;
        if (root < tmin || b.t < root) return;
    }
    if (root < b.t) b = Closest<R>{root, HIT_SPHERE, i, sc.sphere_mat[i]};
}

// sphere_filter_bound.  With the exact binary64 inputs o, c, d, r: DISC = |d|^2 (r^2 - p^2), p the
// line-to-centre distance, so the sign of Y = r^2 - p^2 = r^2 - |OC|^2 + (OC.n)^2 (n = d/|d|) decides.
// The filter evaluates X = (oc32.dn)^2 - |oc32|^2 + r2p + delta in binary32 (u = 2^-24) from rounded
// o, c and the normalized rounded direction dn, with r2p = r^2 + 2^-17 (2|c|^2 + r^2) and
// delta = 2^-16 |o|^2 (both rounded up).  With M_i = |o_i| + |c_i| and Q = sum M_i^2 + r^2 <=
// 2|o|^2 + 2|c|^2 + r^2: oc32 is within 2u M_i of OC per component; dn within 6.5u of n (d rounded u,
// the sum of squares 2.5u, v_rsq_f32 2u, the product u); so the three-term dot oc32.dn is within
// (2 + 6.5 + 3)u |M| of OC.n (3u: the FMA chain's roundings) and |(oc32.dn)^2 - (OC.n)^2| <= 23u Q;
// ||oc32|^2 - |OC|^2| <= 4u Q and the chain that subtracts r2p + delta rounds by <= 6u Q; the final
// FMA's rounding cannot change the sign of X.  So |X - Y - (r2p - r^2) - delta| <= 33u Q, while
// r2p - r^2 + delta >= 2^-17 Q = 128u Q (3.9x margin; 2^-18 .. 2^-20 cut the binary64 tests per RTOW
// segment by 0.3 % at most, host count: most filter survivors are real hits, or the dominant spheres'
// away-rejections).  Hence disc64 >= 0 (Y >= -2^-48 Q) implies X > 0: a rejected
// sphere (X < 0) is a sure binary64 miss.  NaN never rejects.  tests/test_sphere_filter.py checks this on
// adversarial near-tangent cases (observed worst 7.4u with a correctly rounded rsqrt).
// Approximate binary32 reciprocal / reciprocal square root (v_rcp_f32 / v_rsq_f32, <= 1 ulp) for the
// conservative binary32 pre-tests only (sphere filter direction, BVH slab 1/d): their error bounds
// (sphere_filter_bound, bvh_conservative_bound) carry margins of 4x and 16x over a correctly rounded
// one, and a +-inf / NaN result behaves as before (clamped / never rejecting).  The correctly rounded
// divisions they replace cost ~10 VALU each.  RT_FAST_RCP=0: correctly rounded (A/B).
#ifndef RT_FAST_RCP
#define RT_FAST_RCP 1
#endif
RT_HD float rt_rcp_approx(float x) {
#if RT_FAST_RCP && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
RT_HD float rt_rsqrt_approx(float x) {
#if RT_FAST_RCP && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rsqf(x);
#else
    return 1.0f / sqrtf(x);
#endif
}

struct FilterRay { float ox, oy, oz, dx, dy, dz, delta; };

template <class R>
RT_HD FilterRay make_filter_ray(V3<R> o, V3<R> d) {
    FilterRay f;
    f.ox = (float)o.x; f.oy = (float)o.y; f.oz = (float)o.z;
    const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
    const float inv = rt_rsqrt_approx(dx * dx + dy * dy + dz * dz);
    f.dx = dx * inv; f.dy = dy * inv; f.dz = dz * inv;
    f.delta = (f.ox * f.ox + f.oy * f.oy + f.oz * f.oz) * ((float)(2.0 * filter_margin()) * (1.0f + 0x1p-20f));
    return f;
}

// false only if the sphere is certainly missed in binary64 (disc64 < 0): 12 VALU per sphere
RT_HD bool sphere_filter_pass(const SphereFilter& s, const FilterRay& r) {
    RT_HCOUNT(HC_FILTER_TESTS, 1);
    const float ocx = r.ox - s.cx, ocy = r.oy - s.cy, ocz = r.oz - s.cz;
    const float hb = __builtin_fmaf(ocx, r.dx, __builtin_fmaf(ocy, r.dy, ocz * r.dz));
    const float cc = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, __builtin_fmaf(ocz, ocz, -(s.r2p + r.delta))));
    return !(__builtin_fmaf(hb, hb, -cc) < 0.0f);
}

// Scene features a trace kernel is compiled for (FEAT template arguments; the lean kernels, pt_trace.hip
// scene_lean): planes, boxes and triangles among the primitives, every background (else the sky gradient
// only), the orthographic camera and the stochastic / centre AA modes (else the perspective camera with
// supersampling).  A kernel compiled without a feature holds none of its code, nor the scene constants
// that code reads, so fewer scalars stay live across the segment loop (SGPR spills).
enum Feat : int { F_PLANES = 1, F_BOXES = 2, F_TRIS = 4, F_BGALL = 8, F_CAMALL = 16, F_ALL = 31 };

// Closest hit over the whole world: World.hit (world.js:20-33) with every object's hit() inlined.
// All lanes walk the same primitive list in the same order, so every record load — including the
// material index, taken at accept time — is wave-uniform (scalar loads, no LDS).  Only
// (t, kind, index, material) is tracked; the hit record is rebuilt afterwards from (t, primitive),
// which is exact because no primitive's chosen t depends on tMax.
template <class R, int FEAT = F_ALL>
RT_HD Closest<R> closest_hit_runs(const SceneView<R>& sc, V3<R> o, V3<R> d) {
    const R tmin = (R)0.001;
    Closest<R> b{(R)INFINITY, HIT_NONE, 0, 0};
    const R a = dot(d, d);
    for (int r = 0; r < sc.num_runs; ++r) {
        const Run run = sc.runs[r];
        if (run.kind == RUN_SPHERES) {
            if constexpr (sizeof(R) == 8) {
                // Exact mode: every sphere is first tested in binary32 with a rigorous bound E on
                // |disc32 - disc64| (sphere_filter_bound); only spheres the filter cannot reject get
                // the binary64 test below, so every decision is the f64 one, at ~f32 cost per miss.
                const FilterRay fr = make_filter_ray(o, d);
RT_UNROLL(RT_SPHERE_UNROLL)
                for (int i = run.begin; i < run.end; ++i) {
                    if (!sphere_filter_pass(sc.sphere_filter[i], fr)) continue;
                    sphere_test_f64(sc, o, d, a, tmin, i, b);
                }
                continue;
            }
#pragma unroll 2
            for (int i = run.begin; i < run.end; ++i) sphere_test_f64(sc, o, d, a, tmin, i, b);
        } else if ((FEAT & F_PLANES) != 0 && run.kind == RUN_PLANES) {
            for (int i = run.begin; i < run.end; ++i) {                       // geometry.js:56-74
                const PlaneRec<R> p = sc.planes[i];
                R denom = p.nx * d.x + p.ny * d.y + p.nz * d.z;
                if (fabs(denom) < (R)1e-6) continue;
                R t = ((p.px - o.x) * p.nx + (p.py - o.y) * p.ny + (p.pz - o.z) * p.nz) / denom;
                if (t < tmin || t > b.t) continue;
                if (t < b.t) b = Closest<R>{t, HIT_PLANE, i, sc.plane_mat[i]};
            }
        } else if ((FEAT & F_BOXES) != 0 && run.kind == RUN_BOXES) {
            for (int i = run.begin; i < run.end; ++i) {                       // geometry.js:85-117
                const BoxRec<R> bx = sc.boxes[i];
                R t0 = (bx.mnx - o.x) / d.x, t1 = (bx.mxx - o.x) / d.x;
                if (t0 > t1) { R s = t0; t0 = t1; t1 = s; }
                R ty0 = (bx.mny - o.y) / d.y, ty1 = (bx.mxy - o.y) / d.y;
                if (ty0 > ty1) { R s = ty0; ty0 = ty1; ty1 = s; }
                if (t0 > ty1 || ty0 > t1) continue;
                t0 = js_max(t0, ty0);
                t1 = js_min(t1, ty1);
                R tz0 = (bx.mnz - o.z) / d.z, tz1 = (bx.mxz - o.z) / d.z;
                if (tz0 > tz1) { R s = tz0; tz0 = tz1; tz1 = s; }
                if (t0 > tz1 || tz0 > t1) continue;
                t0 = js_max(t0, tz0);
                t1 = js_min(t1, tz1);
                R t = t0 > tmin ? t0 : t1;
                if (t < tmin || t > b.t) continue;                            // NaN passes here ...
                if (t < b.t) b = Closest<R>{t, HIT_BOX, i, sc.box_mat[i]};    // ... and fails here
            }
        } else if ((FEAT & F_TRIS) != 0) {                                    // geometry.js:148-188, 248-262
            const bool mesh = run.kind == RUN_MESH;
            R local = b.t;
            int local_idx = -1;
            for (int i = run.begin; i < run.end; ++i) {
                const TriRec<R> tr = sc.tris[i];
                // h = d x e2 ; a = e1 . h
                R hx = d.y * tr.e2z - d.z * tr.e2y, hy = d.z * tr.e2x - d.x * tr.e2z, hz = d.x * tr.e2y - d.y * tr.e2x;
                R aa = tr.e1x * hx + tr.e1y * hy + tr.e1z * hz;
                if (fabs(aa) < (R)0.0001) continue;
                R f = (R)1 / aa;
                R sx = o.x - tr.v0x, sy = o.y - tr.v0y, sz = o.z - tr.v0z;
                R u = f * (sx * hx + sy * hy + sz * hz);
                if (u < (R)0 || u > (R)1) continue;
                R qx = sy * tr.e1z - sz * tr.e1y, qy = sz * tr.e1x - sx * tr.e1z, qz = sx * tr.e1y - sy * tr.e1x;
                R v = f * (d.x * qx + d.y * qy + d.z * qz);
                if (v < (R)0 || u + v > (R)1) continue;
                R t = f * (tr.e2x * qx + tr.e2y * qy + tr.e2z * qz);
                if (t < tmin || t > local) continue;
                if (mesh) { local = t; local_idx = i; }                       // mesh: <=, last equal-t wins
                else if (t < b.t) { local = t; b = Closest<R>{t, HIT_TRI, i, sc.tri_mat[i]}; }
            }
            if (mesh && local_idx >= 0 && local < b.t) b = Closest<R>{local, HIT_TRI, local_idx, run.mat};
        }
    }
    return b;
}
template <class R>
RT_HD Closest<R> closest_hit(const SceneView<R>& sc, V3<R> o, V3<R> d) { return closest_hit_runs<R, F_ALL>(sc, o, d); }

// ---- BVH mode ---------------------------------------------------------------------------------------
// World.hit's result is the minimum of a total order over the candidates: every object's candidate t
// is independent of tMax (a sphere takes its near root if >= tMin, else its far root; the far root
// is never below the near one), World.hit accepts strictly smaller t (the first of equal t wins) and
// a mesh accepts <= (the last equal-t triangle wins, geometry.js:253-259).  So the winner is the
// least (t, World.objects index ascending, triangle index descending) — order-independent, which lets
// a BVH visit primitives in any order and stay bit-identical to the brute-force walk.  NaN
// candidates never win, nor does +inf (World.hit starts from closestT = Infinity).
template <class R>
RT_HD bool better(R t, int obj, int id, const Closest<R>& b) {
    return t < b.t || (t == b.t && (obj < b.obj || (obj == b.obj && id > b.idx)));
}

// away: reject at once a ray whose origin is outside or on the sphere (c >= 0) and that moves away from
// its centre (hb >= 0).  Exact: then disc = RN(RN(hb^2) - RN(a c)) <= RN(hb^2), and RN(sqrt(RN(hb^2)))
// = hb, so sqrt(disc) <= hb, both roots are <= 0 < tmin, and the reference's test rejects as well (NaN
// operands fail the comparisons and take the full test).  Used for the dominant spheres, which every
// ray leaving them (the RTOW ground: most secondary rays) would otherwise test in full: +0.9 %.
// leave (round 5): the same for an origin just INSIDE the sphere (c < 0, the hit point of the previous
// segment rounded inwards) moving away from the centre (hb > 0): the near root is negative and the far
// one t2 = RN(RN(-hb + sq) / a) with sq = RN(sqrt(RN(RN(hb^2) + RN(a |c|)))) <= (1+u)^2 (hb + a|c|/(2hb)),
// so t2 <= (1+u)^4 (2.01u hb / a + |c| / (2 hb)).  With |c| < hb tmin / 4 and hb 2^-45 < a tmin / 4
// (binary32: 2^-18) that is below tmin / 7: both roots fail `root < tMin`, as in the reference.  This is
// every ray leaving a sphere it was scattered from, whose second root the full test computes (RTOW: 0.46
// second roots per segment, host count).  RT_LEAVE_ALL: both rules for every sphere — measured slower
// (RTOW 256 spp f64 10261 vs 10347, f32 -1.2 %, Cornell and mesh50k +-0.5 %: the lanes that skip still wait
// for the survivor loop's other lanes), so 0: the dominant spheres (their `away` flag) only

// RT_ROOT_RCP: the roots' divisions by a = d.d as Markstein corrections from ya = RN(1/a), computed
// once per closest-hit query (the grid walk; ya = 0: the plain divisions), guarded so that every
// intermediate is normal: 2^-500 <= |-hb -+ sqrt(disc)| <= 2^500 (the caller: 2^-400 <= a <= 2^400;
// binary32: 2^-60, 2^60, 2^-40, 2^40).  0: never / 1: both precisions / 2: binary32 only (RTOW 256
// spp: f32 +2.0 %, f64 ±0 — DESIGN.md §4; bit-identical images either way)
#ifndef RT_ROOT_RCP
#define RT_ROOT_RCP 2
#endif
template <class R> constexpr bool root_rcp_on() { return RT_ROOT_RCP == 1 || (RT_ROOT_RCP == 2 && sizeof(R) == 4); }
template <class R> RT_HD R root_div(R x, R a, R ya) {
    // the same guarded corrections as vdiv_rcp (two in binary64, one in binary32)
    if (root_rcp_on<R>() && ya != (R)0 && div_rcp_range(x)) return div_rcp_1(x, a, ya);
    return x / a;
}
// RN(1/a) for root_div when a lies in its range, else 0
template <class R> RT_HD R root_rcp(R a) {
    const bool in = a >= (R)(sizeof(R) == 8 ? 0x1p-400 : 0x1p-40) && a <= (R)(sizeof(R) == 8 ? 0x1p400 : 0x1p40);
    return root_rcp_on<R>() && in ? (R)1 / a : (R)0;
}

template <class R>
RT_HD bool sphere_candidate(const SphereRec<R>& s, V3<R> o, V3<R> d, R a, R tmin, R& t, bool away = false,
                            R ya = (R)0) {   // geometry.js:15-45
    RT_HCOUNT(HC_F64_TESTS, 1);
    R ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
    R hb = ocx * d.x + ocy * d.y + ocz * d.z;
    R c = (ocx * ocx + ocy * ocy + ocz * ocz) - s.r2;
    if ((away || RT_LEAVE_ALL) && sphere_leaves<R>(hb, c, a, tmin)) return false;
    R disc = hb * hb - a * c;
    if (disc < (R)0) return false;
    RT_HCOUNT(HC_DISC_OK, 1);
    R sq = sqrt(disc);
    t = root_div(-hb - sq, a, ya);
    if (!(t < tmin)) return true;
    RT_HCOUNT(HC_SECOND_ROOT, 1);
    t = root_div(-hb + sq, a, ya);
    return !(t < tmin);
}

template <class R, class Tri>
RT_HD bool triangle_candidate(const Tri& tr, V3<R> o, V3<R> d, R tmin, R& t) {   // geometry.js:148-188
    R hx = d.y * tr.e2z - d.z * tr.e2y, hy = d.z * tr.e2x - d.x * tr.e2z, hz = d.x * tr.e2y - d.y * tr.e2x;
    R aa = tr.e1x * hx + tr.e1y * hy + tr.e1z * hz;
    if (fabs(aa) < (R)0.0001) return false;
    R f = (R)1 / aa;
    R sx = o.x - tr.v0x, sy = o.y - tr.v0y, sz = o.z - tr.v0z;
    R u = f * (sx * hx + sy * hy + sz * hz);
    if (u < (R)0 || u > (R)1) return false;
    R qx = sy * tr.e1z - sz * tr.e1y, qy = sz * tr.e1x - sx * tr.e1z, qz = sx * tr.e1y - sy * tr.e1x;
    R v = f * (d.x * qx + d.y * qy + d.z * qz);
    if (v < (R)0 || u + v > (R)1) return false;
    t = f * (tr.e2x * qx + tr.e2y * qy + tr.e2z * qz);
    return !(t < tmin);
}

// tri_filter_bound.  The binary64 test above decides through four quantities of exact inputs o, d, v0, e1,
// e2: A = e1.(d x e2) (|A| < 1e-4 rejects), X = S.(d x e2) (u = X / A), Y = d.(S x e1) (v = Y / A) and
// Z = e2.(S x e1) (t = Z / A), S = o - v0.  With C = d x S and n = e2 x e1 these are A = d.n, X = -e2.C,
// Y = e1.C, Z = -S.n: the binary32 filter evaluates those forms (21 FMA-chained ops) from o, d, v0, e1,
// e2 rounded to binary32 and n rounded from its binary64 value.  With u = 2^-24, md = |d|inf, me1 = |e1|inf,
// me2 = |e2|inf and Ms = |o|inf + |v0|inf, the rounding of every input and operation bounds the errors
// (components: |d_j S_k - d32_j S32_k| <= 3.02u md Ms, |C32_i - C_i| <= 9.1u md Ms, |n32_i - n_i| <= 2.01u
// me1 me2, three-term dot products adding u (2 + 4 + 6) of their magnitude) by
//   |A32 - A| <= 25u md me1 me2,  |X32 - X| <= 46u md me2 Ms,  |Y32 - Y| <= 46u md me1 Ms,
//   |Z32 - Z| <= 31u me1 me2 Ms,
// and the binary64 test's own values (X64 ...) lie within 46 * 2^-53 of the same magnitudes of the exact
// ones.  The filter uses E = K P with K = 80u (1.7x margin, which also covers the binary32 evaluation of
// the bounds), P the magnitude product above; Ms carries +2^-30, so no E is subnormal.  Given |A32| > Ea
// (so sign(A64) = sign(A32) = s and A64 != 0), it rejects only what the binary64 test rejects:
//   R0  |A32| + Ea < 0.99999e-4            -> |A64| < 1e-4
//   R1  s X32 < -EX                         -> u64 = RN(RN(1/A64) X64) < 0 (nonzero: |X64| >= 0.4 EX)
//   R2  s Y32 < -EY                         -> v64 < 0
//   R4  W = s X32 + s Y32 - |A32| > EX + EY + Ea + 2^-22 (|W| + |A32|)
//                                           -> X / A + Y / A >= 1 + 2^-40, so u64 > 1, v64 < 0 or u64 + v64 > 1
//   R5  G = s Z32 - T |A32|, G + 2^-22 |G| + EZ + T Ea < 0 (T = 0.00099999)
//                                           -> Z / A < T, so t64 < 0.001
//   R6  G = s Z32 - tl |A32|, G - 2^-22 |G| - EZ - tl Ea > 0 (tl = bvh_tlimit(best) >= best (1 + 2^-21))
//                                           -> t64 > best: `better` fails
// (u > 1 alone needs no test of its own: with v >= 0 it implies R4's condition, with v < 0 R2's.)  Every
// test is a comparison that fails on NaN, so NaN inputs, rays with |d|inf outside [2^-30, 2^30] or |o|inf
// above 2^30 (md = NaN) and triangles outside the same range (n = NaN, scene_pack.h) are never rejected.
// tests/test_tri_filter.py checks this on adversarial rays through edges, vertices and grazing planes.
struct TriRay { float o[3], d[3], mo, md, mdK; };

template <class R>
RT_HD TriRay make_tri_ray(V3<R> o, V3<R> d) {
    TriRay r;
    r.o[0] = (float)o.x; r.o[1] = (float)o.y; r.o[2] = (float)o.z;
    r.d[0] = (float)d.x; r.d[1] = (float)d.y; r.d[2] = (float)d.z;
    // bounds on the binary64 values' magnitudes (rounded up), plus the 2^-30 floor of Ms
    const float mo = fmaxf(fabsf(r.o[0]), fmaxf(fabsf(r.o[1]), fabsf(r.o[2]))) * (1.0f + 0x1p-22f);
    const float md = fmaxf(fabsf(r.d[0]), fmaxf(fabsf(r.d[1]), fabsf(r.d[2]))) * (1.0f + 0x1p-22f);
    const bool ok = mo <= 0x1p30f && md >= 0x1p-30f && md <= 0x1p30f;
    r.mo = mo + 0x1p-30f;
    r.md = ok ? md : NAN;
    r.mdK = r.md * 0x5p-20f;                 // K = 80u = 5 * 2^-20
    return r;
}

// false only if the binary64 test (triangle_candidate + `better` against a best whose limit is tl) certainly
// rejects the triangle: tri_filter_bound above
RT_HD bool tri_filter_pass(const TriFilter& f, const TriRay& r, float tl) {
    RT_HCOUNT(HC_TRI_FILTERS, 1);
    const float sx = r.o[0] - f.v0[0], sy = r.o[1] - f.v0[1], sz = r.o[2] - f.v0[2];
    const float cx = __builtin_fmaf(r.d[1], sz, -(r.d[2] * sy));
    const float cy = __builtin_fmaf(r.d[2], sx, -(r.d[0] * sz));
    const float cz = __builtin_fmaf(r.d[0], sy, -(r.d[1] * sx));
    const float A = __builtin_fmaf(r.d[0], f.n[0], __builtin_fmaf(r.d[1], f.n[1], r.d[2] * f.n[2]));
    const float X = __builtin_fmaf(-f.e2[0], cx, __builtin_fmaf(-f.e2[1], cy, -(f.e2[2] * cz)));
    const float Y = __builtin_fmaf(f.e1[0], cx, __builtin_fmaf(f.e1[1], cy, f.e1[2] * cz));
    const float Z = __builtin_fmaf(-sx, f.n[0], __builtin_fmaf(-sy, f.n[1], -(sz * f.n[2])));
    // the bounds: magnitudes of the record (rounded up by their products' slack), then E = K P
    const float me1 = fmaxf(fabsf(f.e1[0]), fmaxf(fabsf(f.e1[1]), fabsf(f.e1[2])));
    const float me2 = fmaxf(fabsf(f.e2[0]), fmaxf(fabsf(f.e2[1]), fabsf(f.e2[2])));
    const float m0 = fmaxf(fabsf(f.v0[0]), fmaxf(fabsf(f.v0[1]), fabsf(f.v0[2])));
    const float msk = (r.mo + m0) * 0x5p-20f, mdmsk = r.md * msk, m12 = me1 * me2;
    const float EX = me2 * mdmsk, EY = me1 * mdmsk, Ea = m12 * r.mdK, EZ = m12 * msk;
    const float aa = fabsf(A);
    const float xs = copysignf(1.0f, A) * X, ys = copysignf(1.0f, A) * Y, zs = copysignf(1.0f, A) * Z;
    const bool r0 = aa + Ea < 0.99999e-4f;
    const bool r1 = xs < -EX, r2 = ys < -EY;
    const float W = (xs + ys) - aa;
    const bool r4 = W > __builtin_fmaf(0x1p-22f, fabsf(W) + aa, (EX + EY) + Ea);
    const float G = __builtin_fmaf(-0.00099999f, aa, zs);
    const bool r5 = G + __builtin_fmaf(0x1p-22f, fabsf(G), __builtin_fmaf(0.00099999f, Ea, EZ)) < 0.0f;
    const float G2 = __builtin_fmaf(-tl, aa, zs);
    const bool r6 = G2 - __builtin_fmaf(0x1p-22f, fabsf(G2), __builtin_fmaf(tl, Ea, EZ)) > 0.0f;
    return !(r0 || (aa > Ea && (r1 || r2 || r4 || r5 || r6)));
}

// bvh_conservative_bound.  A primitive accepted at parameter t has its computed hit point within
// 2^-25 (|o| + |c|) of the primitive's bounding box (the worst case is a near-tangent sphere root,
// whose error is sqrt(u) relative), far inside the node inflation 2^-19 max|bound| (scene_pack.h)
// plus the per-ray origin pad 2^-19 |o|_inf below.  The binary32 slab test then errs by < 2^-22 of
// |bound - o| per axis (rounded o, d, 1/d and the product), which the same margins cover, and the
// ray-length limit is (float)t_best rounded up by 2^-20.  So a node holding a primitive that beats
// the current best is never culled; f64 mode stays bit-identical to the brute-force walk
// (tests/test_hostcheck.py, tests/test_gpu_parity.py).  Directions with a binary32-denormal
// component are clamped to 1/d = 2^126 (t ranges beyond 2^100 are not modelled).
// The two-child walk evaluates (lo - olo) * inv as fma(lo, inv, -olo * inv): one rounding of olo*inv
// more, an error < 2^-23 (|o| + |lo|) |inv| in t, still 16x inside the same margins.
struct BvhRay { float olo[3], ohi[3], inv[3], slo[3], shi[3]; };   // slo = olo * inv, shi = ohi * inv

template <class R>
RT_HD BvhRay make_bvh_ray(V3<R> o, V3<R> d) {
    BvhRay r;
    const float of[3] = {(float)o.x, (float)o.y, (float)o.z};
    const float df[3] = {(float)d.x, (float)d.y, (float)d.z};
    const float m = fmaxf(fabsf(of[0]), fmaxf(fabsf(of[1]), fabsf(of[2])));
    const float pad = m * (0x1p-19f * (1.0f + 0x1p-20f)) + 0x1p-100f;
    for (int k = 0; k < 3; ++k) {
        r.olo[k] = of[k] + pad;      // (lo - olo) * inv and (hi - ohi) * inv widen the slab for both signs of d
        r.ohi[k] = of[k] - pad;
        float inv = rt_rcp_approx(df[k]);
        if (!(fabsf(inv) <= 0x1p126f)) inv = copysignf(0x1p126f, df[k]);
        r.inv[k] = inv;
        r.slo[k] = r.olo[k] * inv;
        r.shi[k] = r.ohi[k] * inv;
    }
    return r;
}

template <class R>
RT_HD float bvh_tlimit(R t) {   // >= t, +inf while nothing was hit
    return (float)t * (1.0f + 0x1p-20f);
}

RT_HD bool bvh_node_hit(const BvhNode& n, const BvhRay& r, float tlimit) {
    const float x0 = (n.lo[0] - r.olo[0]) * r.inv[0], x1 = (n.hi[0] - r.ohi[0]) * r.inv[0];
    const float y0 = (n.lo[1] - r.olo[1]) * r.inv[1], y1 = (n.hi[1] - r.ohi[1]) * r.inv[1];
    const float z0 = (n.lo[2] - r.olo[2]) * r.inv[2], z1 = (n.hi[2] - r.ohi[2]) * r.inv[2];
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tlimit));
    return tn <= tf;
}

struct Work {
    uint32_t nodes, spheres, tris;                // BVH nodes visited, sphere / triangle tests (stats)
    uint32_t lane_trips, wave_trips, uni_trips;   // RT_PROFILE: walk iterations per lane / per wave / uniform
    uint32_t low8, low16;                         // RT_PROFILE: wave iterations with <= 8 / <= 16 lanes walking
};
#ifndef RT_BVH_COUNT
#define RT_BVH_COUNT 1            // 0 measured slower (-2 % RTOW, -9 % mesh50k: worse register allocation)
#endif
#if RT_BVH_COUNT
#define RT_COUNT(x) (x)
#else
#define RT_COUNT(x) ((void)0)
#endif

typedef float rt_f2 __attribute__((ext_vector_type(2)));
typedef unsigned int rt_u2 __attribute__((ext_vector_type(2)));
typedef unsigned int rt_u4 __attribute__((ext_vector_type(4)));

// per-lane traversal stack of the ordered walk: entry k of this lane at base[k * stride] (LDS on the
// GPU, strided by the workgroup size so a wave's accesses are conflict-free).  box / kid: the sphere
// tree's nodes copied to LDS (ACC_BVH_SPHERES_LDS): node i's child boxes at box[3i .. 3i+2], its child
// references at kid[i]
// gcell / grec: the grid's cell offsets and records copied to LDS (ACC_GRID_LDS): binary64 keeps the
// 16-B binary32 filters there (the rest of a record is read from grid_leaf by filter survivors only),
// binary32 the whole 32-B records (grec[2k], grec[2k + 1])
// the triangle tree's breadth-first prefix (scene_pack.h make_wide): at most this many of its top nodes
// are staged in LDS (ACC_BVH_TRI_LDS; 1023 = nine full levels and half the tenth)
#ifndef RT_TRI_TOP_NODES
#define RT_TRI_TOP_NODES 1023
#endif
// ntop (ACC_BVH_TRI_LDS): box / kid hold the triangle tree's first ntop nodes (its breadth-first top
// levels, scene_pack.h make_wide); nodes from ntop on are read from global memory
struct BvhStack {
    int* base; int stride; const rt_u4* box = nullptr; const rt_u2* kid = nullptr;
    const int* gcell = nullptr; const rt_u4* grec = nullptr;
    int ntop = 0;
};

#if defined(__HIP_DEVICE_COMPILE__)
// IEEE 754-2019 minimum / maximum (v_minimum3_f32 / v_maximum3_f32 on gfx950): unlike fminf / fmaxf
// they need no canonicalized inputs, so the loop-carried ray limit is not re-canonicalized at every
// node.  They differ from fminf / fmaxf only for NaN operands (propagated instead of dropped: a NaN
// ray then enters no node, and no leaf could have given it a hit) and in ordering -0 below +0 (equal
// under the <= / < tests below): same decisions
#define RT_SLAB_MIN(a, b) __builtin_elementwise_minimum(a, b)
#define RT_SLAB_MAX(a, b) __builtin_elementwise_maximum(a, b)
#else
#define RT_SLAB_MIN(a, b) fminf(a, b)
#define RT_SLAB_MAX(a, b) fmaxf(a, b)
#endif

// Both children of a two-child node: (lo - olo) * inv as fma(lo, inv, -olo * inv), the pair of
// children at once as packed FMAs (v_pk_fma_f32): 6 per node.
RT_HD void bvh_node2_hit(const Bvh2Node& n, const BvhRay& r, float tlimit, bool& h0, bool& h1, float& t0,
                         float& t1) {
    rt_f2 a[3], b[3];
    for (int k = 0; k < 3; ++k) {
        const rt_f2 inv = {r.inv[k], r.inv[k]};
        const rt_f2 slo = {-r.slo[k], -r.slo[k]}, shi = {-r.shi[k], -r.shi[k]};
        a[k] = __builtin_elementwise_fma(rt_f2{n.lo[k][0], n.lo[k][1]}, inv, slo);
        b[k] = __builtin_elementwise_fma(rt_f2{n.hi[k][0], n.hi[k][1]}, inv, shi);
    }
#define MN RT_SLAB_MIN
#define MX RT_SLAB_MAX
    t0 = MX(MX(MN(a[0].x, b[0].x), MN(a[1].x, b[1].x)), MX(MN(a[2].x, b[2].x), 0.0f));
    t1 = MX(MX(MN(a[0].y, b[0].y), MN(a[1].y, b[1].y)), MX(MN(a[2].y, b[2].y), 0.0f));
    const float f0 = MN(MN(MX(a[0].x, b[0].x), MX(a[1].x, b[1].x)), MN(MX(a[2].x, b[2].x), tlimit));
    const float f1 = MN(MN(MX(a[0].y, b[0].y), MX(a[1].y, b[1].y)), MN(MX(a[2].y, b[2].y), tlimit));
#undef MN
#undef MX
    h0 = t0 <= f0;
    h1 = t1 <= f1;
}

#if defined(__HIP_DEVICE_COMPILE__)
// node i behind a raw buffer descriptor: 32-bit offsets, no 64-bit address arithmetic per node
// (RTOW +1.4 %, f32 +2 %)
__device__ __forceinline__ Bvh2Node load_node(__amdgpu_buffer_rsrc_t rs, int i) {
    const int off = i * (int)sizeof(Bvh2Node);
    rt_u4 q[sizeof(Bvh2Node) / 16];
    for (int k = 0; k < (int)(sizeof(Bvh2Node) / 16); ++k) q[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * k, 0, 0);
    Bvh2Node n;
    memcpy(&n, q, sizeof n);
    return n;
}
#endif

// node i from its LDS copy (three 16-B box reads, one 8-B reference read)
RT_HD Bvh2Node load_node_lds(const BvhStack& s, int i) {
    rt_u4 q[4];
    q[0] = s.box[3 * i];
    q[1] = s.box[3 * i + 1];
    q[2] = s.box[3 * i + 2];
    const rt_u2 k = s.kid[i];
    q[3] = rt_u4{k.x, k.y, 0u, 0u};
    Bvh2Node n;
    memcpy(&n, q, sizeof n);
    return n;
}

// Walk one BVH and call leaf(fc) for every leaf whose box the ray reaches before the current best.
// WIDE: ordered walk over Bvh2Node (both child boxes per 64-B node, nearer child first, the other
// pushed on the lane's stack); otherwise the stackless preorder walk over BvhNode skip links (A/B and
// host cross-check).  Variants measured slower and removed: postponed leaves,
// "while-while" leaf batching, binary16 child boxes, four-child nodes, stack top in a register, leaf
// records as buffer loads.
// LDSN: 0 every node from global memory; 1 every node from the LDS copy in stk (the sphere tree,
// ACC_BVH_SPHERES_LDS); 2 nodes [0, stk.ntop) from the LDS copy, the others from global memory (the
// triangle tree's top levels, ACC_BVH_TRI_LDS).  Wave-uniform steps read the node with scalar loads in
// every mode.
template <bool WIDE, int LDSN = 0, class Leaf>
RT_HD void bvh_walk(const BvhNode* nodes, int count, const Bvh2Node* wide, const BvhRay& br, const float& tl,
                    BvhStack stk, Work& w, Leaf&& leaf) {
    if constexpr (WIDE) {
        int sp = 0, cur = 0;
#if defined(__HIP_DEVICE_COMPILE__)
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)wide, (short)0, 0x7FFFFFFF, 0x00020000);
#endif
        // true: descend to the new cur
        auto step = [&](const Bvh2Node& n) -> bool {
            float t0, t1;
            bool h0, h1;
            bvh_node2_hit(n, br, tl, h0, h1, t0, t1);
            // branch-free child selection: the child indices are consumed by selects ahead of any
            // branch, so their loads issue with the box loads (no dependent round trip after the
            // slab test).  Near child = child 1 iff h1 and (!h0 or t1 < t0), written as plain mask
            // logic: the compiler keeps it in SGPR masks (3 scalar ops) instead of materializing
            // booleans in VGPRs (7 vector ops per node; RTOW +2.7 %)
            const int c0 = n.child[0], c1 = n.child[1];
            const bool take1 = h1 & (!h0 | (t1 < t0));
            const int near_c = take1 ? c1 : c0, far_c = take1 ? c0 : c1;
            if (h0 && h1) stk.base[(sp++) * stk.stride] = far_c;
            cur = (h0 | h1) ? near_c : cur;
            return h0 | h1;
        };
        for (;;) {
#if RT_PROFILE && defined(__HIP_DEVICE_COMPILE__)
            ++w.lane_trips;                       // the first active lane counts the wave's iteration
            const int act = __popcll(__ballot(1));
            if ((int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) {
                ++w.wave_trips;
                if (act <= 8) ++w.low8;
                if (act <= 16) ++w.low16;
            }
            {   // iterations in which every active lane is at the same inner node
                const int first = __builtin_amdgcn_readfirstlane(cur);
                const bool uni = __ballot(cur != first) == 0 && first >= 0;
                if (uni && (int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) ++w.uni_trips;
            }
#endif
            bool down = false;
            if (cur >= 0) {
                RT_COUNT(++w.nodes);
#if defined(__HIP_DEVICE_COMPILE__)
                // every active lane at the same node (30 % of RTOW walk steps, 49 % on mesh50k): read
                // it with scalar loads, which bypass the vector memory pipeline (+3.5 %)
                const int first = __builtin_amdgcn_readfirstlane(cur);
                if constexpr (LDSN == 1) down = __ballot(cur != first) == 0 ? step(wide[first]) : step(load_node_lds(stk, cur));
                else if constexpr (LDSN == 2) {
                    if (__ballot(cur != first) == 0) {
                        down = step(wide[first]);
                    } else {
                        Bvh2Node n;                   // one slab test for both sources
                        if (cur < stk.ntop) n = load_node_lds(stk, cur);
                        else n = load_node(wrs, cur);
                        down = step(n);
                    }
                } else down = __ballot(cur != first) == 0 ? step(wide[first]) : step(load_node(wrs, cur));
#else
                down = step(LDSN == 1 || (LDSN == 2 && cur < stk.ntop) ? load_node_lds(stk, cur) : wide[cur]);
#endif
                if (down) continue;
            } else {
                leaf(~cur);      // (scalar leaf reads for wave-uniform leaves measured 2 % slower)
            }
            if (sp == 0) break;
            cur = stk.base[(--sp) * stk.stride];
        }
    } else {
        int ni = 0;
        while (ni < count) {
            const BvhNode n = nodes[ni];
            RT_COUNT(++w.nodes);
            if (!bvh_node_hit(n, br, tl)) { ni = n.skip; continue; }
            if (n.fc == 0) { ++ni; continue; }
            ni = n.skip;
            leaf(n.fc);
        }
    }
}

// Planes and boxes (usually few, often large) brute force, with their World.objects index.
template <class R, int FEAT = F_ALL>
RT_HD void brute_planes_boxes(const SceneView<R>& sc, V3<R> o, V3<R> d, R tmin, Closest<R>& b) {
    if constexpr ((FEAT & F_PLANES) != 0)
    for (int i = 0; i < sc.num_planes; ++i) {                                 // geometry.js:56-74
        const PlaneRec<R> p = sc.planes[i];
        R denom = p.nx * d.x + p.ny * d.y + p.nz * d.z;
        if (fabs(denom) < (R)1e-6) continue;
        R t = ((p.px - o.x) * p.nx + (p.py - o.y) * p.ny + (p.pz - o.z) * p.nz) / denom;
        if (t < tmin) continue;
        const int obj = sc.plane_obj[i];
        if (better(t, obj, i, b)) b = Closest<R>{t, HIT_PLANE, i, sc.plane_mat[i], obj};
    }
    if constexpr ((FEAT & F_BOXES) != 0)
    for (int i = 0; i < sc.num_boxes; ++i) {                                  // geometry.js:85-117
        const BoxRec<R> bx = sc.boxes[i];
        R t0 = (bx.mnx - o.x) / d.x, t1 = (bx.mxx - o.x) / d.x;
        if (t0 > t1) { R s = t0; t0 = t1; t1 = s; }
        R ty0 = (bx.mny - o.y) / d.y, ty1 = (bx.mxy - o.y) / d.y;
        if (ty0 > ty1) { R s = ty0; ty0 = ty1; ty1 = s; }
        if (t0 > ty1 || ty0 > t1) continue;
        t0 = js_max(t0, ty0);
        t1 = js_min(t1, ty1);
        R tz0 = (bx.mnz - o.z) / d.z, tz1 = (bx.mxz - o.z) / d.z;
        if (tz0 > tz1) { R s = tz0; tz0 = tz1; tz1 = s; }
        if (t0 > tz1 || tz0 > t1) continue;
        t0 = js_max(t0, tz0);
        t1 = js_min(t1, tz1);
        R t = t0 > tmin ? t0 : t1;
        if (t < tmin) continue;
        const int obj = sc.box_obj[i];
        if (better(t, obj, i, b)) b = Closest<R>{t, HIT_BOX, i, sc.box_mat[i], obj};
    }
}

// Sphere records [first, end) of `recs` (a BVH leaf, or the dominant spheres) against the current best.
template <class R>
RT_HD void sphere_records(const SphereLeaf<R>* recs, int first, int end, V3<R> o, V3<R> d, R a, const FilterRay& fr,
                          R tmin, Closest<R>& b, float& tl, Work& w, bool away = false, R ya = (R)0) {
    RT_COUNT(w.spheres += end - first);
    for (int k = first; k < end; ++k) {
        const SphereLeaf<R> L = recs[k];
        if constexpr (sizeof(R) == 8)
            if (!sphere_filter_pass(L.f, fr)) continue;
        R t;
        if (!sphere_candidate(L.s, o, d, a, tmin, t, away, ya)) continue;
        if (better(t, L.obj, L.id, b)) {
            RT_HCOUNT(HC_ACCEPT, 1);
            b = Closest<R>{t, HIT_SPHERE, L.id, L.mat, L.obj};
            tl = bvh_tlimit(b.t);
        }
    }
}

// The primitives of one BVH leaf (fc = (first << 4) | count) against the current best.
template <class R>
RT_HD void sphere_leaf(const SceneView<R>& sc, int fc, V3<R> o, V3<R> d, R a, const FilterRay& fr, R tmin,
                       Closest<R>& b, float& tl, Work& w) {
    sphere_records(sc.bvh_sphere_leaf, fc >> 4, (fc >> 4) + (fc & 15), o, d, a, fr, tmin, b, tl, w);
}

template <class R>
RT_HD void tri_leaf(const SceneView<R>& sc, int fc, V3<R> o, V3<R> d, R tmin, Closest<R>& b, float& tl, Work& w) {
    const int first = fc >> 4, end = first + (fc & 15);
    RT_COUNT(w.tris += end - first);
    for (int k = first; k < end; ++k) {
        const TriLeaf<R> L = sc.bvh_tri_leaf[k];
        R t;
        RT_HCOUNT(HC_TRI_TESTS, 1);
        if (!triangle_candidate(L.t, o, d, tmin, t)) continue;
        if (better(t, L.obj, L.id, b)) {
            b = Closest<R>{t, HIT_TRI, L.id, sc.tri_mat[L.id], L.obj};
            tl = bvh_tlimit(b.t);
        }
    }
}

// RT_TRI_FILTER (binary64): a leaf's triangles first through the binary32 pre-filter (48-B records,
// tri_filter_bound) into a mask of survivors, then the binary64 test over the survivors only, reading
// their 80-B records — the mirror of the sphere survivor masks (RT_GRID_COMPACT).  Same decisions as
// tri_leaf (the filter rejects only what the binary64 test rejects; `better` is a total order, so the
// survivors' order does not matter).  0: every triangle through the binary64 test.
// Round 5: +1.5 % on config 5.  Since the exit skip (tri_exit_bound) the walks left are the camera and
// ground rays that reach the mesh, and the filter no longer pays: mesh50k 256 spp f64 kernel time 58.7–59.0
// without it vs 59.4–59.8 ms (interleaved x2, identical images), so it is off by default (1: A/B).
#ifndef RT_TRI_FILTER
#define RT_TRI_FILTER 0
#endif
template <class R>
RT_HD void tri_leaf_filtered(const SceneView<R>& sc, int fc, const TriRay& tr, V3<R> o, V3<R> d, R tmin,
                             Closest<R>& b, float& tl, Work& w) {
    const int first = fc >> 4, n = fc & 15;
    RT_COUNT(w.tris += n);
    uint32_t pass = 0;
    for (int i = 0; i < n; ++i)
        if (tri_filter_pass(sc.tri_filter[first + i], tr, tl)) pass |= 1u << i;
    while (pass) {
        const int k = first + __builtin_ctz(pass);
        pass &= pass - 1;
        const TriLeaf<R> L = sc.bvh_tri_leaf[k];
        R t;
        RT_HCOUNT(HC_TRI_TESTS, 1);
        if (!triangle_candidate(L.t, o, d, tmin, t)) continue;
        if (better(t, L.obj, L.id, b)) {
            b = Closest<R>{t, HIT_TRI, L.id, sc.tri_mat[L.id], L.obj};
            tl = bvh_tlimit(b.t);
        }
    }
}

// Closest hit through the BVHs: planes and boxes brute force first (their t shortens the walks),
// then the sphere BVH and the triangle BVH.  Lanes walk their own paths (per-lane node loads); leaf
// records are contiguous in leaf order.  WIDE: the ordered two-child walk (default); else the
// stackless preorder walk.
// TRI = false (ACC_BVH_SPHERES): scenes without triangles; the triangle walk's code is left out.
// LDSN: the sphere tree's nodes are read from their LDS copy in stk (ACC_BVH_SPHERES_LDS).
// TLDS: the triangle tree's top levels are read from their LDS copy in stk (ACC_BVH_TRI_LDS).
template <class R, bool WIDE, bool TRI = true, bool LDSN = false, bool TLDS = false, int FEAT = F_ALL>
RT_HD Closest<R> closest_hit_bvh(const SceneView<R>& sc, V3<R> o, V3<R> d, Work& w, BvhStack stk, bool skip_tri = false) {
    const R tmin = (R)0.001;
    Closest<R> b{(R)INFINITY, HIT_NONE, 0, 0, -1};
    brute_planes_boxes<R, FEAT>(sc, o, d, tmin, b);
    const BvhRay br = make_bvh_ray(o, d);
    float tl = bvh_tlimit(b.t);
    if (sc.num_sphere_nodes > 0 || sc.num_big_spheres > 0) {
        const R a = dot(d, d);
        FilterRay fr{};
        if constexpr (sizeof(R) == 8) fr = make_filter_ray(o, d);
        // dominant spheres first: their hit bounds the walk (scene_pack.h peel_big_spheres)
        if (sc.num_big_spheres > 0) sphere_records(sc.big_spheres, 0, sc.num_big_spheres, o, d, a, fr, tmin, b, tl, w, true);
        auto leaf = [&](int fc) { sphere_leaf(sc, fc, o, d, a, fr, tmin, b, tl, w); };
        if (sc.num_sphere_nodes > 0)
            bvh_walk<WIDE, LDSN ? 1 : 0>(sc.sphere_nodes, sc.num_sphere_nodes, sc.sphere_wide, br, tl, stk, w, leaf);
    }
    if (TRI && sc.num_tri_nodes > 0 && !skip_tri) {
        if constexpr (sizeof(R) == 8 && RT_TRI_FILTER != 0) {
            const TriRay tr = make_tri_ray(o, d);
            auto leaf = [&](int fc) { tri_leaf_filtered(sc, fc, tr, o, d, tmin, b, tl, w); };
            bvh_walk<WIDE, TLDS ? 2 : 0>(sc.tri_nodes, sc.num_tri_nodes, sc.tri_wide, br, tl, stk, w, leaf);
        } else {
            auto leaf = [&](int fc) { tri_leaf(sc, fc, o, d, tmin, b, tl, w); };
            bvh_walk<WIDE, TLDS ? 2 : 0>(sc.tri_nodes, sc.num_tri_nodes, sc.tri_wide, br, tl, stk, w, leaf);
        }
    }
    return b;
}

// Closest hit through the uniform grid (sphere-only scenes): planes and boxes brute force, the dominant
// spheres, then the cells the ray crosses in order of t (3D-DDA in binary32), every sphere registered
// in a cell tested as in a BVH leaf, until the best hit lies before the exit of the current cell.
// grid_bound: a sphere is registered in every cell its box, padded by m (scene_pack.h build_grid),
// overlaps.  The DDA's cells cover the parameter range [t0, T] it has walked without gaps (each cell's
// entry is its predecessor's computed exit), and the exact ray point at any t of a cell's computed
// interval lies within e <= 2^-19 (|o|_inf + B) of that cell (B: the grid's coordinate bound; binary32
// origin, boundary and product roundings, approximate reciprocal), so any sphere hit at t' <= T in
// binary64 is registered in a cell already walked when m >= e: build_grid sets m = 2^-12 (B + extent)
// and grid_far = 2^6 (B + extent) bounds |o|_inf, so e <= 2^-19 (2^6 + 1) (B + extent) < m
// (scene_pack.h kGridMargin / kGridFar, static_assert there) (rays from farther away
// test every sphere).  The walk stops when the best t is below the current cell's exit, so a sphere
// reaching the best t exactly (a tie that World.hit's order decides) is still tested.  The closest hit
// is therefore World.hit's, as for the BVH (tests/test_hostcheck.py, tests/test_gpu_parity.py).
// RT_GRID_UNIFORM: cells that every active lane shares read through scalar loads — binary32 only (RTOW
// 256 spp: f32 +0.6 %, f64 −0.8 %); 0 / 1: never / both precisions (A/B)
#ifndef RT_GRID_UNIFORM
#define RT_GRID_UNIFORM 2
#endif
#ifndef RT_GRID_DIV
#define RT_GRID_DIV 0
#endif
// Grid records [first, end) read from their LDS copy (ACC_GRID_LDS): binary64 tests the binary32 filter
// from LDS and reads the rest of the record from recs only when it passes; binary32 reads the whole
// record from LDS.  The same tests in the same order as sphere_records: same hits, same bits.
// RT_GRID_COMPACT (binary64): a cell's records are filtered first, 32 at a time, into a per-lane mask of
// survivors, and the binary64 tests then run over each lane's survivors: lanes whose survivors sit at
// different positions of their cells run the binary64 test together instead of each in its own record
// iteration.  The order of the tests within a cell does not matter (`better` is a total order).
#ifndef RT_GRID_COMPACT
#define RT_GRID_COMPACT 1
#endif
template <class R>
RT_HD void sphere_records_lds(const rt_u4* lrec, const SphereLeaf<R>* recs, int first, int end, V3<R> o, V3<R> d,
                              R a, const FilterRay& fr, R tmin, Closest<R>& b, float& tl, Work& w, R ya = (R)0,
                              int origin = -1) {
    RT_COUNT(w.spheres += end - first);
    if constexpr (sizeof(R) == 8 && RT_GRID_COMPACT != 0) {
        for (int base = first; base < end; base += 32) {
            const int n = end - base < 32 ? end - base : 32;
            uint32_t pass = 0;
            for (int i = 0; i < n; ++i) {                // (unrolled x2 / x4: -1.0 / -3.5 %)
                const rt_u4 q = lrec[base + i];
                SphereFilter f;
                memcpy(&f, &q, sizeof f);
                if (sphere_filter_pass(f, fr)) pass |= 1u << i;
            }
            while (pass) {
                const int k = base + __builtin_ctz(pass);
                pass &= pass - 1;
                const SphereRec<R> s = recs[k].s;
                const int id = recs[k].id, obj = recs[k].obj, mat = recs[k].mat;
                R t;
                // RT_ORIGIN_LEAVE: the sphere the segment starts on takes the exact leave rule (sphere_leaves)
                if (!sphere_candidate(s, o, d, a, tmin, t, RT_ORIGIN_LEAVE && id == origin, ya)) continue;
                if (better(t, obj, id, b)) {
                    RT_HCOUNT(HC_ACCEPT, 1);
                    b = Closest<R>{t, HIT_SPHERE, id, mat, obj};
                    tl = bvh_tlimit(b.t);
                }
            }
        }
        return;
    }
    for (int k = first; k < end; ++k) {
        SphereRec<R> s;
        int id, obj, mat;
        if constexpr (sizeof(R) == 8) {
            const rt_u4 q = lrec[k];
            SphereFilter f;
            memcpy(&f, &q, sizeof f);
            if (!sphere_filter_pass(f, fr)) continue;
            s = recs[k].s;
            id = recs[k].id; obj = recs[k].obj; mat = recs[k].mat;
        } else {
            const rt_u4 q0 = lrec[2 * k], q1 = lrec[2 * k + 1];
            memcpy(&s, &q0, sizeof s);
            id = (int)q1.x; obj = (int)q1.y; mat = (int)q1.z;
        }
        R t;
        if (!sphere_candidate(s, o, d, a, tmin, t, false, ya)) continue;
        if (better(t, obj, id, b)) {
            RT_HCOUNT(HC_ACCEPT, 1);
            b = Closest<R>{t, HIT_SPHERE, id, mat, obj};
            tl = bvh_tlimit(b.t);
        }
    }
}

// The grid's LDS copy (ACC_GRID_LDS): record k's binary32 filter (binary64) or whole record (binary32)
// at grec, the cell offsets at gcell; lanes t, t + threads, ... of a workgroup copy their share
template <class R>
RT_HD size_t grid_lds_rec_bytes(const SceneView<R>& sc) { return (size_t)sc.num_grid_recs * (sizeof(R) == 8 ? 16 : 32); }
template <class R>
RT_HD size_t grid_lds_bytes(const SceneView<R>& sc) {
    return grid_lds_rec_bytes(sc) + 4 * (size_t)(sc.num_grid_cells + 1);
}
template <class R>
RT_HD void copy_grid_lds(const SceneView<R>& sc, rt_u4* grec, int* gcell, int t, int threads) {
    const rt_u4* g = reinterpret_cast<const rt_u4*>(sc.grid_leaf);
    for (int k = t; k < sc.num_grid_recs; k += threads) {
        if constexpr (sizeof(R) == 8) grec[k] = g[4 * k];               // the 16-B filter of a 64-B record
        else { grec[2 * k] = g[2 * k]; grec[2 * k + 1] = g[2 * k + 1]; }
    }
    for (int k = t; k <= sc.num_grid_cells; k += threads) gcell[k] = sc.grid_cell[k];
}

// The grid's walk parameters as the walk reads them (SceneView grid_n .. grid_far)
struct GridRefs { const int* n; const float *lo, *hi, *cs, *ics; float far; };

// LDSG: the cell offsets and records come from their LDS copy in stk (ACC_GRID_LDS)
// FEAT: the scene features compiled in (Feat; the grid's lean kernel: spheres only)
// LOCAL: sc is a local copy (closest_hit_acc's kernel-argument reload): its axis-indexed reads are
// selects, not a private array indexed per lane
template <class R, bool LDSG = false, int FEAT = F_ALL, bool LOCAL = false>
RT_HD Closest<R> closest_hit_grid(const SceneView<R>& sc, V3<R> o, V3<R> d, Work& w, const BvhStack& stk, int origin = -1) {
    const R tmin = (R)0.001;
    Closest<R> b{(R)INFINITY, HIT_NONE, 0, 0, -1};
    brute_planes_boxes<R, FEAT>(sc, o, d, tmin, b);
    float tl = bvh_tlimit(b.t);
    const R a = dot(d, d), ya = root_rcp(a);
    FilterRay fr{};
    if constexpr (sizeof(R) == 8) fr = make_filter_ray(o, d);
    if (sc.num_big_spheres > 0) sphere_records(sc.big_spheres, 0, sc.num_big_spheres, o, d, a, fr, tmin, b, tl, w, true, ya);
    if (sc.num_grid_cells <= 0) return b;
    const GridRefs gp{sc.grid_n, sc.grid_lo, sc.grid_hi, sc.grid_cs, sc.grid_ics, sc.grid_far};
    auto at = [](const auto* a, int k) {
        if constexpr (LOCAL) return k == 0 ? a[0] : (k == 1 ? a[1] : a[2]);
        else return a[k];
    };
    const float of[3] = {(float)o.x, (float)o.y, (float)o.z};
    const float df[3] = {(float)d.x, (float)d.y, (float)d.z};
    if (!(fmaxf(fabsf(of[0]), fmaxf(fabsf(of[1]), fabsf(of[2]))) <= gp.far)) {
        // far origin (or NaN): every grid sphere once, in cell order (duplicates are harmless)
        sphere_records(sc.grid_leaf, 0, sc.grid_cell[sc.num_grid_cells], o, d, a, fr, tmin, b, tl, w);
        return b;
    }
    float inv[3], t0 = 0.0f, t1 = tl;
    for (int k = 0; k < 3; ++k) {
        float v = rt_rcp_approx(df[k]);
        if (!(fabsf(v) <= 0x1p126f)) v = copysignf(0x1p126f, df[k]);
        inv[k] = v;
        const float ta = (gp.lo[k] - of[k]) * v, tb = (gp.hi[k] - of[k]) * v;
        t0 = fmaxf(t0, fminf(ta, tb));
        t1 = fminf(t1, fmaxf(ta, tb));
    }
    if (!(t0 <= t1)) return b;
    int cell[3], step[3];
    float tmax[3];
    for (int k = 0; k < 3; ++k) {
        const float p = of[k] + t0 * df[k];
        // the entry cell: binary32 through the rounded reciprocal (a cell index off by one at a boundary
        // leaves p within 2^-22 of the grid's extent of the chosen cell, inside grid_bound's margin;
        // RTOW f32 +2.7 %); binary64 keeps the correctly rounded division, which measured 3 % faster
        // there (register allocation).  RT_GRID_DIV: 1 division / 2 reciprocal in both (A/B)
        const bool by_div = RT_GRID_DIV == 1 || (RT_GRID_DIV == 0 && sizeof(R) == 8);
        int c = by_div ? (int)floorf((p - gp.lo[k]) / gp.cs[k])
                       : (int)floorf((p - gp.lo[k]) * gp.ics[k]);
        c = c < 0 ? 0 : (c >= gp.n[k] ? gp.n[k] - 1 : c);
        cell[k] = c;
        step[k] = df[k] > 0.0f ? 1 : (df[k] < 0.0f ? -1 : 0);
        tmax[k] = step[k] == 0 ? INFINITY
                               : (gp.lo[k] + (float)(c + (step[k] > 0)) * gp.cs[k] - of[k]) * inv[k];
    }
    for (;;) {
        RT_COUNT(++w.nodes);
        const int ci = cell[0] + gp.n[0] * (cell[1] + gp.n[1] * cell[2]);
        if constexpr (LDSG) {
            sphere_records_lds(stk.grec, sc.grid_leaf, stk.gcell[ci], stk.gcell[ci + 1], o, d, a, fr, tmin, b, tl, w, ya, origin);
        } else {
#if RT_GRID_UNIFORM && defined(__HIP_DEVICE_COMPILE__)
        // every active lane in one cell: its range and records through scalar loads
        const int first = __builtin_amdgcn_readfirstlane(ci);
        if ((RT_GRID_UNIFORM == 1 || sizeof(R) == 4) && __ballot(ci != first) == 0)
            sphere_records(sc.grid_leaf, sc.grid_cell[first], sc.grid_cell[first + 1], o, d, a, fr, tmin, b, tl, w);
        else
#endif
        sphere_records(sc.grid_leaf, sc.grid_cell[ci], sc.grid_cell[ci + 1], o, d, a, fr, tmin, b, tl, w);
        }
        const int ax = tmax[0] <= tmax[1] ? (tmax[0] <= tmax[2] ? 0 : 2) : (tmax[1] <= tmax[2] ? 1 : 2);
        const float tx = tmax[ax];
        // the best hit lies before this cell's exit; or the ray never leaves this cell at a finite t
        // (zero / NaN direction; t beyond binary32's range is not modelled, as for the BVH)
        if (b.t < (R)tx || !(tx < INFINITY)) break;
        const int nc = cell[ax] + step[ax];
        if (nc < 0 || nc >= at(gp.n, ax)) break;
        cell[ax] = nc;
        tmax[ax] = (at(gp.lo, ax) + (float)(nc + (step[ax] > 0)) * at(gp.cs, ax) - of[ax]) * inv[ax];
    }
    return b;
}

// acceleration modes of the trace kernel
// ACC_BVH_SPHERES: the ordered walk for scenes without triangles (sphere tree + planes/boxes only): the
// kernel then holds no triangle-test code, and its binary64 form fits 5 waves/SIMD (RTOW +1.7 %)
// ACC_BVH_SPHERES_LDS: the same walk with the sphere tree's nodes in LDS (trace_pool_lds_kernel)
// ACC_GRID: sphere-only scenes through the uniform grid (closest_hit_grid)
// ACC_GRID_LDS: the same walk with the grid's cell offsets and records (binary64: their filters) in LDS
// ACC_BVH_TRI_LDS: the general ordered walk (scenes with triangles) with the triangle tree's top levels in
// LDS (trace_pool_lds_kernel's persistent multi-wave workgroups, round 6)
enum Accel : int { ACC_BRUTE = 0, ACC_BRUTE_LEAN = 1, ACC_BVH = 2, ACC_BVH_STACK = 3, ACC_BVH_SPHERES = 4, ACC_BVH_SPHERES_LDS = 5,
                   ACC_GRID = 6, ACC_GRID_LDS = 7, ACC_BVH_TRI_LDS = 8, ACC_GRID_LDS_LEAN = 9,
                   ACC_BVH_STACK_LEAN = 10 };
// The lean kernels (pt_trace.hip scene_feat): compiled for the common scene shapes only, the sky
// gradient, the perspective camera and supersampling AA —
//   ACC_GRID_LDS_LEAN: ACC_GRID_LDS for spheres alone (no planes, boxes or triangles; RTOW);
//   ACC_BVH_STACK_LEAN: ACC_BVH_STACK without boxes (spheres, planes, triangles; config 5)
//   ACC_BRUTE_LEAN: World order for spheres and planes (config 2's Cornell box)
template <int ACC> constexpr int feat_of() {
    return ACC == ACC_GRID_LDS_LEAN ? 0 : ACC == ACC_BVH_STACK_LEAN ? (F_PLANES | F_TRIS)
         : ACC == ACC_BRUTE_LEAN ? F_PLANES : F_ALL;
}

// RT_SC_RELOAD (bit mask of lean kernels: 1 tree, 2 grid, 4 brute force; default 2): the closest-hit
// query's scene fields read from the kernel-argument segment at every query (a copy the compiler cannot
// hoist) instead of kept in SGPRs across the segment loop, whose spills it reloads there by VALU
// v_readlane.  Binary64 only.  Config 3's binary64 grid kernel, with RT_CAM_RELOAD_LEAN64: SGPR spills
// 55 -> 28, the segment loop's static v_readlanes 24 -> 4, same speed (11,170 vs 11,155 Msamples/s,
// interleaved); measured and not taken: the tree and brute-force kernels (mesh50k -10 %,
// Cornell -3.5 %: their waves then wait on the scalar loads, where a v_readlane costs one VALU slot), and
// binary32 (-1.5 %).  The kernels that instantiate the lean ACCs take the SceneView at offset 0 of their
// arguments (static_asserts in pt_trace.hip).
#ifndef RT_SC_RELOAD
#define RT_SC_RELOAD 2
#endif
template <class R, int ACC> constexpr bool sc_reload() {
    return sizeof(R) == 8 && (((RT_SC_RELOAD & 1) && ACC == ACC_BVH_STACK_LEAN) ||
                              ((RT_SC_RELOAD & 2) && ACC == ACC_GRID_LDS_LEAN) || ((RT_SC_RELOAD & 4) && ACC == ACC_BRUTE_LEAN));
}
// LOCAL: sc is closest_hit_acc's own reloaded copy
template <class R, int ACC, bool LOCAL = false>
RT_HD Closest<R> closest_hit_acc(const SceneView<R>& sc, V3<R> o, V3<R> d, Work& w, BvhStack stk, bool skip_tri = false,
                                 int origin = -1) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (!LOCAL && sc_reload<R, ACC>()) {
        typedef const __attribute__((address_space(4))) SceneView<R>* SvPtr;
        SvPtr p = (SvPtr)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(p));
        const SceneView<R> scl = *p;
        return closest_hit_acc<R, ACC, true>(scl, o, d, w, stk, skip_tri, origin);
    }
#endif
    if constexpr (ACC == ACC_BVH) return closest_hit_bvh<R, false>(sc, o, d, w, stk, skip_tri);
    else if constexpr (ACC == ACC_BVH_STACK) return closest_hit_bvh<R, true>(sc, o, d, w, stk, skip_tri);
    else if constexpr (ACC == ACC_BVH_SPHERES) return closest_hit_bvh<R, true, false>(sc, o, d, w, stk);
    else if constexpr (ACC == ACC_BVH_SPHERES_LDS) return closest_hit_bvh<R, true, false, true>(sc, o, d, w, stk);
    else if constexpr (ACC == ACC_GRID) return closest_hit_grid<R>(sc, o, d, w, stk);
    else if constexpr (ACC == ACC_GRID_LDS) return closest_hit_grid<R, true>(sc, o, d, w, stk);
    else if constexpr (ACC == ACC_GRID_LDS_LEAN) return closest_hit_grid<R, true, feat_of<ACC>(), LOCAL>(sc, o, d, w, stk, origin);
    else if constexpr (ACC == ACC_BVH_STACK_LEAN)
        return closest_hit_bvh<R, true, true, false, false, feat_of<ACC>()>(sc, o, d, w, stk, skip_tri);
    else if constexpr (ACC == ACC_BVH_TRI_LDS) return closest_hit_bvh<R, true, true, false, true>(sc, o, d, w, stk);
    else return closest_hit_runs<R, feat_of<ACC>()>(sc, o, d);
}

template <class R>
struct Hit { V3<R> p, n; bool front; int mat; };

template <class R>
RT_HD void set_face(Hit<R>& h, V3<R> d, V3<R> outward) {       // math.js:55-58
    h.front = dot(d, outward) < (R)0;
    h.n = h.front ? outward : outward * (R)-1;
}

// Rebuild the HitRecord of the winning primitive (point = origin + dir*t, math.js:41).  FEAT: the kinds a
// scene without the missing features cannot hit are left out
template <class R, int FEAT = F_ALL>
RT_HD Hit<R> hit_record(const SceneView<R>& sc, V3<R> o, V3<R> d, const Closest<R>& c) {
    Hit<R> h;
    h.p = o + d * c.t;
    h.mat = c.mat;
    if ((FEAT & (F_PLANES | F_BOXES | F_TRIS)) == 0 || c.kind == HIT_SPHERE) {
        const SphereRec<R> s = sc.spheres[c.idx];
#if RT_DIV_RCP
        set_face(h, d, vdiv_rcp(h.p - mk(s.cx, s.cy, s.cz), sc.sphere_r[c.idx], sc.sphere_inv_r[c.idx]));
#else
        set_face(h, d, vdiv(h.p - mk(s.cx, s.cy, s.cz), sc.sphere_r[c.idx]));
#endif
    } else if ((FEAT & F_PLANES) != 0 && c.kind == HIT_PLANE) {
        const PlaneRec<R> p = sc.planes[c.idx];
        set_face(h, d, mk(p.nx, p.ny, p.nz));
    } else if ((FEAT & F_BOXES) != 0 && c.kind == HIT_BOX) {                          // geometry.js:118-126
        const BoxRec<R> b = sc.boxes[c.idx];
        const R eps = (R)1e-6;
        V3<R> n;
        if (fabs(h.p.x - b.mnx) < eps) n = mk<R>(-1, 0, 0);
        else if (fabs(h.p.x - b.mxx) < eps) n = mk<R>(1, 0, 0);
        else if (fabs(h.p.y - b.mny) < eps) n = mk<R>(0, -1, 0);
        else if (fabs(h.p.y - b.mxy) < eps) n = mk<R>(0, 1, 0);
        else if (fabs(h.p.z - b.mnz) < eps) n = mk<R>(0, 0, -1);
        else n = mk<R>(0, 0, 1);
        set_face(h, d, n);
    } else {
        const TriRec<R> tr = sc.tris[c.idx];
        set_face(h, d, mk(tr.nx, tr.ny, tr.nz));
    }
    return h;
}

template <class R>
RT_HD V3<R> random_in_unit_sphere(Rng<R>& g) {                  // math.js:22-26
    // A draw is u * 2^-24 (u a 24-bit integer), so 2r - 1 = (u - 2^23) * 2^-23 exactly, and
    // lengthSquared() of such a point is EXACT in binary64 (squares < 2^-46 granularity, sum < 3):
    // the binary64 test p.lengthSquared() < 1 is the integer test X^2 + Y^2 + Z^2 < 2^46 — the same
    // decisions at integer cost (and the exact decision in f32 mode too).
    int64_t x, y, z;
    do {
        RT_HCOUNT(HC_SPHERE_DRAW_ROUNDS, 1);
        x = (int64_t)g.next_u24() - (1 << 23);
        y = (int64_t)g.next_u24() - (1 << 23);
        z = (int64_t)g.next_u24() - (1 << 23);
    } while (x * x + y * y + z * z >= ((int64_t)1 << 46));
    return mk((R)x * (R)0x1p-23, (R)y * (R)0x1p-23, (R)z * (R)0x1p-23);
}

template <class R>
RT_HD V3<R> random_in_unit_disk(Rng<R>& g) {                    // math.js:27-31
    int64_t x, y;                                                 // exact, as random_in_unit_sphere
    do {
        RT_HCOUNT(HC_DISK_DRAW_ROUNDS, 1);
        x = (int64_t)g.next_u24() - (1 << 23);
        y = (int64_t)g.next_u24() - (1 << 23);
    } while (x * x + y * y >= ((int64_t)1 << 46));
    return mk<R>((R)x * (R)0x1p-23, (R)y * (R)0x1p-23, 0);
}

// ---- backgrounds (world.js:35-110, Perlin noise.js:29-61) ---------------------------------------
template <class R> RT_HD R fade(R t) { return t * t * t * (t * (t * (R)6 - (R)15) + (R)10); }
template <class R> RT_HD R lerp(R t, R a, R b) { return a + t * (b - a); }
template <class R> RT_HD R grad(int hash, R x, R y, R z) {
    int h = hash & 15;
    R u = h < 8 ? x : y;
    R v = h < 4 ? y : (h == 12 || h == 14) ? x : z;
    return ((h & 1) == 0 ? u : -u) + ((h & 2) == 0 ? v : -v);
}
template <class R>
__host__ __device__ R perlin(const int* p, R x, R y, R z) {
    R fx0 = floor(x), fy0 = floor(y), fz0 = floor(z);
    int X = ((int)(long long)fx0) & 255, Y = ((int)(long long)fy0) & 255, Z = ((int)(long long)fz0) & 255;
    R fx = x - fx0, fy = y - fy0, fz = z - fz0;
    R u = fade(fx), v = fade(fy), w = fade(fz);
    int A = p[X] + Y, AA = p[A] + Z, AB = p[A + 1] + Z;
    int B = p[X + 1] + Y, BA = p[B] + Z, BB = p[B + 1] + Z;
    return lerp(w,
                lerp(v, lerp(u, grad(p[AA], fx, fy, fz), grad(p[BA], fx - (R)1, fy, fz)),
                     lerp(u, grad(p[AB], fx, fy - (R)1, fz), grad(p[BB], fx - (R)1, fy - (R)1, fz))),
                lerp(v, lerp(u, grad(p[AA + 1], fx, fy, fz - (R)1), grad(p[BA + 1], fx - (R)1, fy, fz - (R)1)),
                     lerp(u, grad(p[AB + 1], fx, fy - (R)1, fz - (R)1), grad(p[BB + 1], fx - (R)1, fy - (R)1, fz - (R)1))));
}

// Backgrounds the hot loop rarely or never takes (hdri, procedural sky with Perlin noise) are kept
// out of line (RT_COLD_BG): their code then does not take part in the trace kernel's register
// allocation.

template <class R>
__host__ __device__ RT_COLD V3<R> background_hdri(const SceneView<R>& sc, V3<R> d) {             // world.js:74-110
    const R I = sc.sky_intensity;
    V3<R> dir = normalize(d);
    V3<R> sun = normalize(mk<R>(-0.3, 0.6, -0.5));
    R sd = js_max<R>(0, dot(dir, sun));
    R mask = sd > ((R)1 - (R)0.04) ? (R)1 : (R)0;
    V3<R> sun_c = mk<R>(1.0, 0.95, 0.8) * (mask * (R)20);
    R corona = js_max<R>(0, (sd - ((R)1 - (R)0.2)) / (R)0.2);
    V3<R> cor_c = mk<R>(1.0, 0.8, 0.6) * (js_pow<R>(corona, (R)2) * (R)3);
    R y = dir.y;
    V3<R> sky_c = mk<R>(0.3, 0.5, 0.8) * (js_max<R>(0, y * (R)0.5 + (R)0.5) * (R)2);
    V3<R> gnd_c = mk<R>(0.2, 0.15, 0.1) * js_max<R>(0, -y * (R)0.3);
    V3<R> sc_c = mk<R>(0.8, 0.9, 1.0) * (js_pow<R>(js_max<R>(0, (R)1 - fabs(y)), (R)2) * (R)0.3);
    return ((((sky_c + gnd_c) + sc_c) + sun_c) + cor_c) * I;
}

template <class R>
__host__ __device__ RT_COLD V3<R> background_procedural(const SceneView<R>& sc, V3<R> d) {       // world.js:46-72
    const R I = sc.sky_intensity;
    V3<R> dir = normalize(d);
    V3<R> sun = normalize(mk<R>(0.3, 0.6, 0.8));
    R sd = js_max<R>(0, dot(dir, sun));
    V3<R> sun_c = mk<R>(1.0, 0.95, 0.8) * (js_pow<R>(sd, (R)512) * (R)10);
    V3<R> sky_c = mk<R>(0.4, 0.7, 1.0) * (js_max<R>(0, dir.y) * (R)0.8);
    V3<R> glow_c = mk<R>(1.0, 0.8, 0.6) * (js_exp<R>(-fabs(dir.y) * (R)4) * (R)0.3);
    V3<R> gnd_c = mk<R>(0.1, 0.15, 0.1) * js_max<R>(0, -dir.y * (R)0.5);
    R cloud = js_max<R>(0, perlin<R>(sc.perm, dir.x * (R)10, dir.y * (R)3 + (R)2, dir.z * (R)10) * (R)0.8 + (R)0.2);
    V3<R> cl_c = mk<R>(0.9, 0.9, 1.0) * (cloud * js_max<R>(0, dir.y) * (R)0.5);
    return ((((sky_c + glow_c) + gnd_c) + sun_c) + cl_c) * I;
}

// unit: normalize(d), computed by the caller (shade_segment shares it with the scatter of other lanes)
template <class R, int FEAT = F_ALL>
__host__ __device__ V3<R> background(const SceneView<R>& sc, V3<R> d, V3<R> unit) {
    const R I = sc.sky_intensity;
    if constexpr ((FEAT & F_BGALL) == 0) {                                            // skyGradient only
        R t = (R)0.5 * (unit.y + (R)1);
        return (mk<R>(1, 1, 1) * ((R)1 - t) + mk<R>(0.5, 0.7, 1.0) * t) * I;
    }
    switch (sc.background) {
    case 0: {                                                                         // skyGradient
        R t = (R)0.5 * (unit.y + (R)1);
        return (mk<R>(1, 1, 1) * ((R)1 - t) + mk<R>(0.5, 0.7, 1.0) * t) * I;
    }
    case 1:                                                                           // solid
        return mk(sc.solid[0], sc.solid[1], sc.solid[2]) * I;
    case 2:                                                                           // hdri
        return background_hdri(sc, d);
    case 3:                                                                           // proceduralSky
        return background_procedural(sc, d);
    default:                                                                          // JSON solid/hdri bug
        return mk<R>((R)NAN, (R)NAN, (R)NAN);
    }
}

}  // namespace rt
