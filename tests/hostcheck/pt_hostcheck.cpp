// pt_hostcheck.cpp — TEST INFRASTRUCTURE: runs the megakernel's per-lane code (pt_path.h,
// pt_core.h, scene_pack.h — the very same source the GPU kernel compiles) on the CPU, one pixel at a
// time, so CPU-only tests can check the flattened path loop, the run packing and the record layout
// against the oracle.  Built host-only; never part of librt_hip.so, never loaded by product code.
#include <string>

#include "../../blenderraytracer_amd/csrc/pt_path.h"
#include "../../blenderraytracer_amd/csrc/scene_pack.h"
#include "../../blenderraytracer_amd/csrc/pool_order.h"

using namespace rt;

// host-side scene staging exactly as rt_scene_create builds it (pack_host, build_bvhs, make_records)
template <class R>
struct HostView {
    HostScene hs;
    HostRecords<R> rec;
    SceneView<R> v{};
    bool init(const rt_scene_desc* d) {
        std::string err;
        if (!pack_host(*d, hs, err)) return false;
        build_bvhs(hs);
        choose_walk(hs, *d);
        make_records(hs, *d, rec);
        v.runs = hs.runs.data();
        v.spheres = rec.spheres.data(); v.sphere_filter = rec.sphere_filter.data(); v.sphere_r = rec.sphere_r.data(); v.sphere_inv_r = rec.sphere_inv_r.data(); v.planes = rec.planes.data();
        v.boxes = rec.boxes.data(); v.tris = rec.tris.data(); v.sphere_mat = hs.sphere_mat.data();
        v.plane_mat = hs.plane_mat.data(); v.box_mat = hs.box_mat.data(); v.tri_mat = hs.tri_mat.data();
        v.mats = rec.mats.data(); v.perm = rec.perm.data();
        v.plane_obj = hs.plane_obj.data(); v.box_obj = hs.box_obj.data();
        v.sphere_nodes = hs.sphere_bvh.data(); v.tri_nodes = hs.tri_bvh.data();
        v.bvh_sphere_leaf = rec.bvh_sphere_leaf.data(); v.bvh_tri_leaf = rec.bvh_tri_leaf.data();
        v.tri_filter = rec.tri_filter.data(); v.tri_exit = hs.tri_exit.data();
        v.big_spheres = rec.big_sphere_leaf.data();
        v.sphere_wide = hs.sphere_wide.data(); v.tri_wide = hs.tri_wide.data();
        v.grid_cell = hs.grid_cell.data(); v.grid_leaf = rec.grid_leaf.data();
        fill_view_constants(v, hs, *d);
        return hs.bvh_depth <= 64;                   // the host walks use 64-entry stacks
    }
};

template <class R>
static int render(const rt_scene_desc* d, const rt_settings* s, double* sum, uint32_t* segs, uint32_t* draws) {
    HostView<R> hv;
    if (!hv.init(d)) return -1;
    const SceneView<R>& v = hv.v;
    ImageParams im{};
    im.width = s->width; im.height = s->height;
    im.x0 = s->crop_x0; im.y0 = s->crop_y0;
    im.cw = s->crop_w > 0 ? s->crop_w : s->width;
    im.ch = s->crop_h > 0 ? s->crop_h : s->height;
    im.samples = s->samples;
    im.s_begin = s->sample_begin > 0 ? s->sample_begin : 0;
    im.s_end = s->sample_end > 0 ? s->sample_end : s->samples;
    im.max_depth = s->max_depth;
    im.aa_mode = s->aa_mode;
    im.seedm = host_seed_mix(s->seed);
    int stack[64];
    const BvhStack stk{stack, 1};
    for (int cy = 0; cy < im.ch; ++cy)
        for (int cx = 0; cx < im.cw; ++cx) {
            const size_t q = (size_t)cy * im.cw + cx;
            PixelResult r{0, 0, {0, 0, 0}};
            double* acc = sum + 3 * q;
            // accel: RT_ACCEL_BVH = the ordered two-child walk (the kernel's); hostcheck-only
            // selector 3 = the stackless preorder walk
            if (im.max_depth > 0)
                r = s->accel == RT_ACCEL_BVH ? trace_pixel<R, true, ACC_BVH_STACK>(v, im, cx, cy, im.s_end, acc, stk)
                  : s->accel == 3            ? trace_pixel<R, true, ACC_BVH>(v, im, cx, cy, im.s_end, acc)
                  : s->accel == 4            ? trace_pixel<R, true, ACC_GRID>(v, im, cx, cy, im.s_end, acc)
                                             : trace_pixel<R, true, ACC_BRUTE>(v, im, cx, cy, im.s_end, acc);
            segs[q] = r.segments;
            draws[q] = r.draws;
        }
    return 0;
}

extern "C" int ptc_render(const rt_scene_desc* d, const rt_settings* s, double* sum, uint32_t* segs, uint32_t* draws) {
    return s->precision == RT_PREC_F32 ? render<float>(d, s, sum, segs, draws) : render<double>(d, s, sum, segs, draws);
}

// Adversarial check of the binary32 sphere pre-filter (pt_core.h sphere_filter_pass): random spheres
// over 7 decades of scale, rays aimed at |p| = r (1 +- eps) from the centre so disc64 sits at 0.
// Returns the number of spheres the filter rejected although disc64 >= 0 (must be 0); writes the
// largest |disc32 - disc64| / (A Q) seen and the fraction of sure misses the filter rejects.
#include <cmath>
#include <cstring>
#include <random>
extern "C" int ptc_sphere_filter_check(long long n, unsigned seed, double* max_ratio, double* reject_frac) {
    std::mt19937_64 gen(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long long violations = 0, misses = 0, rejected = 0;
    double worst = 0;
    for (long long it = 0; it < n; ++it) {
        const double scale = std::pow(10.0, 4.0 * U(gen) + 0.5);      // scene scale 10^-3.5 .. 10^4.5
        const double r = std::fabs(U(gen)) * scale * 0.5 + 1e-9;
        const double c[3] = {U(gen) * scale, U(gen) * scale, U(gen) * scale};
        double dd[3] = {U(gen), U(gen), U(gen)};
        const double dl = std::pow(10.0, 3.0 * U(gen));                // |d| 10^-3 .. 10^3 (unnormalized)
        // a point at distance r*(1+eps) from the centre, perpendicular to d, then back off along d
        double w[3] = {U(gen), U(gen), U(gen)};
        const double wd = (w[0] * dd[0] + w[1] * dd[1] + w[2] * dd[2]) / (dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
        for (int k = 0; k < 3; ++k) w[k] -= wd * dd[k];
        const double wn = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        const double eps = (it & 1 ? 1 : -1) * std::pow(10.0, -7.0 * std::fabs(U(gen)) - 1.0);
        const double back = U(gen) * 4 * scale;
        double o[3], d[3];
        for (int k = 0; k < 3; ++k) {
            d[k] = dd[k] * dl;
            o[k] = c[k] + w[k] / wn * r * (1 + eps) - dd[k] * back;
        }
        const double ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
        const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double hb = ocx * d[0] + ocy * d[1] + ocz * d[2];
        const double cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r * r;
        const double disc64 = hb * hb - a * cc;
        const double k = 2.0 * (c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) + r * r;
        SphereFilter f{(float)c[0], (float)c[1], (float)c[2], (float)((r * r + filter_margin() * k) * (1.0 + 0x1p-20))};
        const FilterRay fr = make_filter_ray(V3<double>{o[0], o[1], o[2]}, V3<double>{d[0], d[1], d[2]});
        const bool pass = sphere_filter_pass(f, fr);
        if (disc64 >= 0 && !pass) ++violations;
        if (disc64 < 0) { ++misses; rejected += !pass; }
        // observed |X - Y - margin| / Q of the binary32 evaluation (X, Y as in sphere_filter_bound)
        const float fx = fr.ox - (float)c[0], fy = fr.oy - (float)c[1], fz = fr.oz - (float)c[2];
        const float fhb = __builtin_fmaf(fx, fr.dx, __builtin_fmaf(fy, fr.dy, fz * fr.dz));
        const float fcc = __builtin_fmaf(fx, fx, __builtin_fmaf(fy, fy, __builtin_fmaf(fz, fz, -(float)(r * r))));
        const double X = (double)__builtin_fmaf(fhb, fhb, -fcc);
        const double Y = disc64 / a;
        double Q = 0;
        for (int q = 0; q < 3; ++q) Q += (std::fabs(o[q]) + std::fabs(c[q])) * (std::fabs(o[q]) + std::fabs(c[q]));
        Q += r * r;
        const double ratio = std::fabs(X - Y) / Q;
        if (ratio > worst) worst = ratio;
    }
    *max_ratio = worst;
    *reject_frac = misses ? (double)rejected / misses : 0;
    return (int)violations;
}

// The reference's Sphere.hit decision and root (geometry.js:15-45) in binary64, without any early rule
static bool sphere_full(const SphereRec<double>& s, V3<double> o, V3<double> d, double a, double tmin, double& t) {
    const double ocx = o.x - s.cx, ocy = o.y - s.cy, ocz = o.z - s.cz;
    const double hb = ocx * d.x + ocy * d.y + ocz * d.z;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - s.r2;
    const double disc = hb * hb - a * c;
    if (disc < 0) return false;
    const double sq = std::sqrt(disc);
    t = (-hb - sq) / a;
    if (!(t < tmin)) return true;
    t = (-hb + sq) / a;
    return !(t < tmin);
}

// Away and leave rejections (sphere_candidate's early rules): rays leaving a sphere's surface — the
// origin is the hit point o + t d of a previous ray computed in binary64 (just inside or just outside),
// the new direction random (outward, inward, grazing) — and random rays elsewhere, at 8 decades of scale.
// Returns the number of cases where sphere_candidate's decision or t differs from the full test;
// *taken counts the cases an early rule rejected (full test: a miss that computed a root).
extern "C" long long ptc_away_check(long long n, unsigned seed, long long* taken) {
    std::mt19937_64 gen(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long long bad = 0, early = 0;
    for (long long it = 0; it < n; ++it) {
        const double scale = std::pow(10.0, 4.0 * U(gen));
        const double r = (it % 3 == 0 ? 1000.0 : std::fabs(U(gen)) + 1e-3) * scale * (U(gen) < 0 ? -1 : 1);
        const SphereRec<double> s{U(gen) * scale, U(gen) * scale, U(gen) * scale, r * r};
        V3<double> o, d{U(gen), U(gen), U(gen)};
        if (it & 1) {                       // a hit point on the sphere from a ray aimed at it
            const V3<double> o0{s.cx + 3 * std::fabs(r) * U(gen), s.cy + 3 * std::fabs(r) * U(gen), s.cz + 3 * std::fabs(r) * U(gen)};
            const V3<double> d0{s.cx - o0.x + 0.5 * r * U(gen), s.cy - o0.y + 0.5 * r * U(gen), s.cz - o0.z + 0.5 * r * U(gen)};
            double t0;
            if (!sphere_candidate(s, o0, d0, dot(d0, d0), 0.001, t0)) continue;
            o = o0 + d0 * t0;
            if (it & 2) {                   // nearly tangent outgoing directions
                const V3<double> nrm = (o - mk(s.cx, s.cy, s.cz)) * (1.0 / r);
                d = d - nrm * dot(d, nrm) + nrm * (1e-9 * U(gen));
            }
        } else {
            o = V3<double>{s.cx + 4 * std::fabs(r) * U(gen), s.cy + 4 * std::fabs(r) * U(gen), s.cz + 4 * std::fabs(r) * U(gen)};
        }
        const double a = dot(d, d);
        double ta = 0, tb = 0;
        const bool ha = sphere_candidate(s, o, d, a, 0.001, ta, true);
        const bool hb = sphere_full(s, o, d, a, 0.001, tb);
        if (ha != hb || (ha && ta != tb)) ++bad;
        const V3<double> oc = o - mk(s.cx, s.cy, s.cz);
        const double cc = (oc.x * oc.x + oc.y * oc.y + oc.z * oc.z) - s.r2, hh = oc.x * d.x + oc.y * d.y + oc.z * d.z;
        early += hh >= 0 && (cc >= 0 || (-cc < hh * 0.00025 && hh * 0x1p-45 < a * 0.00025));
    }
    *taken = early;
    return bad;
}

// BVH stress rays: n random rays per scene that start at random points and aim at random primitives'
// surfaces (near-tangent for spheres, near edges and vertices for triangles) to exercise the
// conservative node bounds.  Writes up to n rays (origin xyz, direction xyz) into rays; returns the count.
static long long bvh_rays(const HostScene& hs, long long n, unsigned seed, double* rays) {
    std::mt19937_64 gen(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const int ns = (int)hs.sphere_r.size(), nt = (int)hs.tri_mat.size();
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int i = 0; i < ns; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], hs.spheres[4 * i + a] - std::fabs(hs.sphere_r[i]));
            hi[a] = std::max(hi[a], hs.spheres[4 * i + a] + std::fabs(hs.sphere_r[i]));
        }
    for (int i = 0; i < 3 * nt; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], hs.tri_verts[3 * i + a]);
            hi[a] = std::max(hi[a], hs.tri_verts[3 * i + a]);
        }
    long long m = 0;
    for (long long it = 0; it < n; ++it) {
        double o[3], target[3];
        for (int a = 0; a < 3; ++a) o[a] = lo[a] + (hi[a] - lo[a]) * (0.5 + 0.75 * U(gen));
        const int pick = (int)(std::fabs(U(gen)) * (ns + nt));
        const double eps = std::pow(10.0, -10.0 * std::fabs(U(gen)) - 2.0) * (U(gen) < 0 ? -1 : 1);
        if (pick < ns) {                   // a point at distance r (1 + eps) from the centre, off the ray
            const double* c = &hs.spheres[4 * pick];
            double w[3] = {U(gen), U(gen), U(gen)};
            const double wn = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            for (int a = 0; a < 3; ++a) target[a] = c[a] + w[a] / wn * std::fabs(hs.sphere_r[pick]) * (1 + eps);
        } else if (nt > 0) {               // a point on or just off an edge / vertex of a triangle
            const double* t = &hs.tri_verts[9 * std::min(pick - ns, nt - 1)];
            double u = std::fabs(U(gen)), w = std::fabs(U(gen));
            const int mode = (int)(std::fabs(U(gen)) * 3);
            if (mode == 0) w = 0;                        // edge v0-v1
            else if (mode == 1) { u = 1 + eps; w = 0; }  // past vertex v1
            else { w = 1 - u + eps; }                     // edge v1-v2
            for (int a = 0; a < 3; ++a) target[a] = t[a] + u * (t[3 + a] - t[a]) + w * (t[6 + a] - t[a]);
        } else {
            continue;
        }
        const double dl = std::pow(10.0, 2.0 * U(gen));
        double* r = rays + 6 * m++;
        for (int a = 0; a < 3; ++a) {
            r[a] = o[a];
            r[3 + a] = (target[a] - o[a]) * dl;
        }
    }
    return m;
}

// The stress rays of bvh_rays for the device test (tests/test_gpu_parity.py runs them through
// rt_closest_hits) with the host's World-order closest hit of the first host_n: t (+inf on a miss), kind,
// index.
extern "C" long long ptc_bvh_rays(const rt_scene_desc* d, long long n, unsigned seed, long long host_n, double* rays,
                                  double* t, int* kind, int* idx) {
    HostView<double> hv;
    if (!hv.init(d)) return -1;
    const long long m = bvh_rays(hv.hs, n, seed, rays);
    for (long long k = 0; k < std::min(m, host_n); ++k) {
        const double* r = rays + 6 * k;
        const Closest<double> a = closest_hit<double>(hv.v, V3<double>{r[0], r[1], r[2]}, V3<double>{r[3], r[4], r[5]});
        t[k] = a.kind == HIT_NONE ? INFINITY : a.t;
        kind[k] = a.kind;
        idx[k] = a.kind == HIT_NONE ? -1 : a.idx;
    }
    return m;
}

// BVH stress on the host: closest_hit (World order) vs closest_hit_bvh (both walks) on the bvh_rays.
// Returns the number of rays whose (t, primitive kind, index) differ.
extern "C" long long ptc_bvh_check(const rt_scene_desc* d, long long n, unsigned seed, long long* hits) {
    HostView<double> hv;
    if (!hv.init(d)) return -1;
    const SceneView<double>& v = hv.v;
    std::vector<double> rays(6 * (size_t)std::max(0LL, n));
    const long long m = bvh_rays(hv.hs, n, seed, rays.data());
    std::vector<rt_u4> grid_rec_copy(grid_lds_rec_bytes(v) / 16 + 1);
    std::vector<int> grid_cell_copy((size_t)v.num_grid_cells + 1);
    if (v.num_grid_cells > 0) copy_grid_lds(v, grid_rec_copy.data(), grid_cell_copy.data(), 0, 1);
    long long bad = 0, nh = 0;
    for (long long it = 0; it < m; ++it) {
        const double* r = &rays[6 * it];
        V3<double> O{r[0], r[1], r[2]}, D{r[3], r[4], r[5]};
        const Closest<double> a = closest_hit<double>(v, O, D);
        Work w{0, 0, 0};
        int stack[RT_BVH_STACK];
        const Closest<double> b = closest_hit_bvh<double, false>(v, O, D, w, BvhStack{nullptr, 0});
        const Closest<double> c = closest_hit_bvh<double, true>(v, O, D, w, BvhStack{stack, 1});
        const bool grid = v.num_grid_cells > 0 && v.num_tri_nodes == 0;
        const Closest<double> g = grid ? closest_hit_grid<double>(v, O, D, w, BvhStack{stack, 1}) : c;
        // the LDS-copy form of the grid walk (ACC_GRID_LDS) over a host copy of the grid
        BvhStack gs{stack, 1};
        gs.gcell = grid_cell_copy.data();
        gs.grec = grid_rec_copy.data();
        const Closest<double> gl = grid ? closest_hit_grid<double, true>(v, O, D, w, gs) : c;
        if (a.kind != HIT_NONE) ++nh;
        for (const Closest<double>& x : {b, c, g, gl}) {
            const bool same = a.kind == x.kind && (a.kind == HIT_NONE || (a.idx == x.idx && a.mat == x.mat &&
                                                                         std::memcmp(&a.t, &x.t, 8) == 0));
            bad += !same;
        }
    }
    if (hits) *hits = nh;
    return bad;
}

// BVH shape: deepest leaf of the binary trees, their two-child node count, and the dominant spheres
// tested before the walk (their sphere indices into big[0..*nbig), at most 8 written)
extern "C" int ptc_bvh_info(const rt_scene_desc* d, int* depth, int* nodes2, int* nbig, int* big) {
    HostView<double> hv;
    hv.init(d);
    *depth = hv.hs.bvh_depth;
    *nodes2 = (int)(hv.hs.sphere_wide.size() + hv.hs.tri_wide.size());
    *nbig = (int)hv.hs.big_spheres.size();
    for (int k = 0; k < *nbig && k < 8; ++k) big[k] = hv.hs.big_spheres[k];
    return 0;
}

// Work totals of the two-child walk (s->accel other than below), the grid walk (4) or World order
// (RT_ACCEL_BRUTE) over a crop (host experiments on BVH quality and the instruction-floor model,
// TEST/DEV TOOL): out = {segments, nodes or cells, sphere tests, triangle tests}
extern "C" int ptc_work(const rt_scene_desc* d, const rt_settings* s, double* out) {
    HostView<double> hv;
    if (!hv.init(d)) return -1;
    ImageParams im{};
    im.width = s->width; im.height = s->height;
    im.x0 = s->crop_x0; im.y0 = s->crop_y0;
    im.cw = s->crop_w > 0 ? s->crop_w : s->width;
    im.ch = s->crop_h > 0 ? s->crop_h : s->height;
    im.samples = s->samples;
    im.s_begin = 0;
    im.s_end = s->samples;
    im.max_depth = s->max_depth;
    im.aa_mode = s->aa_mode;
    im.seedm = host_seed_mix(s->seed);
    int stack[64];
    const BvhStack stk{stack, 1};
    for (int k = 0; k < 4; ++k) out[k] = 0;
    for (int cy = 0; cy < im.ch; ++cy)
        for (int cx = 0; cx < im.cw; ++cx) {
            double acc[3] = {0, 0, 0};
            const PixelResult r = s->accel == 4 ? trace_pixel<double, true, ACC_GRID>(hv.v, im, cx, cy, im.s_end, acc)
                                : s->accel == RT_ACCEL_BRUTE ? trace_pixel<double, true, ACC_BRUTE>(hv.v, im, cx, cy, im.s_end, acc)
                                                : trace_pixel<double, true, ACC_BVH_STACK>(hv.v, im, cx, cy, im.s_end, acc, stk);
            out[0] += r.segments; out[1] += r.work.nodes; out[2] += r.work.spheres; out[3] += r.work.tris;
        }
    return 0;
}

#ifdef RT_HOST_COUNTERS
// event counts of the kernel's code on the host (pt_core.h RT_HCOUNT, the instruction-floor model, DEV TOOL)
namespace rt { unsigned long long rt_host_count[16]; }
extern "C" void ptc_host_counts(unsigned long long* out, int reset) {
    for (int k = 0; k < 16; ++k) {
        out[k] = rt::rt_host_count[k];
        if (reset) rt::rt_host_count[k] = 0;
    }
}
#endif

// pow5_rn (pt_path.h) on the host, for the comparison with libm pow (TEST TOOL)
extern "C" void ptc_pow5(const double* x, double* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = rt::pow5_rn<double>(x[i]);
}
// the kernel's Schlick decision (pt_path.h schlick_reflects) for n (r0, cosine, draw) triples
extern "C" void ptc_schlick(const double* r0, const double* cos_t, const double* u, uint8_t* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = rt::schlick_reflects<double>(r0[i], cos_t[i], u[i]) ? 1 : 0;
}
// the kernel's Math.pow / Math.exp (csrc/js_math.h), host build
extern "C" void ptc_js_pow(const double* x, const double* y, double* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = jsm::pow(x[i], y[i]);
}
extern "C" void ptc_js_exp(const double* x, double* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = jsm::exp(x[i]);
}
extern "C" void ptc_js_trig(int f, const double* x, double* out, long long n) {     // 0 sin, 1 cos, 2 tan
    for (long long i = 0; i < n; ++i) out[i] = f == 0 ? jsm::sin(x[i]) : f == 1 ? jsm::cos(x[i]) : jsm::tan(x[i]);
}


// Grid shape (build_grid): cells per axis and sphere registrations (TEST/DEV TOOL)
extern "C" int ptc_grid_info(const rt_scene_desc* d, int* n3, long long* regs, int* use_grid) {
    HostView<double> hv;
    hv.init(d);
    for (int k = 0; k < 3; ++k) n3[k] = hv.hs.grid_n[k];
    *regs = (long long)hv.hs.grid_ids.size();
    *use_grid = hv.hs.use_grid ? 1 : 0;
    return 0;
}

// The sample pool's visiting order (pool_order.h, TEST TOOL): out[b] = the item (chunk * tiles + tile)
// that one-wave workgroup b of a cw x ch x `chunks` launch traces (one_wave), or that queue position b
// of the LDS kernel takes; params = {RT_TILE_BLOCK, RT_XCD_RUN, tiles}
extern "C" long long ptc_pool_order(int cw, int ch, int chunks, int one_wave, unsigned* out, int* params) {
    ImageParams im{};
    im.cw = cw;
    im.ch = ch;
    const int tiles = ((cw + 7) / 8) * ((ch + 7) / 8);
    const unsigned n = (unsigned)tiles * (unsigned)chunks;
    for (unsigned b = 0; b < n; ++b) out[b] = item_at(im, one_wave ? pool_position(b, n) : b, tiles);
    params[0] = RT_TILE_BLOCK;
    params[1] = RT_XCD_RUN;
    params[2] = tiles;
    return n;
}

// Band-major order (pool_order.h band_item, TEST TOOL): out[p] = the item at queue position p of a banded
// launch; band[p] = band_of_tile of that item's tile; counts[b] = band_items(b)
extern "C" long long ptc_band_order(int cw, int ch, int chunks, int bands, unsigned* out, int* band, unsigned* counts) {
    ImageParams im{};
    im.cw = cw;
    im.ch = ch;
    im.bands = bands;
    im.band_chunks = chunks;
    const int tiles = ((cw + 7) / 8) * ((ch + 7) / 8);
    const unsigned n = (unsigned)tiles * (unsigned)chunks;
    for (unsigned p = 0; p < n; ++p) {
        out[p] = item_at(im, p, tiles);
        band[p] = band_of_tile(im, (int)(out[p] % (unsigned)tiles));
    }
    for (int b = 0; b < bands; ++b) counts[b] = band_items(im, b);
    return n;
}

// chunk_range (pool_order.h, TEST TOOL): (batch, chunk, first sample, end sample) of launch chunk gci
extern "C" void ptc_chunk_range(int s_begin, int s_end, int batch_samples, int batch_chunks, int gci, int chunk, int* out) {
    ImageParams im{};
    im.s_begin = s_begin;
    im.s_end = s_end;
    im.batch_samples = batch_samples;
    im.batch_chunks = batch_chunks;
    const ChunkRange r = chunk_range(im, gci, chunk);
    out[0] = r.b; out[1] = r.ci; out[2] = r.sb; out[3] = r.se;
}
// ... of a device's launch in the whole-batch split (ImageParams::batch_ways)
extern "C" void ptc_chunk_range_ways(int s_begin, int s_end, int batch_samples, int batch_chunks, int ways, int gci,
                                     int chunk, int* out) {
    ImageParams im{};
    im.s_begin = s_begin;
    im.s_end = s_end;
    im.batch_samples = batch_samples;
    im.batch_chunks = batch_chunks;
    im.batch_ways = ways;
    const ChunkRange r = chunk_range(im, gci, chunk);
    out[0] = r.b; out[1] = r.ci; out[2] = r.sb; out[3] = r.se;
}

// root_div (pt_core.h RT_ROOT_RCP, TEST TOOL): x / a through RN(1 / a) and a Markstein correction
extern "C" void ptc_root_div(const double* x, const double* a, double* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = rt::root_div<double>(x[i], a[i], rt::root_rcp<double>(a[i]));
}
extern "C" void ptc_root_div_f32(const float* x, const float* a, float* out, long long n) {
    for (long long i = 0; i < n; ++i) out[i] = rt::root_div<float>(x[i], a[i], rt::root_rcp<float>(a[i]));
}

// vdiv_rcp's scalar division (pt_core.h div_rcp_1, TEST TOOL).  Binary32: every significand of x in
// [1, 2) against `ndiv` divisors (the 64 largest significands, all ones first, then random ones); returns
// the mismatches against the IEEE division.  Binary64: out2 = div_rcp_1 (two corrections), out1 = the
// single correction of round 4 (for the record) of given pairs (tests/test_root_div.py builds hard cases).
static float f32_bits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
extern "C" long long ptc_div_rcp_f32_exhaustive(int ndiv, unsigned seed) {
    std::mt19937 gen(seed);
    long long bad = 0;
    for (int ib = 0; ib < ndiv; ++ib) {
        const uint32_t bm = ib < 64 ? 0x7FFFFFu - (uint32_t)ib : (uint32_t)(gen() >> 9);
        const float s = f32_bits(0x3F800000u | bm), y = 1.0f / s;
        for (uint32_t am = 0; am < (1u << 23); ++am) {
            const float x = f32_bits(0x3F800000u | am);
            bad += rt::div_rcp_1<float>(x, s, y) != x / s;
        }
    }
    return bad;
}
extern "C" void ptc_div_rcp_f64(const double* x, const double* s, double* out2, double* out1, long long n) {
    for (long long i = 0; i < n; ++i) {
        const double y = 1.0 / s[i], q0 = x[i] * y;
        out2[i] = rt::div_rcp_1<double>(x[i], s[i], y);
        out1[i] = std::fma(std::fma(-q0, s[i], x[i]), y, q0);
    }
}

// normalize<float> (vdiv_rcp_unit: the min3 guard) against three IEEE divisions by the same l, bit for
// bit, on vectors whose components spread over 2^-149 .. 2^70 (zeros, subnormals, overflowing squares
// and mixed magnitudes included).  Returns the number of mismatching components (NaN == NaN).
extern "C" long long ptc_normalize_check(long long n, unsigned seed) {
    std::mt19937_64 gen(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long long bad = 0;
    auto comp = [&]() -> float {
        const int kind = (int)(gen() % 10);
        if (kind == 0) return 0.0f;
        const double e = kind == 1 ? -149 + 30 * U(gen) : kind == 2 ? 40 + 30 * U(gen) : -70 + 100 * U(gen);
        const float v = (float)(std::ldexp(1.0 + U(gen), (int)std::floor(e)));
        return (gen() & 1) ? -v : v;
    };
    for (long long i = 0; i < n; ++i) {
        const rt::V3<float> a{comp(), comp(), comp()};
        const rt::V3<float> q = rt::normalize<float>(a);
        const float l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
        const rt::V3<float> r = l > 0.0f ? rt::vdiv<float>(a, l) : rt::V3<float>{0, 0, 0};
        auto same = [](float u, float v) { return (u != u && v != v) || memcmp(&u, &v, 4) == 0; };
        bad += !same(q.x, r.x) + !same(q.y, r.y) + !same(q.z, r.z);
    }
    return bad;
}

// Adversarial check of the binary32 triangle pre-filter (pt_core.h tri_filter_pass, tri_filter_bound):
// random triangles over 7 decades of scale and shape (slivers included), rays through points at
// barycentric distance 10^-1 .. 10^-12 from an edge or a vertex (inside and outside), rays whose A = d.n
// sits at the 1e-4 threshold, origins at t = 0.001 (1 +- eps) before the plane, and a best hit at the
// triangle's t (1 +- eps).  Returns the number of cases the filter rejected although the binary64 test
// (triangle_candidate + `better`) accepts (must be 0); *reject_frac: the fraction of the binary64
// rejections the filter also rejects; *pass_frac: the fraction of all cases it lets through.
extern "C" long long ptc_tri_filter_check(long long n, unsigned seed, double* reject_frac, double* pass_frac) {
    std::mt19937_64 gen(seed);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long long bad = 0, rej64 = 0, rej_both = 0, passed = 0;
    for (long long it = 0; it < n; ++it) {
        const double scale = std::pow(10.0, 3.5 * U(gen));
        const double size = scale * std::pow(10.0, -3.0 * std::fabs(U(gen)));   // triangle size vs position
        double t9[12];
        for (int k = 0; k < 3; ++k) t9[k] = U(gen) * scale;
        double e1[3], e2[3];
        for (int k = 0; k < 3; ++k) { e1[k] = U(gen) * size; e2[k] = U(gen) * size; }
        if (it % 7 == 0) for (int k = 0; k < 3; ++k) e2[k] = e1[k] * (1 + 1e-3 * U(gen)) + 1e-6 * size * U(gen);   // sliver
        for (int k = 0; k < 3; ++k) { t9[3 + k] = (t9[k] + e1[k]) - t9[k]; t9[6 + k] = (t9[k] + e2[k]) - t9[k]; }
        // target: barycentric (bu, bv) near an edge / vertex / inside
        const int mode = (int)(gen() % 5);
        const double eps = std::pow(10.0, -11.0 * std::fabs(U(gen)) - 1.0) * (U(gen) < 0 ? -1 : 1);
        double bu = std::fabs(U(gen)), bv = std::fabs(U(gen));
        if (bu + bv > 1) { bu = 1 - bu; bv = 1 - bv; }
        if (mode == 0) bu = eps;                      // edge u = 0
        else if (mode == 1) bv = eps;                 // edge v = 0
        else if (mode == 2) bv = 1 - bu + eps;        // edge u + v = 1
        else if (mode == 3) { bu = 1 + eps; bv = 0; } // vertex v1
        double P[3];
        for (int k = 0; k < 3; ++k) P[k] = t9[k] + bu * t9[3 + k] + bv * t9[6 + k];
        // direction: random, or grazing (|d.n| ~ 1e-4 threshold), of length 10^-2 .. 10^2
        double dd[3] = {U(gen), U(gen), U(gen)};
        const double nn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double nl = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        const double dl = std::pow(10.0, 2.0 * U(gen));
        if (it % 3 == 1 && nl > 0) {
            // d = in-plane part + the normal component that puts |A| at 1e-4 (1 + eps2)
            const double dn = (dd[0] * nn[0] + dd[1] * nn[1] + dd[2] * nn[2]) / (nl * nl);
            for (int k = 0; k < 3; ++k) dd[k] -= dn * nn[k];
            const double want = 1e-4 * (1 + std::pow(10.0, -10.0 * std::fabs(U(gen)) - 2.0) * (U(gen) < 0 ? -1 : 1));
            for (int k = 0; k < 3; ++k) dd[k] = dd[k] * dl + (U(gen) < 0 ? -1 : 1) * want * nn[k] / (nl * nl);
        } else {
            for (int k = 0; k < 3; ++k) dd[k] *= dl;
        }
        // origin: back along d by tb (tb = 0.001 (1 + eps) some of the time: the tmin edge)
        const double tb = it % 4 == 2 ? 0.001 * (1 + std::pow(10.0, -10.0 * std::fabs(U(gen)) - 2.0) * (U(gen) < 0 ? -1 : 1))
                                      : std::pow(10.0, 3.0 * U(gen));
        double o[3];
        for (int k = 0; k < 3; ++k) o[k] = P[k] - dd[k] * tb;
        TriRec<double> tr{t9[0], t9[1], t9[2], t9[3], t9[4], t9[5], t9[6], t9[7], t9[8], 0, 0, 0};
        const V3<double> O{o[0], o[1], o[2]}, D{dd[0], dd[1], dd[2]};
        double t = 0;
        const bool cand = triangle_candidate(tr, O, D, 0.001, t);
        // the current best: none, or at the triangle's t (1 + eps), ties won by this triangle
        Closest<double> b{INFINITY, HIT_NONE, 0, 0, 1 << 30};
        if (it & 1) b.t = (cand ? t : tb) * (1 + std::pow(10.0, -12.0 * std::fabs(U(gen)) - 1.0) * (U(gen) < 0 ? -1 : 1));
        if (it % 16 == 5 && cand) b.t = t;             // exact tie
        const bool accept = cand && better(t, 0, 0, b);
        const TriFilter f = make_tri_filter(t9);
        const bool pass = tri_filter_pass(f, make_tri_ray(O, D), bvh_tlimit(b.t));
        if (accept && !pass) ++bad;
        if (!accept) { ++rej64; rej_both += !pass; }
        passed += pass;
    }
    *reject_frac = rej64 ? (double)rej_both / rej64 : 0;
    *pass_frac = n ? (double)passed / n : 0;
    return bad;
}
