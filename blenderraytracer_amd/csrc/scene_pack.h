// scene_pack.h — rt_scene_desc (include/rt_hip.h) -> the kernel's record arrays.
//
// World objects are grouped into runs of consecutive same-kind objects, preserving the
// World.objects insertion order that decides ties (js/world.js:24-30).  A mesh is always its own
// run: inside it the LAST equal-t triangle wins (geometry.js:253-259).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_hip.h"
#include "pt_core.h"

namespace rt {

struct HostScene {   // precision-independent staging, binary64 as packed by the host
    std::vector<Run> runs;
    std::vector<double> spheres, sphere_r, planes, boxes, tris;   // 4, 1, 6, 6, 12 doubles per record
    std::vector<int> sphere_mat, plane_mat, box_mat, tri_mat;
    std::vector<int> sphere_obj, plane_obj, box_obj, tri_obj;     // World.objects index (tie order)
    std::vector<double> tri_verts;                                // v0, v1, v2 as given (BVH bounds)
    std::vector<BvhNode> sphere_bvh, tri_bvh;                     // built by build_bvhs()
    std::vector<int> sphere_bvh_prims, tri_bvh_prims;
    std::vector<int> big_spheres;                                 // dominant spheres kept out of the tree
    std::vector<Bvh2Node> sphere_wide, tri_wide;                  // the same trees, two-child nodes
    std::vector<int> grid_cell, grid_ids;                         // build_grid: cell offsets, sphere ids
    int grid_n[3] = {0, 0, 0};
    float grid_lo[3] = {0, 0, 0}, grid_hi[3] = {0, 0, 0}, grid_cs[3] = {1, 1, 1}, grid_far = 0;
    bool use_grid = false;                                        // choose_walk(): the grid walks cheaper
    int bvh_depth = 0;                                            // deepest leaf of either tree
    int num_prims = 0;
    double record_bytes = 0;      // SURVEY §8d canonical bytes tested per segment
    // build_tri_exit (pt_core.h tri_exit_bound): {C+, C-} per triangle and the bound's constants
    std::vector<double> tri_exit;
    double exit_k0 = 0, exit_k1 = 0, exit_k2 = 0, exit_l1 = -1, exit_l2 = -1;
};

inline bool pack_host(const rt_scene_desc& d, HostScene& hs, std::string& err) {
    char buf[256];
    auto push_run = [&](int kind, int begin, int end, int mat) {
        if (!hs.runs.empty() && hs.runs.back().kind == kind && kind != RUN_MESH && hs.runs.back().end == begin)
            hs.runs.back().end = end;
        else
            hs.runs.push_back(Run{kind, begin, end, mat});
    };
    for (int i = 0; i < d.num_objects; ++i) {
        const rt_object_desc& o = d.objects[i];
        if (o.material < 0 || o.material >= d.num_materials) {
            snprintf(buf, sizeof buf, "object %d: material index %d out of range", i, o.material);
            err = buf;
            return false;
        }
        switch (o.type) {
        case RT_OBJ_SPHERE: {
            const int k = (int)hs.sphere_mat.size();
            const double r = o.g[3];
            hs.spheres.insert(hs.spheres.end(), {o.g[0], o.g[1], o.g[2], r * r});
            hs.sphere_r.push_back(r);
            hs.sphere_mat.push_back(o.material);
            hs.sphere_obj.push_back(i);
            push_run(RUN_SPHERES, k, k + 1, -1);
            hs.num_prims += 1;
            hs.record_bytes += 16;
            break;
        }
        case RT_OBJ_PLANE: {
            const int k = (int)hs.plane_mat.size();
            hs.planes.insert(hs.planes.end(), o.g, o.g + 6);
            hs.plane_mat.push_back(o.material);
            hs.plane_obj.push_back(i);
            push_run(RUN_PLANES, k, k + 1, -1);
            hs.num_prims += 1;
            hs.record_bytes += 24;
            break;
        }
        case RT_OBJ_BOX: {
            const int k = (int)hs.box_mat.size();
            hs.boxes.insert(hs.boxes.end(), o.g, o.g + 6);
            hs.box_mat.push_back(o.material);
            hs.box_obj.push_back(i);
            push_run(RUN_BOXES, k, k + 1, -1);
            hs.num_prims += 1;
            hs.record_bytes += 24;
            break;
        }
        case RT_OBJ_TRIANGLE:
        case RT_OBJ_MESH: {
            const int cnt = o.type == RT_OBJ_TRIANGLE ? 1 : o.count;
            if (o.first < 0 || cnt < 0 || (long long)o.first + cnt > d.num_triangles) {
                snprintf(buf, sizeof buf, "object %d: triangle range [%d, %d) outside %d triangles", i, o.first,
                         o.first + cnt, d.num_triangles);
                err = buf;
                return false;
            }
            if (cnt == 0) break;   // an empty mesh never hits
            const int k = (int)hs.tri_mat.size();
            for (int t = 0; t < cnt; ++t) {
                const double* v = d.triangles + 12 * (size_t)(o.first + t);
                // geometry.js:150-151 recomputes the edges per call; v1-v0 is the same double every
                // time, so storing e1 = v1-v0 and e2 = v2-v0 once is exact
                hs.tris.insert(hs.tris.end(), {v[0], v[1], v[2], v[3] - v[0], v[4] - v[1], v[5] - v[2],
                                               v[6] - v[0], v[7] - v[1], v[8] - v[2], v[9], v[10], v[11]});
                hs.tri_mat.push_back(o.material);
                hs.tri_obj.push_back(i);
                hs.tri_verts.insert(hs.tri_verts.end(), v, v + 9);
            }
            push_run(o.type == RT_OBJ_TRIANGLE ? RUN_TRIANGLES : RUN_MESH, k, k + cnt, o.material);
            hs.num_prims += cnt;
            hs.record_bytes += 36.0 * cnt;
            break;
        }
        default:
            snprintf(buf, sizeof buf, "object %d: unknown type %d", i, o.type);
            err = buf;
            return false;
        }
    }
    return true;
}

// ---- BVH (binned SAH, preorder with skip links) over spheres and over triangles ---------------------
// Node bounds are inflated on every axis by 2^-19 max|bound| (the node's largest coordinate) and
// rounded outward to binary32, so that the binary32 slab test of pt_core.h (bvh_node_hit) is
// conservative; see bvh_conservative_bound there.
struct BuildPrim { double lo[3], hi[3], c[3]; int idx; };

inline float round_down_f32(double y) {
    float f = (float)y;
    if ((double)f > y) f = std::nextafter(f, -INFINITY);
    return f;
}
inline float round_up_f32(double y) {
    float f = (float)y;
    if ((double)f < y) f = std::nextafter(f, INFINITY);
    return f;
}
// a primitive with a NaN coordinate never wins a closest-hit comparison; its bounds become the whole
// space so that it cannot poison the bounds of the primitives sharing its nodes
inline void sanitize_prim(BuildPrim& p) {
    bool bad = false;
    for (int a = 0; a < 3; ++a) bad |= p.lo[a] != p.lo[a] || p.hi[a] != p.hi[a];
    if (!bad) return;
    for (int a = 0; a < 3; ++a) { p.lo[a] = -INFINITY; p.hi[a] = INFINITY; p.c[a] = 0; }
}

struct BvhBuilder {
    std::vector<BuildPrim> prims;
    std::vector<BvhNode> nodes;
    std::vector<int> order;
    int max_depth = 0;                              // deepest leaf (root = 0)
#ifndef RT_BVH_LEAF
#define RT_BVH_LEAF 2             // triangles: measured 1 / 2 / 4 / 8 within 3 % on RTOW, 2 best on mesh50k
#endif
#ifndef RT_BVH_SPHERE_LEAF
#define RT_BVH_SPHERE_LEAF 1      // spheres: 1 vs 2 vs 3 on RTOW (dominant sphere peeled): +0.9 % / 0 / -1.2 %
#endif
#ifndef RT_BVH_BINS
#define RT_BVH_BINS 16
#endif
#ifndef RT_BVH_SWEEP
#define RT_BVH_SWEEP 0            // 1: full-sweep SAH over all three axes instead of binned on the widest
#endif
    int kLeafMax = RT_BVH_LEAF;                     // primitives per leaf (<= 15)
    static constexpr int kBins = RT_BVH_BINS;      // SAH bins

    static double area(const double* lo, const double* hi) {
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x * y + y * z + z * x;
    }

    // levels a median-split subtree of `count` primitives needs below its root
    int median_levels(int count) const {
        int l = 0;
        for (long long c = (count + kLeafMax - 1) / kLeafMax; c > 1; c = (c + 1) / 2) ++l;
        return l;
    }

    // depth: of this node (root 0).  Leaves stay at depth <= RT_BVH_STACK (the ordered walk's stack
    // holds at most one entry per level): when SAH could go deeper, the split becomes a median.
    int build(int begin, int end, int depth = 0) {
        const int me = (int)nodes.size();
        nodes.push_back(BvhNode{});
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = begin; k < end; ++k)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], prims[k].lo[a]);
                hi[a] = std::max(hi[a], prims[k].hi[a]);
                clo[a] = std::min(clo[a], prims[k].c[a]);
                chi[a] = std::max(chi[a], prims[k].c[a]);
            }
        BvhNode n{};
        double m = 0;
        for (int a = 0; a < 3; ++a) m = std::max(m, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
        const double pad = m * 0x1p-19 + 0x1p-100;
        for (int a = 0; a < 3; ++a) {
            n.lo[a] = round_down_f32(lo[a] - pad);
            n.hi[a] = round_up_f32(hi[a] + pad);
        }
        const int count = end - begin;
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        const double extent = chi[axis] - clo[axis];
        int mid = -1;
        const bool force_median = depth + 1 + median_levels(count) >= RT_BVH_STACK;
        if (RT_BVH_SWEEP && count > kLeafMax && extent > 0 && !force_median) {
            // full-sweep SAH: every object split along every axis (centroid order)
            double best = INFINITY;
            int best_axis = -1, best_i = -1;
            std::vector<double> right_area(count + 1);
            for (int a = 0; a < 3; ++a) {
                if (!(chi[a] - clo[a] > 0)) continue;
                std::sort(prims.begin() + begin, prims.begin() + end,
                          [&](const BuildPrim& p, const BuildPrim& q) { return p.c[a] < q.c[a] || (p.c[a] == q.c[a] && p.idx < q.idx); });
                double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (int i = count - 1; i >= 1; --i) {
                    const BuildPrim& p = prims[begin + i];
                    for (int k = 0; k < 3; ++k) { blo[k] = std::min(blo[k], p.lo[k]); bhi[k] = std::max(bhi[k], p.hi[k]); }
                    right_area[i] = area(blo, bhi);
                }
                for (int k = 0; k < 3; ++k) { blo[k] = INFINITY; bhi[k] = -INFINITY; }
                for (int i = 1; i < count; ++i) {
                    const BuildPrim& p = prims[begin + i - 1];
                    for (int k = 0; k < 3; ++k) { blo[k] = std::min(blo[k], p.lo[k]); bhi[k] = std::max(bhi[k], p.hi[k]); }
                    const double cost = i * area(blo, bhi) + (count - i) * right_area[i];
                    if (cost < best) { best = cost; best_axis = a; best_i = i; }
                }
            }
            if (best_axis >= 0) {
                std::sort(prims.begin() + begin, prims.begin() + end, [&](const BuildPrim& p, const BuildPrim& q) {
                    return p.c[best_axis] < q.c[best_axis] || (p.c[best_axis] == q.c[best_axis] && p.idx < q.idx);
                });
                mid = begin + best_i;
            } else {
                mid = (begin + end) / 2;
            }
        } else if (count > kLeafMax && extent > 0 && !force_median) {
            // binned SAH along the widest centroid axis
            struct Bin { double lo[3], hi[3]; int n; };
            Bin bins[kBins];
            for (auto& b : bins) {
                b.n = 0;
                for (int a = 0; a < 3; ++a) { b.lo[a] = INFINITY; b.hi[a] = -INFINITY; }
            }
            auto bin_of = [&](const BuildPrim& p) {
                int b = (int)((p.c[axis] - clo[axis]) / extent * kBins);
                return std::min(kBins - 1, std::max(0, b));
            };
            for (int k = begin; k < end; ++k) {
                Bin& b = bins[bin_of(prims[k])];
                b.n++;
                for (int a = 0; a < 3; ++a) {
                    b.lo[a] = std::min(b.lo[a], prims[k].lo[a]);
                    b.hi[a] = std::max(b.hi[a], prims[k].hi[a]);
                }
            }
            double best = INFINITY;
            int best_split = -1;
            for (int s = 1; s < kBins; ++s) {
                double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                double rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                int nl = 0, nr = 0;
                for (int b = 0; b < kBins; ++b) {
                    double* l = b < s ? llo : rlo;
                    double* h = b < s ? lhi : rhi;
                    (b < s ? nl : nr) += bins[b].n;
                    for (int a = 0; a < 3; ++a) {
                        l[a] = std::min(l[a], bins[b].lo[a]);
                        h[a] = std::max(h[a], bins[b].hi[a]);
                    }
                }
                if (!nl || !nr) continue;
                const double cost = nl * area(llo, lhi) + nr * area(rlo, rhi);
                if (cost < best) { best = cost; best_split = s; }
            }
            if (best_split > 0) {
                auto it = std::partition(prims.begin() + begin, prims.begin() + end,
                                         [&](const BuildPrim& p) { return bin_of(p) < best_split; });
                mid = (int)(it - prims.begin());
            }
            if (mid <= begin || mid >= end) {       // degenerate binning: median split
                mid = (begin + end) / 2;
                std::nth_element(prims.begin() + begin, prims.begin() + mid, prims.begin() + end,
                                 [&](const BuildPrim& p, const BuildPrim& q) { return p.c[axis] < q.c[axis]; });
            }
        } else if (count > kLeafMax) {              // depth cap or all centroids equal: median split
            mid = (begin + end) / 2;
            std::nth_element(prims.begin() + begin, prims.begin() + mid, prims.begin() + end,
                             [&](const BuildPrim& p, const BuildPrim& q) { return p.c[axis] < q.c[axis]; });
        }
        if (mid < 0) {                              // leaf
            max_depth = std::max(max_depth, depth);
            n.fc = ((int)order.size() << 4) | count;
            for (int k = begin; k < end; ++k) order.push_back(prims[k].idx);
        } else {
            n.fc = 0;
            build(begin, mid, depth + 1);           // first child = me + 1 (preorder)
            build(mid, end, depth + 1);
        }
        n.skip = (int)nodes.size();                 // next node after this subtree
        nodes[me] = n;
        return me;
    }
};

// preorder BvhNode tree -> Bvh2Node array of its inner nodes (root first); a tree that is a single leaf
// becomes one node whose second child is an empty leaf.  The first `top` inner nodes in breadth-first
// order come first (indices [0, top): the tree's top levels, which trace_pool_lds_kernel's triangle walk
// copies into LDS, ACC_BVH_TRI_LDS), the rest follow in preorder (a subtree's nodes stay close in
// memory).  A permutation of the nodes only: every walk visits the same children in the same order.
// (Round 1: breadth-first top levels staged in LDS by one-wave workgroups measured slower — the copy was
// paid per item; round 4: the layout alone measured +-1.5 %, noise.)  RT_TRI_TOP_NODES: pt_core.h
inline std::vector<Bvh2Node> make_wide(const std::vector<BvhNode>& t, int top = 0) {
    std::vector<Bvh2Node> out;
    if (t.empty()) return out;
    auto box = [&](Bvh2Node& n, int k, int i) {    // child k's bounds = tree node i's
        for (int a = 0; a < 3; ++a) { n.lo[a][k] = t[i].lo[a]; n.hi[a][k] = t[i].hi[a]; }
    };
    if (t[0].fc != 0) {
        Bvh2Node n{};
        box(n, 0, 0);
        box(n, 1, 0);
        n.child[0] = ~t[0].fc;
        n.child[1] = ~0;                           // fc 0: no primitives
        out.push_back(n);
        return out;
    }
    std::vector<int> map(t.size(), -1);
    int k = 0;
    if (top > 0) {                                  // breadth-first: root, its inner children, ...
        std::vector<int> q{0};
        for (size_t h = 0; h < q.size() && k < top; ++h) {
            const int i = q[h];
            map[i] = k++;
            const int l = i + 1, r = t[l].skip;
            if (t[l].fc == 0) q.push_back(l);
            if (t[r].fc == 0) q.push_back(r);
        }
    }
    for (size_t i = 0; i < t.size(); ++i)           // the rest in preorder
        if (t[i].fc == 0 && map[i] < 0) map[i] = k++;
    out.resize(k);
    auto ref = [&](int i) { return t[i].fc ? ~t[i].fc : map[i]; };
    for (size_t i = 0; i < t.size(); ++i) {
        if (t[i].fc != 0) continue;
        const int l = (int)i + 1, r = t[l].skip;
        Bvh2Node n{};
        box(n, 0, l);
        box(n, 1, r);
        n.child[0] = ref(l);
        n.child[1] = ref(r);
        out[map[i]] = n;
    }
    return out;
}

#ifndef RT_BIG_SPHERES
#define RT_BIG_SPHERES 4          // at most this many dominant spheres tested before the walk (0: none)
#endif
#ifndef RT_PEEL_FRAC
#define RT_PEEL_FRAC (1.0 / 64)   // RTOW: the ground, then its three r = 1 spheres (1/48 of the rest's box
#endif                            // area each): +6.4 % f64, +6.2 % f32 over peeling the ground alone (1.0)

// Dominant spheres (the RTOW ground, R = 1000 under spheres of r <= 1, then its three r = 1 spheres):
// a sphere whose bounding box has a surface area above 1/64 of the bounds of all the other remaining
// spheres together is taken out of the tree and tested before the walk (closest_hit_bvh), largest
// first, at most RT_BIG_SPHERES.  In the tree it would sit in a leaf that many rays enter, often
// visited after a subtree it hides; tested first, its hit shortens the ray before the walk, so the
// nodes behind it are culled, for one binary32 pre-test per segment.  Results are unchanged (the
// closest hit is order-independent, comment above `better`).
inline std::vector<int> peel_big_spheres(const HostScene& hs, std::vector<BuildPrim>& prims) {
    std::vector<int> big;
    for (int it = 0; it < RT_BIG_SPHERES && prims.size() > 2; ++it) {
        size_t best = 0;
        for (size_t k = 1; k < prims.size(); ++k)
            if (std::fabs(hs.sphere_r[prims[k].idx]) > std::fabs(hs.sphere_r[prims[best].idx])) best = k;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = 0; k < prims.size(); ++k)
            if (k != best)
                for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], prims[k].lo[a]); hi[a] = std::max(hi[a], prims[k].hi[a]); }
        const double mine = BvhBuilder::area(prims[best].lo, prims[best].hi), rest = BvhBuilder::area(lo, hi);
        if (!(mine > RT_PEEL_FRAC * rest) || !std::isfinite(mine)) break;
        big.push_back(prims[best].idx);
        prims.erase(prims.begin() + best);
    }
    return big;
}

#ifndef RT_GRID_LAMBDA
#define RT_GRID_LAMBDA 0.09       // cells per sphere (before rounding each axis up).  RTOW 256 spp f64 / f32,
#endif                            // round 4 (survivor masks, deferred regeneration): 0.0625 10154 / -,
                                  // 0.09 10157 / 13052, 0.125 10073 / 12871, 0.25 9911 / 13183, 0.35 9771 / -
                                  // (round 3, before the masks: 0.25 best, 0.0625 -1.7 %)
// Uniform grid over the spheres of the sphere tree (closest_hit_grid, pt_core.h): the box of those
// spheres padded by m = 2^-12 (B + E) (B: largest |coordinate|, E: largest extent), ~RT_GRID_LAMBDA
// cells per sphere of about cubic shape, every sphere registered in each cell its box padded by m
// overlaps, in the cells' binary32 coordinates lo + k cs that the walk uses.  No grid when a sphere box
// is not finite or the spheres are too few.
// The two factors of the grid's exactness argument (pt_core.h closest_hit_grid, "grid_bound"): the
// registration margin m = kGridMargin (B + E) and the origin bound grid_far = kGridFar (B + E).  A ray
// point's error is at most 2^-19 (|o|_inf + B) <= 2^-19 (kGridFar + 1) (B + E), which must not exceed m.
constexpr double kGridMargin = 0x1p-12, kGridFar = 0x1p6;
static_assert(0x1p-19 * (kGridFar + 1) <= kGridMargin, "grid_far too large for the registration margin");
inline void build_grid(HostScene& hs, const std::vector<BuildPrim>& prims) {
    hs.grid_cell.clear();
    hs.grid_ids.clear();
    hs.grid_n[0] = hs.grid_n[1] = hs.grid_n[2] = 0;
    if (prims.size() < 8) return;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const BuildPrim& p : prims)
        for (int a = 0; a < 3; ++a) {
            if (!std::isfinite(p.lo[a]) || !std::isfinite(p.hi[a])) return;
            lo[a] = std::min(lo[a], p.lo[a]);
            hi[a] = std::max(hi[a], p.hi[a]);
        }
    double B = 0, E = 0;
    for (int a = 0; a < 3; ++a) {
        B = std::max(B, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
        E = std::max(E, hi[a] - lo[a]);
    }
    if (!(B + E > 0) || !(B + E < 1e30)) return;
    const double m = kGridMargin * (B + E);
    double ext[3], vol = 1;
    for (int a = 0; a < 3; ++a) {
        lo[a] -= m;
        hi[a] += m;
        ext[a] = hi[a] - lo[a];
        vol *= ext[a];
    }
    const double side = std::cbrt(vol / (RT_GRID_LAMBDA * (double)prims.size()));
    long long total = 1;
    for (int a = 0; a < 3; ++a) {
        const double n = std::ceil(ext[a] / side);
        hs.grid_n[a] = (int)std::min(256.0, std::max(1.0, n));
        total *= hs.grid_n[a];
        // binary32 cell geometry, rounded outward so that lo + n cs >= hi
        float flo = (float)lo[a];
        if ((double)flo > lo[a]) flo = std::nextafter(flo, -INFINITY);
        float cs = (float)((hi[a] - (double)flo) / hs.grid_n[a]);
        while ((double)flo + (double)hs.grid_n[a] * (double)cs < hi[a]) cs = std::nextafter(cs, INFINITY);
        hs.grid_lo[a] = flo;
        hs.grid_cs[a] = cs;
        float fhi = (float)((double)flo + (double)hs.grid_n[a] * (double)cs);
        if ((double)fhi < hi[a]) fhi = std::nextafter(fhi, INFINITY);
        hs.grid_hi[a] = fhi;
    }
    hs.grid_far = (float)(kGridFar * (B + E));
    if (total > (1LL << 22)) { hs.grid_n[0] = hs.grid_n[1] = hs.grid_n[2] = 0; return; }
    auto range = [&](const BuildPrim& p, int a, int& k0, int& k1) {
        const double c = (double)hs.grid_cs[a], o = (double)hs.grid_lo[a];
        k0 = (int)std::floor((p.lo[a] - m - o) / c);
        k1 = (int)std::floor((p.hi[a] + m - o) / c);
        k0 = std::max(0, std::min(hs.grid_n[a] - 1, k0));
        k1 = std::max(0, std::min(hs.grid_n[a] - 1, k1));
    };
    long long regs = 0;           // registrations: give up on spheres too large for the cells
    for (const BuildPrim& p : prims) {
        long long r = 1;
        for (int a = 0; a < 3; ++a) {
            int k0, k1;
            range(p, a, k0, k1);
            r *= k1 - k0 + 1;
        }
        regs += r;
    }
    if (regs > 16LL * (long long)prims.size() + total) {
        hs.grid_n[0] = hs.grid_n[1] = hs.grid_n[2] = 0;
        return;
    }
    std::vector<int> count((size_t)total + 1, 0), cursor;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {            // count[c] -> offset of cell c; count[total] = registrations
            for (size_t c = 1; c <= (size_t)total; ++c) count[c] += count[c - 1];
            hs.grid_cell = count;
            cursor.assign(count.begin(), count.end() - 1);
            hs.grid_ids.assign((size_t)count[(size_t)total], 0);
        }
        for (const BuildPrim& p : prims) {
            int k0[3], k1[3];
            for (int a = 0; a < 3; ++a) range(p, a, k0[a], k1[a]);
            for (int z = k0[2]; z <= k1[2]; ++z)
                for (int y = k0[1]; y <= k1[1]; ++y)
                    for (int x = k0[0]; x <= k1[0]; ++x) {
                        const size_t c = (size_t)x + (size_t)hs.grid_n[0] * ((size_t)y + (size_t)hs.grid_n[1] * z);
                        if (pass == 0) ++count[c + 1];
                        else hs.grid_ids[(size_t)cursor[c]++] = p.idx;
                    }
        }
    }
}

// tri_exit_bound (pt_core.h): for every triangle A and each side N = +-n of its stored normal n, an upper
// bound C of N.w over the exact vertices w in {v0, v0 + e1, v0 + e2} of every triangle, found by a
// branch-and-bound walk of the triangle tree: a subtree is skipped when the support of its box,
// sum_k max(N_k lo_k, N_k hi_k) + 2^-17 max|box| (the box's own rounding and the exact vertices' offsets from
// the given ones), is below the best value so far.  A side gets C = +inf when some vertex lies more than
// 0.002 in front of A's own vertices (no exit ray, |d|_2 <= 2, could then pass the check: the walk stops
// there), when |n|_2 is not within 1e-6 of 1, or when any triangle has a non-finite coordinate.  The visited
// values carry the rounding pad 16 eps (Mv + Me) + 4 eps |C|.
#ifndef RT_TRI_EXIT_MAX
#define RT_TRI_EXIT_MAX (1 << 23)        // triangles; larger scenes skip the bounds (every C = +inf)
#endif
inline void build_tri_exit(HostScene& hs) {
    const size_t T = hs.tri_mat.size();
    hs.tri_exit.assign(2 * T, INFINITY);
    hs.exit_l1 = hs.exit_l2 = -1;       // no exit ray passes
    if (T == 0 || T > (size_t)RT_TRI_EXIT_MAX || hs.tri_bvh.empty()) return;
    double Mv = 0, Me = 0;
    for (size_t i = 0; i < T; ++i) {
        const double* t = &hs.tris[12 * i];
        for (int k = 0; k < 9; ++k)
            if (!std::isfinite(t[k])) return;
        for (int k = 0; k < 3; ++k) {
            Mv = std::max(Mv, std::fabs(t[k]));
            Me = std::max(Me, std::max(std::fabs(t[3 + k]), std::fabs(t[6 + k])));
        }
    }
    if (!(Me > 0) || !(Me < 1e100) || !(Mv < 1e100)) return;
    const double eps = 0x1p-53;
    hs.exit_k0 = 2 * eps * (42 * Me + 12 * Mv);
    hs.exit_k1 = 2 * eps * 8.96e6 * Me * Me;
    hs.exit_k2 = Mv + 1.01 * Me;
    hs.exit_l1 = 0.99 * (0.004 / (1e4 * 64 * eps * Me));          // L1: 1e4 (EX + 1.01 EA) <= 0.004
    hs.exit_l2 = 0.99 * (1e-9 / (64 * eps * Me * Me)) - Mv;       // L2: EZ <= 1e-9
    const double pad = 16 * eps * (Mv + Me);
    const BvhNode* nodes = hs.tri_bvh.data();
    const int count = (int)hs.tri_bvh.size();
    auto side = [&](const double* A, const double N[3]) -> double {
        auto phi3 = [&](const double* t, double& mx) {
            const double p0 = N[0] * t[0] + N[1] * t[1] + N[2] * t[2];
            const double p1 = p0 + (N[0] * t[3] + N[1] * t[4] + N[2] * t[5]);
            const double p2 = p0 + (N[0] * t[6] + N[1] * t[7] + N[2] * t[8]);
            mx = std::max(mx, std::max(p0, std::max(p1, p2)));
        };
        double best = -INFINITY;
        phi3(A, best);
        const double stop = best + 0.002;
        int ni = 0;
        while (ni < count) {
            const BvhNode& n = nodes[ni];
            double sup = 0, mb = 0;
            for (int k = 0; k < 3; ++k) {
                sup += std::max(N[k] * (double)n.lo[k], N[k] * (double)n.hi[k]);
                mb = std::max(mb, std::max(std::fabs((double)n.lo[k]), std::fabs((double)n.hi[k])));
            }
            if (sup + 0x1p-17 * mb <= best) { ni = n.skip; continue; }
            if (n.fc == 0) { ++ni; continue; }
            for (int k = n.fc >> 4, e = k + (n.fc & 15); k < e; ++k) phi3(&hs.tris[12 * (size_t)hs.tri_bvh_prims[k]], best);
            if (!(best <= stop)) return INFINITY;
            ni = n.skip;
        }
        return best + (pad + 4 * eps * std::fabs(best));
    };
    auto work = [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) {
            const double* t = &hs.tris[12 * i];
            const double nn = t[9] * t[9] + t[10] * t[10] + t[11] * t[11];
            if (!(std::fabs(nn - 1.0) <= 1e-6)) continue;              // |n|_2 within 5e-7 of 1
            const double np[3] = {t[9], t[10], t[11]}, nm[3] = {-t[9], -t[10], -t[11]};
            hs.tri_exit[2 * i] = side(t, np);
            hs.tri_exit[2 * i + 1] = side(t, nm);
        }
    };
    const size_t nt = std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (T < 4096 || nt == 1) { work(0, T); return; }
    std::vector<std::thread> th;
    size_t started = 0;
    try {
        for (; started < nt; ++started) th.emplace_back(work, T * started / nt, T * (started + 1) / nt);
    } catch (...) {               // no thread to be had: this thread takes the ranges not started
    }
    for (size_t w = started; w < nt; ++w) work(T * w / nt, T * (w + 1) / nt);
    for (auto& x : th) x.join();
}

inline void build_bvhs(HostScene& hs) {
    BvhBuilder sb;
    sb.kLeafMax = RT_BVH_SPHERE_LEAF;
    for (size_t i = 0; i < hs.sphere_r.size(); ++i) {
        const double* s = &hs.spheres[4 * i];
        const double r = std::fabs(hs.sphere_r[i]);       // negative radius: same sphere, inverted normal
        BuildPrim p;
        for (int a = 0; a < 3; ++a) { p.lo[a] = s[a] - r; p.hi[a] = s[a] + r; p.c[a] = s[a]; }
        p.idx = (int)i;
        sanitize_prim(p);
        sb.prims.push_back(p);
    }
    hs.big_spheres = peel_big_spheres(hs, sb.prims);
    build_grid(hs, sb.prims);
    if (!sb.prims.empty()) sb.build(0, (int)sb.prims.size());
    hs.bvh_depth = sb.max_depth;
    hs.sphere_bvh = std::move(sb.nodes);
    hs.sphere_bvh_prims = std::move(sb.order);
    BvhBuilder tb;
    for (size_t i = 0; i < hs.tri_mat.size(); ++i) {
        const double* v = &hs.tri_verts[9 * i];
        BuildPrim p;
        for (int a = 0; a < 3; ++a) {
            p.lo[a] = std::min(v[a], std::min(v[3 + a], v[6 + a]));
            p.hi[a] = std::max(v[a], std::max(v[3 + a], v[6 + a]));
            p.c[a] = (p.lo[a] + p.hi[a]) * 0.5;
        }
        p.idx = (int)i;
        sanitize_prim(p);
        tb.prims.push_back(p);
    }
    if (!tb.prims.empty()) tb.build(0, (int)tb.prims.size());
    hs.bvh_depth = std::max(hs.bvh_depth, tb.max_depth);
    hs.tri_bvh = std::move(tb.nodes);
    hs.tri_bvh_prims = std::move(tb.order);
    hs.sphere_wide = make_wide(hs.sphere_bvh);
    hs.tri_wide = make_wide(hs.tri_bvh, RT_TRI_TOP_NODES);
    build_tri_exit(hs);
}

// The binary32 pre-filter record of a triangle {v0, e1, e2, ...} (binary64, pt_core.h tri_filter_bound):
// the rounded vertex and edges and n = e2 x e1 (binary64 cross product, rounded); a triangle whose
// |e1|inf or |e2|inf lies outside [2^-30, 2^30], or |v0|inf above 2^30, or with a non-finite coordinate,
// gets n = NaN and is never rejected by the filter.
inline TriFilter make_tri_filter(const double* t) {
    TriFilter f;
    double me1 = 0, me2 = 0, m0 = 0;
    bool finite = true;
    for (int k = 0; k < 3; ++k) {
        f.v0[k] = (float)t[k];
        f.e1[k] = (float)t[3 + k];
        f.e2[k] = (float)t[6 + k];
        m0 = std::max(m0, std::fabs(t[k]));
        me1 = std::max(me1, std::fabs(t[3 + k]));
        me2 = std::max(me2, std::fabs(t[6 + k]));
        finite = finite && std::isfinite(t[k]) && std::isfinite(t[3 + k]) && std::isfinite(t[6 + k]);
    }
    const double* e1 = t + 3;
    const double* e2 = t + 6;
    const double n[3] = {e2[1] * e1[2] - e2[2] * e1[1], e2[2] * e1[0] - e2[0] * e1[2], e2[0] * e1[1] - e2[1] * e1[0]};
    const bool ok = finite && m0 <= 0x1p30 && me1 >= 0x1p-30 && me1 <= 0x1p30 && me2 >= 0x1p-30 && me2 <= 0x1p30;
    for (int k = 0; k < 3; ++k) f.n[k] = ok ? (float)n[k] : NAN;
    return f;
}

// Record arrays of one precision (host memory); rt_capi.cpp uploads them, tests/hostcheck uses them.
template <class R>
struct HostRecords {
    std::vector<SphereRec<R>> spheres;
    std::vector<SphereFilter> sphere_filter;
    std::vector<R> sphere_r, sphere_inv_r;
    std::vector<PlaneRec<R>> planes;
    std::vector<BoxRec<R>> boxes;
    std::vector<TriRec<R>> tris;
    std::vector<MatRec<R>> mats;
    std::vector<int> perm;
    // BVH leaf-order records (bvh_sphere_leaf[k] describes spheres[bvh_sphere_leaf[k].id], same for
    // triangles)
    std::vector<SphereLeaf<R>> bvh_sphere_leaf;
    std::vector<TriLeaf<R>> bvh_tri_leaf;
    std::vector<TriFilter> tri_filter;            // binary64: bvh_tri_leaf's binary32 pre-filter records
    std::vector<SphereLeaf<R>> big_sphere_leaf;   // HostScene::big_spheres, tested before the walk
    std::vector<SphereLeaf<R>> grid_leaf;         // HostScene::grid_ids, cell by cell
};

template <class R>
void make_records(const HostScene& hs, const rt_scene_desc& d, HostRecords<R>& out) {
    out.spheres.resize(hs.sphere_r.size());
    for (size_t i = 0; i < out.spheres.size(); ++i) {
        const double* s = &hs.spheres[4 * i];
        const R r = (R)hs.sphere_r[i];
        // binary64: r*r once, bit-identical to geometry.js:19's per-call radius*radius
        out.spheres[i] = SphereRec<R>{(R)s[0], (R)s[1], (R)s[2], sizeof(R) == 8 ? (R)s[3] : r * r};
    }
    out.sphere_r.assign(hs.sphere_r.begin(), hs.sphere_r.end());
    out.sphere_inv_r.resize(out.sphere_r.size());
    for (size_t i = 0; i < out.sphere_r.size(); ++i) out.sphere_inv_r[i] = (R)1 / out.sphere_r[i];
    out.sphere_filter.resize(hs.sphere_r.size());
    for (size_t i = 0; i < out.sphere_filter.size(); ++i) {
        const double* s = &hs.spheres[4 * i];
        const double k = 2.0 * (s[0] * s[0] + s[1] * s[1] + s[2] * s[2]) + s[3];
        // r2p = r^2 + 2^RT_FILTER_MARGIN k, rounded up (sphere_filter_bound in pt_core.h)
        out.sphere_filter[i] = SphereFilter{(float)s[0], (float)s[1], (float)s[2],
                                            (float)((s[3] + filter_margin() * k) * (1.0 + 0x1p-20))};
    }
    out.planes.resize(hs.plane_mat.size());
    for (size_t i = 0; i < out.planes.size(); ++i) {
        const double* p = &hs.planes[6 * i];
        out.planes[i] = PlaneRec<R>{(R)p[0], (R)p[1], (R)p[2], (R)p[3], (R)p[4], (R)p[5]};
    }
    out.boxes.resize(hs.box_mat.size());
    for (size_t i = 0; i < out.boxes.size(); ++i) {
        const double* b = &hs.boxes[6 * i];
        out.boxes[i] = BoxRec<R>{(R)b[0], (R)b[1], (R)b[2], (R)b[3], (R)b[4], (R)b[5]};
    }
    out.tris.resize(hs.tri_mat.size());
    for (size_t i = 0; i < out.tris.size(); ++i) {
        const double* t = &hs.tris[12 * i];
        out.tris[i] = TriRec<R>{(R)t[0], (R)t[1], (R)t[2], (R)t[3], (R)t[4],  (R)t[5],
                                (R)t[6], (R)t[7], (R)t[8], (R)t[9], (R)t[10], (R)t[11]};
    }
    out.mats.resize(d.num_materials);
    for (int i = 0; i < d.num_materials; ++i) {
        const rt_material_desc& m = d.materials[i];
        MatRec<R> r{};
        r.type = m.type;
        const double* c = m.type == RT_MAT_EMISSIVE ? m.emission : m.albedo;
        for (int k = 0; k < 3; ++k) r.c[k] = (R)c[k];
        r.p = (R)(m.type == RT_MAT_METAL ? m.roughness : m.ior);
        if (m.type == RT_MAT_DIELECTRIC) {
            // the two refraction ratios' values that Dielectric.scatter derives from the index alone,
            // in R arithmetic exactly as the kernel would (materials.js:53, :79-80): c[0] = 1 / ior (the
            // front face's ratio), c[1] / c[2] = Schlick's r0 for the front / back face's ratio
            const R ior = r.p, inv = (R)1 / ior;
            R f = ((R)1 - inv) / ((R)1 + inv), bk = ((R)1 - ior) / ((R)1 + ior);
            r.c[0] = inv;
            r.c[1] = f * f;
            r.c[2] = bk * bk;
        }
        out.mats[i] = r;
    }
    out.perm.assign(d.perm, d.perm + 512);
    auto leaf = [&](int id) {
        SphereLeaf<R> L{};
        if constexpr (sizeof(R) == 8) L.f = out.sphere_filter[id];
        L.s = out.spheres[id];
        L.id = id;
        L.obj = hs.sphere_obj[id];
        L.mat = hs.sphere_mat[id];
        return L;
    };
    for (int id : hs.sphere_bvh_prims) out.bvh_sphere_leaf.push_back(leaf(id));
    for (int id : hs.big_spheres) out.big_sphere_leaf.push_back(leaf(id));
    for (int id : hs.grid_ids) out.grid_leaf.push_back(leaf(id));
    for (int id : hs.tri_bvh_prims) {
        const TriRec<R>& r = out.tris[id];
        out.bvh_tri_leaf.push_back(TriLeaf<R>{{r.v0x, r.v0y, r.v0z, r.e1x, r.e1y, r.e1z, r.e2x, r.e2y, r.e2z},
                                              id, hs.tri_obj[id]});
        if constexpr (sizeof(R) == 8) out.tri_filter.push_back(make_tri_filter(&hs.tris[12 * (size_t)id]));
    }
}

// Camera / background constants of the SceneView (pointers are set by the caller).
template <class R>
void fill_view_constants(SceneView<R>& v, const HostScene& hs, const rt_scene_desc& d) {
    v.num_runs = (int)hs.runs.size();
    v.num_spheres = (int)hs.sphere_r.size();
    v.num_prims = hs.num_prims;
    v.num_planes = (int)hs.plane_mat.size();
    v.num_mats = d.num_materials;
    v.num_boxes = (int)hs.box_mat.size();
    v.num_sphere_nodes = (int)hs.sphere_bvh.size();
    v.num_tri_nodes = (int)hs.tri_bvh.size();
    v.num_sphere_wide = (int)hs.sphere_wide.size();
    v.num_tri_wide = (int)hs.tri_wide.size();
    v.num_big_spheres = (int)hs.big_spheres.size();
    v.num_grid_cells = hs.grid_n[0] * hs.grid_n[1] * hs.grid_n[2];
    v.num_grid_recs = (int)hs.grid_ids.size();
    for (int k = 0; k < 3; ++k) {
        v.grid_n[k] = hs.grid_n[k];
        v.grid_lo[k] = hs.grid_lo[k];
        v.grid_hi[k] = hs.grid_hi[k];
        v.grid_cs[k] = hs.grid_cs[k];
        v.grid_ics[k] = hs.grid_cs[k] > 0.0f ? 1.0f / hs.grid_cs[k] : 0.0f;
    }
    v.grid_far = hs.grid_far;
    v.use_grid = hs.use_grid ? 1 : 0;
    v.stack_entries = std::max(1, hs.bvh_depth);
    v.exit_k0 = hs.exit_k0; v.exit_k1 = hs.exit_k1; v.exit_k2 = hs.exit_k2;
    v.exit_l1 = hs.exit_l1; v.exit_l2 = hs.exit_l2;
    const rt_camera_desc& c = d.camera;
    for (int k = 0; k < 3; ++k) {
        v.cam_o[k] = (R)c.origin[k];
        v.cam_llc[k] = (R)c.lower_left[k];
        v.cam_h[k] = (R)c.horizontal[k];
        v.cam_v[k] = (R)c.vertical[k];
        v.cam_u[k] = (R)c.u[k];
        v.cam_vv[k] = (R)c.v[k];
        v.cam_w[k] = (R)c.w[k];
        v.solid[k] = (R)d.solid_color[k];
    }
    v.lens_radius = (R)c.lens_radius;
    v.cam_ortho = c.type == RT_CAM_ORTHOGRAPHIC;
    v.background = d.background;
    v.sky_intensity = (R)d.sky_intensity;
}

inline uint32_t host_seed_mix(uint32_t seed) {
    uint32_t x = seed ^ 0x3C6EF372U;
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// Walk choice for a sphere-only scene with a grid: the BVH and the grid walk give the same closest hit,
// so the choice is about speed only.  Both host walks (the kernel's own code) run over a sample of the
// scene's rays — a 48 x 27 raster of pixel-centre camera rays and, from each hit, one ray in a random
// direction — and the grid is chosen when its estimated cost (cells + 0.5 per sphere test) is below
// 0.8 x the tree's (nodes + 0.5 per sphere test); RTOW: ~3.9 vs ~8.0.
#ifndef RT_GRID_CHOICE
#define RT_GRID_CHOICE 0.8
#endif
// A binary64 SceneView over host copies of the records (the host walks of choose_walk)
inline SceneView<double> host_view(const HostScene& hs, const rt_scene_desc& d, HostRecords<double>& rec) {
    make_records(hs, d, rec);
    SceneView<double> v{};
    v.runs = hs.runs.data();
    v.spheres = rec.spheres.data(); v.sphere_filter = rec.sphere_filter.data(); v.sphere_r = rec.sphere_r.data();
    v.sphere_inv_r = rec.sphere_inv_r.data();
    v.planes = rec.planes.data(); v.boxes = rec.boxes.data(); v.tris = rec.tris.data();
    v.sphere_mat = hs.sphere_mat.data(); v.plane_mat = hs.plane_mat.data(); v.box_mat = hs.box_mat.data();
    v.tri_mat = hs.tri_mat.data(); v.mats = rec.mats.data(); v.perm = rec.perm.data();
    v.plane_obj = hs.plane_obj.data(); v.box_obj = hs.box_obj.data();
    v.sphere_nodes = hs.sphere_bvh.data(); v.tri_nodes = hs.tri_bvh.data();
    v.bvh_sphere_leaf = rec.bvh_sphere_leaf.data(); v.bvh_tri_leaf = rec.bvh_tri_leaf.data();
    v.tri_filter = rec.tri_filter.data(); v.tri_exit = hs.tri_exit.data();
    v.big_spheres = rec.big_sphere_leaf.data();
    v.sphere_wide = hs.sphere_wide.data(); v.tri_wide = hs.tri_wide.data();
    v.grid_cell = hs.grid_cell.data(); v.grid_leaf = rec.grid_leaf.data();
    fill_view_constants(v, hs, d);
    return v;
}

inline void choose_walk(HostScene& hs, const rt_scene_desc& d) {
    hs.use_grid = false;
    if (hs.grid_n[0] * hs.grid_n[1] * hs.grid_n[2] <= 0 || !hs.tri_mat.empty() || hs.bvh_depth > 64) return;
    HostRecords<double> rec;
    const SceneView<double> v = host_view(hs, d, rec);
    const rt_camera_desc& c = d.camera;
    int stack[64];
    double tree = 0, grid = 0;
    uint32_t rng = 0x9e3779b9u;
    auto uni = [&]() { rng = rng * 1664525u + 1013904223u; return (double)(rng >> 8) * 0x1p-24 * 2.0 - 1.0; };
    for (int j = 0; j < 27; ++j)
        for (int i = 0; i < 48; ++i) {
            const double u = (i + 0.5) / 48, w = (j + 0.5) / 27;
            V3<double> o{c.origin[0], c.origin[1], c.origin[2]};
            V3<double> dir{c.lower_left[0] + u * c.horizontal[0] + w * c.vertical[0] - o.x,
                           c.lower_left[1] + u * c.horizontal[1] + w * c.vertical[1] - o.y,
                           c.lower_left[2] + u * c.horizontal[2] + w * c.vertical[2] - o.z};
            for (int bounce = 0; bounce < 2; ++bounce) {
                Work wt{}, wg{};
                const Closest<double> h = closest_hit_bvh<double, true, false>(v, o, dir, wt, BvhStack{stack, 1});
                closest_hit_grid<double>(v, o, dir, wg, BvhStack{stack, 1});
                tree += wt.nodes + 0.5 * wt.spheres;
                grid += wg.nodes + 0.5 * wg.spheres;
                if (h.kind == HIT_NONE) break;
                o = o + dir * h.t;
                dir = V3<double>{uni(), uni(), uni()};
            }
        }
    hs.use_grid = grid < RT_GRID_CHOICE * tree;
    if (getenv("RT_WALK_DEBUG"))
        fprintf(stderr, "[rt] walk choice: tree %.3g, grid %.3g (%d x %d x %d cells) -> %s\n", tree, grid, hs.grid_n[0],
                hs.grid_n[1], hs.grid_n[2], hs.use_grid ? "grid" : "tree");
}

}  // namespace rt
