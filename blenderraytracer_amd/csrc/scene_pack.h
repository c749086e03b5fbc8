// scene_pack.h — rt_scene_desc (include/rt_hip.h) -> the kernel's record arrays.
//
// World objects are grouped into runs of consecutive same-kind objects, preserving the
// World.objects insertion order that decides ties (js/world.js:24-30).  A mesh is always its own
// run: inside it the LAST equal-t triangle wins (geometry.js:253-259).
#pragma once
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "pt_core.h"

namespace rt {

struct HostScene {   // precision-independent staging, binary64 as packed by the host
    std::vector<Run> runs;
    std::vector<double> spheres, sphere_r, planes, boxes, tris;   // 4, 1, 6, 6, 12 doubles per record
    std::vector<int> sphere_mat, plane_mat, box_mat, tri_mat;
    int num_prims = 0;
    double record_bytes = 0;      // SURVEY §8d canonical bytes tested per segment
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
            push_run(RUN_SPHERES, k, k + 1, -1);
            hs.num_prims += 1;
            hs.record_bytes += 16;
            break;
        }
        case RT_OBJ_PLANE: {
            const int k = (int)hs.plane_mat.size();
            hs.planes.insert(hs.planes.end(), o.g, o.g + 6);
            hs.plane_mat.push_back(o.material);
            push_run(RUN_PLANES, k, k + 1, -1);
            hs.num_prims += 1;
            hs.record_bytes += 24;
            break;
        }
        case RT_OBJ_BOX: {
            const int k = (int)hs.box_mat.size();
            hs.boxes.insert(hs.boxes.end(), o.g, o.g + 6);
            hs.box_mat.push_back(o.material);
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

// Record arrays of one precision (host memory); rt_capi.cpp uploads them, tests/hostcheck uses them.
template <class R>
struct HostRecords {
    std::vector<SphereRec<R>> spheres;
    std::vector<SphereFilter> sphere_filter;
    std::vector<R> sphere_r;
    std::vector<PlaneRec<R>> planes;
    std::vector<BoxRec<R>> boxes;
    std::vector<TriRec<R>> tris;
    std::vector<MatRec<R>> mats;
    std::vector<int> perm;
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
    out.sphere_filter.resize(hs.sphere_r.size());
    for (size_t i = 0; i < out.sphere_filter.size(); ++i) {
        const double* s = &hs.spheres[4 * i];
        const double k = 2.0 * (s[0] * s[0] + s[1] * s[1] + s[2] * s[2]) + s[3];
        // r2p = r^2 + 2^-17 k, rounded up (sphere_filter_bound in pt_core.h)
        out.sphere_filter[i] = SphereFilter{(float)s[0], (float)s[1], (float)s[2], (float)((s[3] + 0x1p-17 * k) * (1.0 + 0x1p-20))};
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
        for (int k = 0; k < 3; ++k) {
            r.albedo[k] = (R)m.albedo[k];
            r.emit[k] = (R)m.emission[k];
        }
        r.rough = (R)m.roughness;
        r.ior = (R)m.ior;
        out.mats[i] = r;
    }
    out.perm.assign(d.perm, d.perm + 512);
}

// Camera / background constants of the SceneView (pointers are set by the caller).
template <class R>
void fill_view_constants(SceneView<R>& v, const HostScene& hs, const rt_scene_desc& d) {
    v.num_runs = (int)hs.runs.size();
    v.num_spheres = (int)hs.sphere_r.size();
    v.num_prims = hs.num_prims;
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

}  // namespace rt
