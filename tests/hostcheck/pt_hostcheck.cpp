// pt_hostcheck.cpp — TEST INFRASTRUCTURE: runs the megakernel's per-lane code (pt_path.h,
// pt_core.h, scene_pack.h — the very same source the GPU kernel compiles) on the CPU, one pixel at a
// time, so CPU-only tests can check the flattened path loop, the run packing and the record layout
// against the oracle.  Built host-only; never part of librt_hip.so, never loaded by product code.
#include <string>

#include "../../blenderraytracer_amd/csrc/pt_path.h"
#include "../../blenderraytracer_amd/csrc/scene_pack.h"

using namespace rt;

template <class R>
static int render(const rt_scene_desc* d, const rt_settings* s, double* sum, uint32_t* segs, uint32_t* draws) {
    HostScene hs;
    std::string err;
    if (!pack_host(*d, hs, err)) return -1;
    HostRecords<R> rec;
    make_records(hs, *d, rec);
    SceneView<R> v{};
    v.runs = hs.runs.data();
    v.spheres = rec.spheres.data(); v.sphere_r = rec.sphere_r.data(); v.planes = rec.planes.data();
    v.boxes = rec.boxes.data(); v.tris = rec.tris.data(); v.sphere_mat = hs.sphere_mat.data();
    v.plane_mat = hs.plane_mat.data(); v.box_mat = hs.box_mat.data(); v.tri_mat = hs.tri_mat.data();
    v.mats = rec.mats.data(); v.perm = rec.perm.data();
    fill_view_constants(v, hs, *d);
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
    for (int cy = 0; cy < im.ch; ++cy)
        for (int cx = 0; cx < im.cw; ++cx) {
            const size_t q = (size_t)cy * im.cw + cx;
            PixelResult r{0, 0};
            if (im.max_depth > 0) r = trace_pixel<R, true>(v, im, cx, cy, im.s_end, sum + 3 * q);
            segs[q] = r.segments;
            draws[q] = r.draws;
        }
    return 0;
}

extern "C" int ptc_render(const rt_scene_desc* d, const rt_settings* s, double* sum, uint32_t* segs, uint32_t* draws) {
    return s->precision == RT_PREC_F32 ? render<float>(d, s, sum, segs, draws) : render<double>(d, s, sum, segs, draws);
}
