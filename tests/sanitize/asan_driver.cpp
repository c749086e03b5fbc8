// asan_driver.cpp — TEST INFRASTRUCTURE (SURVEY §5 "sanitizers on the host CPU restatement"): the host
// code of the path built with -fsanitize=address,undefined and run on the repository's scenes:
//   * the C++ scene-JSON loader of librt_hip.so (csrc/scene_json.cpp) and the host scene packing and
//     BVH builder (csrc/scene_pack.h, via tests/hostcheck),
//   * the kernel's own per-lane code compiled for the CPU (tests/hostcheck/pt_hostcheck.cpp): World
//     order, the two-child BVH walk and the stackless walk,
//   * the C oracle (oracle/pt_oracle.c).
// Every scene renders a crop with each of them; segment / draw counts must agree exactly and the
// means within 1e-12.  Any sanitizer report aborts the process (halt_on_error / -fno-sanitize-recover).
// usage: asan_driver scene.json...
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_scene_json.h"

extern "C" int orc_render(const rt_scene_desc* sc, const rt_settings* st, double* mean, double* post, uint8_t* rgba,
                          uint32_t* segs, uint32_t* draws);
extern "C" int ptc_render(const rt_scene_desc* d, const rt_settings* s, double* sum, uint32_t* segs, uint32_t* draws);

namespace rt {
int set_error(int code, const char* msg) {   // rt_capi.cpp's error hook (the driver has no librt_hip.so)
    std::fprintf(stderr, "loader: %s\n", msg);
    return code;
}
}  // namespace rt

int main(int argc, char** argv) {
    int bad = 0;
    for (int a = 1; a < argc; ++a) {
        FILE* f = std::fopen(argv[a], "rb");
        if (!f) { std::fprintf(stderr, "%s: cannot open\n", argv[a]); return 2; }
        std::string json;
        char buf[1 << 16];
        size_t k;
        while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) json.append(buf, k);
        std::fclose(f);
        rt_json_scene* js = nullptr;
        if (rt_json_scene_load(json.data(), json.size(), 96, 64, 7, &js) != RT_OK) { std::fprintf(stderr, "%s: load failed\n", argv[a]); return 2; }
        const rt_scene_desc* d = rt_json_scene_desc(js);
        int32_t W = 0, H = 0;
        rt_json_scene_size(js, &W, &H);
        rt_settings st{};
        st.width = W; st.height = H; st.samples = 3; st.max_depth = 5; st.aa_mode = RT_AA_SUPERSAMPLING;
        st.exposure = 1; st.gamma = 2.2; st.seed = 11;
        st.crop_w = W < 12 ? W : 12; st.crop_h = H < 9 ? H : 9;
        st.crop_x0 = (W - st.crop_w) / 2; st.crop_y0 = (H - st.crop_h) / 2;
        const size_t n = (size_t)st.crop_w * st.crop_h;
        std::vector<double> om(3 * n), op(3 * n), sum(3 * n);
        std::vector<uint8_t> rgba(4 * n);
        std::vector<uint32_t> os(n), od(n), hs(n), hd(n);
        orc_render(d, &st, om.data(), op.data(), rgba.data(), os.data(), od.data());
        for (int accel : {(int)RT_ACCEL_BRUTE, (int)RT_ACCEL_BVH, 3}) {        // 3: hostcheck's stackless walk
            st.accel = accel;
            std::fill(sum.begin(), sum.end(), 0.0);
            if (ptc_render(d, &st, sum.data(), hs.data(), hd.data()) != 0) { std::fprintf(stderr, "%s: hostcheck failed\n", argv[a]); return 2; }
            for (size_t q = 0; q < n; ++q) {
                bool ok = hs[q] == os[q] && hd[q] == od[q];
                for (int c = 0; c < 3; ++c) {
                    const double m = sum[3 * q + c] / st.samples, o = om[3 * q + c];
                    if (!(std::isnan(m) && std::isnan(o)) && !(std::fabs(m - o) <= 1e-12 * std::fmax(1.0, std::fabs(o)))) ok = false;
                }
                if (!ok) { ++bad; std::fprintf(stderr, "%s accel %d pixel %zu differs\n", argv[a], accel, q); break; }
            }
        }
        std::printf("%s: %dx%d crop %dx%d ok\n", argv[a], W, H, st.crop_w, st.crop_h);
        rt_json_scene_destroy(js);
    }
    return bad ? 1 : 0;
}
