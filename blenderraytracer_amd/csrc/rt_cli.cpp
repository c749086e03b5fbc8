// rt_cli.cpp — Node-free command line front end of librt_hip.so (SURVEY §8b "a C++ bench CLI").
//
//   rt_render_cli scene.json [--width W] [--height H] [--spp S] [--depth D] [--seed N]
//                 [--aa supersampling|stochastic|none] [--tone reinhard|aces|linear]
//                 [--exposure E] [--gamma G] [--denoise STRENGTH] [--precision f64|f32]
//                 [--accel auto|bvh|brute] [--frames K] [--warmup W] [--batch B] [--device N]
//                 [--out image.ppm|image.pam]
//
// Does what a reference user does in the browser: RayTracer(width, height) -> loadFromJSON(scene)
// (rt_json_scene_load: scene-loader.js semantics incl. a camera "resolution" resize) ->
// updateRenderSettings({...}) (ray-tracer.js:554-566, `||` defaults) -> render() (rt_render).
// Prints one JSON line with the timing of the timed frames; writes the RGBA8 image of the last
// frame as binary PPM (RGB) or PAM (RGBA).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "../../include/rt_scene_json.h"
#include "js_math.h"

namespace {

[[noreturn]] void die(const char* what, const char* detail = "") {
    fprintf(stderr, "rt_render_cli: %s%s\n", what, detail);
    exit(2);
}

void check(int status, const char* what) {
    if (status != RT_OK) die(what, (std::string(": ") + rt_last_error()).c_str());
}

std::string read_file(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) die("cannot open ", path);
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    return s;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// `value || dflt` for a numeric setting (updateRenderSettings, ray-tracer.js:556-565)
double js_or(double v, double dflt) { return (v == 0 || v != v) ? dflt : v; }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2 || !strcmp(argv[1], "--help")) {
        fprintf(stderr, "usage: rt_render_cli scene.json [--width W --height H --spp S --depth D --seed N --aa MODE "
                        "--tone MAP --exposure E --gamma G --denoise STRENGTH --precision f64|f32 --accel auto|bvh|brute "
                        "--frames K --warmup W --batch B --device N --out FILE]\n");
        return argc < 2 ? 2 : 0;
    }
    const char* scene_path = argv[1];
    int width = 800, height = 600, frames = 1, warmup = 0, batch = 0, device = 0;
    double spp = 4, depth = 5, exposure = 1.0, gamma = 2.2, denoise = 0;
    uint32_t seed = 1;
    std::string aa = "supersampling", tone = "reinhard", precision = "f64", accel = "auto", out;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (i + 1 >= argc) die("missing value for ", a.c_str());
        const char* v = argv[++i];
        if (a == "--width") width = atoi(v);
        else if (a == "--height") height = atoi(v);
        else if (a == "--spp") spp = atof(v);
        else if (a == "--depth") depth = atof(v);
        else if (a == "--seed") seed = (uint32_t)strtoul(v, nullptr, 0);
        else if (a == "--aa") aa = v;
        else if (a == "--tone") tone = v;
        else if (a == "--exposure") exposure = atof(v);
        else if (a == "--gamma") gamma = atof(v);
        else if (a == "--denoise") denoise = atof(v);
        else if (a == "--precision") precision = v;
        else if (a == "--accel") accel = v;
        else if (a == "--frames") frames = atoi(v);
        else if (a == "--warmup") warmup = atoi(v);
        else if (a == "--batch") batch = atoi(v);
        else if (a == "--device") device = atoi(v);
        else if (a == "--out") out = v;
        else die("unknown option ", a.c_str());
    }
    if (frames < 1 || warmup < 0) die("--frames must be >= 1 and --warmup >= 0");

    const std::string text = read_file(scene_path);
    rt_json_scene* js = nullptr;
    check(rt_json_scene_load(text.data(), text.size(), width, height, seed, &js), "loading the scene");
    rt_json_scene_size(js, &width, &height);                 // a camera "resolution" resizes
    rt_scene* scene = nullptr;
    const double t_up = now_ms();
    check(rt_scene_create(rt_json_scene_desc(js), device, &scene), "uploading the scene");
    const double upload_ms = now_ms() - t_up;

    rt_settings s{};
    s.width = width;
    s.height = height;
    s.samples = aa == "none" ? 1 : (int)js_or(spp, 4);     // sampleCount (ray-tracer.js:201)
    s.max_depth = (int)js_or(depth, 5);
    s.aa_mode = aa == "supersampling" ? RT_AA_SUPERSAMPLING : (aa == "stochastic" ? RT_AA_STOCHASTIC : RT_AA_CENTER);
    s.tone_map = tone == "aces" ? RT_TM_ACES : (tone == "linear" ? RT_TM_LINEAR : RT_TM_REINHARD);
    s.exposure = js_or(exposure, 1.0);
    s.gamma = js_or(gamma, 2.2);
    s.seed = seed;
    s.precision = precision == "f32" ? RT_PREC_F32 : RT_PREC_F64;
    s.accel = accel == "bvh" ? RT_ACCEL_BVH : (accel == "brute" ? RT_ACCEL_BRUTE : RT_ACCEL_AUTO);
    s.batch_samples = batch;
    if (denoise > 0) {                                       // post-processor.js:55 weights, host exp
        s.denoise = 1;
        s.denoise_weights[0] = jsm::exp(-1.0 / (2 * denoise * denoise));   // V8's Math.exp (post-processor.js:60)
        s.denoise_weights[1] = jsm::exp(-2.0 / (2 * denoise * denoise));
    }
    const size_t n = (size_t)width * height;
    std::vector<uint8_t> rgba(4 * n);
    rt_output o{};
    o.rgba8 = rgba.data();
    rt_stats st{};
    for (int k = 0; k < warmup; ++k) check(rt_render(scene, &s, &o, nullptr, nullptr, &st), "rendering");
    double wall = 0, kernel = 0;
    uint64_t segments = 0, nodes = 0;
    for (int k = 0; k < frames; ++k) {
        const double t0 = now_ms();
        check(rt_render(scene, &s, &o, nullptr, nullptr, &st), "rendering");
        wall += now_ms() - t0;
        kernel += st.kernel_ms;
        segments += st.segments;
        nodes += st.node_visits;
    }
    const double samples = (double)n * s.samples * frames;
    printf("{\"scene\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d, \"max_depth\": %d, \"precision\": \"%s\", "
           "\"accel\": \"%s\", \"frames\": %d, \"msamples_per_s\": %.3f, \"kernel_msamples_per_s\": %.3f, "
           "\"ms_per_frame\": %.3f, \"kernel_ms_per_frame\": %.3f, \"upload_ms\": %.3f, \"segments_per_sample\": %.4f, "
           "\"bvh_nodes_per_segment\": %.3f}\n",
           scene_path, width, height, s.samples, s.max_depth, precision.c_str(), accel.c_str(), frames,
           samples / (wall * 1e-3) / 1e6, samples / (kernel * 1e-3) / 1e6, wall / frames, kernel / frames, upload_ms,
           segments / samples, segments ? (double)nodes / segments : 0.0);
    if (!out.empty()) {
        FILE* f = fopen(out.c_str(), "wb");
        if (!f) die("cannot write ", out.c_str());
        const bool pam = out.size() > 4 && out.compare(out.size() - 4, 4, ".pam") == 0;
        if (pam) {
            fprintf(f, "P7\nWIDTH %d\nHEIGHT %d\nDEPTH 4\nMAXVAL 255\nTUPLTYPE RGB_ALPHA\nENDHDR\n", width, height);
            fwrite(rgba.data(), 1, rgba.size(), f);
        } else {
            fprintf(f, "P6\n%d %d\n255\n", width, height);
            std::vector<uint8_t> rgb(3 * n);
            for (size_t q = 0; q < n; ++q) memcpy(&rgb[3 * q], &rgba[4 * q], 3);
            fwrite(rgb.data(), 1, rgb.size(), f);
        }
        fclose(f);
    }
    rt_scene_destroy(scene);
    rt_json_scene_destroy(js);
    return 0;
}
