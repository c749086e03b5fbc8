// scene_json.cpp — RayTracer.loadFromJSON / SceneLoader.loadFromJSON in C++ (include/rt_scene_json.h).
//
// A small JSON reader (RFC 8259; duplicate keys: the last wins, as JSON.parse) plus the reference
// loader's JavaScript value semantics, evaluated in binary64 in the reference's operation order so
// the packed camera vectors and plane/triangle normals are bit-identical to the JS objects
// (tests/test_scene_json.py compares them with the Python host and the JS host).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rt_scene_json.h"
#include "js_math.h"
#include "pt_core.h"
#include "scene_pack.h"

namespace rt {
int set_error(int code, const char* msg);   // rt_capi.cpp: rt_last_error()'s thread-local message
}

namespace {

// ---- JSON values ------------------------------------------------------------------------------------
struct JVal {
    enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
    bool b = false;
    double n = 0;
    std::string s;
    std::vector<JVal> a;
    std::vector<std::pair<std::string, JVal>> o;
    const JVal* get(const char* key) const {       // undefined -> nullptr; duplicate keys: last wins
        if (t != Obj) return nullptr;
        for (size_t i = o.size(); i-- > 0;)
            if (o[i].first == key) return &o[i].second;
        return nullptr;
    }
};

struct Parser {
    const char* p;
    const char* end;
    std::string err;
    int depth = 0;

    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool fail(const char* what) {
        if (err.empty()) {
            char buf[96];
            snprintf(buf, sizeof buf, "JSON: %s", what);
            err = buf;
        }
        return false;
    }
    static void utf8(std::string& s, unsigned cp) {
        if (cp < 0x80) s += (char)cp;
        else if (cp < 0x800) { s += (char)(0xC0 | cp >> 6); s += (char)(0x80 | (cp & 63)); }
        else if (cp < 0x10000) { s += (char)(0xE0 | cp >> 12); s += (char)(0x80 | (cp >> 6 & 63)); s += (char)(0x80 | (cp & 63)); }
        else { s += (char)(0xF0 | cp >> 18); s += (char)(0x80 | (cp >> 12 & 63)); s += (char)(0x80 | (cp >> 6 & 63)); s += (char)(0x80 | (cp & 63)); }
    }
    bool hex4(unsigned& v) {
        if (end - p < 4) return fail("bad \\u escape");
        v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return fail("bad \\u escape");
        }
        return true;
    }
    bool string(std::string& s) {
        ++p;   // opening quote
        while (p < end && *p != '"') {
            const unsigned char c = (unsigned char)*p++;
            if (c < 0x20) return fail("control character in string");
            if (c != '\\') { s += (char)c; continue; }
            if (p >= end) return fail("unterminated string");
            const char e = *p++;
            switch (e) {
            case '"': s += '"'; break;
            case '\\': s += '\\'; break;
            case '/': s += '/'; break;
            case 'b': s += '\b'; break;
            case 'f': s += '\f'; break;
            case 'n': s += '\n'; break;
            case 'r': s += '\r'; break;
            case 't': s += '\t'; break;
            case 'u': {
                unsigned cp;
                if (!hex4(cp)) return false;
                if (cp >= 0xD800 && cp < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                    p += 2;
                    unsigned lo;
                    if (!hex4(lo)) return false;
                    cp = (lo >= 0xDC00 && lo < 0xE000) ? 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00) : 0xFFFD;
                }
                utf8(s, cp);
                break;
            }
            default: return fail("bad escape");
            }
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    bool number(double& v) {
        const char* s = p;
        if (p < end && *p == '-') ++p;
        if (p < end && *p == '0') ++p;
        else if (p < end && *p >= '1' && *p <= '9') while (p < end && *p >= '0' && *p <= '9') ++p;
        else return fail("bad number");
        if (p < end && *p == '.') {
            ++p;
            if (!(p < end && *p >= '0' && *p <= '9')) return fail("bad number");
            while (p < end && *p >= '0' && *p <= '9') ++p;
        }
        if (p < end && (*p == 'e' || *p == 'E')) {
            ++p;
            if (p < end && (*p == '+' || *p == '-')) ++p;
            if (!(p < end && *p >= '0' && *p <= '9')) return fail("bad number");
            while (p < end && *p >= '0' && *p <= '9') ++p;
        }
        const std::string tok(s, p);
        v = strtod(tok.c_str(), nullptr);   // correctly rounded, like JSON.parse
        return true;
    }
    bool literal(const char* w) {
        const size_t n = strlen(w);
        if ((size_t)(end - p) < n || memcmp(p, w, n) != 0) return fail("bad literal");
        p += n;
        return true;
    }
    bool value(JVal& v) {
        if (++depth > 512) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end");
        bool ok = true;
        switch (*p) {
        case '{': {
            v.t = JVal::Obj;
            ++p;
            ws();
            if (p < end && *p == '}') { ++p; break; }
            for (;;) {
                ws();
                if (p >= end || *p != '"') { ok = fail("expected key"); break; }
                std::pair<std::string, JVal> kv;
                if (!(ok = string(kv.first))) break;
                ws();
                if (p >= end || *p != ':') { ok = fail("expected ':'"); break; }
                ++p;
                if (!(ok = value(kv.second))) break;
                v.o.push_back(std::move(kv));
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == '}') { ++p; break; }
                ok = fail("expected ',' or '}'");
                break;
            }
            break;
        }
        case '[': {
            v.t = JVal::Arr;
            ++p;
            ws();
            if (p < end && *p == ']') { ++p; break; }
            for (;;) {
                v.a.emplace_back();
                if (!(ok = value(v.a.back()))) break;
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == ']') { ++p; break; }
                ok = fail("expected ',' or ']'");
                break;
            }
            break;
        }
        case '"': v.t = JVal::Str; ok = string(v.s); break;
        case 't': v.t = JVal::Bool; v.b = true; ok = literal("true"); break;
        case 'f': v.t = JVal::Bool; v.b = false; ok = literal("false"); break;
        case 'n': v.t = JVal::Null; ok = literal("null"); break;
        default: v.t = JVal::Num; ok = number(v.n); break;
        }
        --depth;
        return ok;
    }
};

// ---- JavaScript value semantics (the loader reads raw JSON values) ---------------------------------
bool truthy(const JVal* v) {                       // ToBoolean; nullptr = undefined
    if (!v) return false;
    switch (v->t) {
    case JVal::Null: return false;
    case JVal::Bool: return v->b;
    case JVal::Num: return !(v->n == 0 || v->n != v->n);
    case JVal::Str: return !v->s.empty();
    default: return true;
    }
}

double str_to_number(const std::string& s) {       // ToNumber(String)
    size_t a = 0, b = s.size();
    while (a < b && strchr(" \t\n\r\v\f", s[a])) ++a;
    while (b > a && strchr(" \t\n\r\v\f", s[b - 1])) --b;
    if (a == b) return 0;
    const std::string t = s.substr(a, b - a);
    if (t == "Infinity" || t == "+Infinity") return INFINITY;
    if (t == "-Infinity") return -INFINITY;
    char* e = nullptr;
    const double v = strtod(t.c_str(), &e);
    if (*e != 0 || t.find_first_of("xXnN") != std::string::npos) return NAN;   // no hex floats / nan / inf words
    return v;
}

double num(const JVal* v) {                        // ToNumber as the arithmetic applies it
    if (!v) return NAN;                            // undefined
    switch (v->t) {
    case JVal::Null: return 0;
    case JVal::Bool: return v->b ? 1 : 0;
    case JVal::Num: return v->n;
    case JVal::Str: return str_to_number(v->s);
    case JVal::Arr:                                // ToPrimitive: [] -> "", [x] -> String(x)
        if (v->a.empty()) return 0;
        if (v->a.size() == 1) return v->a[0].t == JVal::Str ? str_to_number(v->a[0].s) : num(&v->a[0]);
        return NAN;
    default: return NAN;
    }
}

const JVal* js_or(const JVal* a, const JVal* b) { return truthy(a) ? a : b; }

struct V { double x, y, z; };
V vadd(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V vsub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V vmul(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
V vdiv(V a, double s) { return {a.x / s, a.y / s, a.z / s}; }
V vcross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double vlen(V a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
V vnorm(V a) {                                     // math.js:18
    const double l = vlen(a);
    return l > 0 ? vdiv(a, l) : V{0, 0, 0};
}

V parse_vec3(const JVal* v) {                      // scene-loader.js:268-273
    if (v && v->t == JVal::Arr && v->a.size() >= 3) return {num(&v->a[0]), num(&v->a[1]), num(&v->a[2])};
    return {0, 0, 0};
}

std::string lower(const std::string& s) {
    std::string r = s;
    for (char& c : r)
        if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    return r;
}

struct LoadError {
    std::string msg;
};

// `x.type.toLowerCase()` on a non-string throws in the reference; loadFromJSON then returns false
std::string type_of(const JVal* t, const char* what) {
    if (!t || t->t != JVal::Str) throw LoadError{std::string(what) + ".type is not a string"};
    return lower(t->s);
}

struct Camera {                                    // camera.js:8-36
    V origin, llc, horizontal, vertical, u, v, w;
    double lens_radius, fov, aperture, focus_dist;
    bool perspective, orthographic;
};

Camera make_camera(V from, V at, V vup, double vfov, double aspect, double aperture, double focus,
                   const std::string& type) {
    Camera c{};
    c.fov = vfov;
    c.aperture = aperture;
    c.focus_dist = focus;
    c.perspective = type == "perspective";
    c.orthographic = type == "orthographic";
    const double theta = vfov * M_PI / 180;
    const double h = jsm::tan(theta / 2);                  // V8's Math.tan (camera.js:15; js_math.h)
    const double vh = 2.0 * h;
    const double vw = aspect * vh;
    c.w = vnorm(vsub(from, at));
    c.u = vnorm(vcross(vup, c.w));
    c.v = vcross(c.w, c.u);
    c.origin = from;
    if (c.perspective) {
        c.horizontal = vmul(c.u, vw * focus);
        c.vertical = vmul(c.v, vh * focus);
        c.llc = vsub(vsub(vsub(c.origin, vdiv(c.horizontal, 2)), vdiv(c.vertical, 2)), vmul(c.w, focus));
    } else {
        c.horizontal = vmul(c.u, vw);
        c.vertical = vmul(c.v, vh);
        c.llc = vsub(vsub(c.origin, vdiv(c.horizontal, 2)), vdiv(c.vertical, 2));
    }
    c.lens_radius = aperture / 2;
    return c;
}

double js_or_num(double v, double dflt) { return (v == 0 || v != v) ? dflt : v; }

}  // namespace

struct rt_json_scene {
    std::vector<rt_object_desc> objects;
    std::vector<rt_material_desc> materials;
    std::vector<double> triangles;
    rt_scene_desc desc{};
    int32_t width = 0, height = 0;
};

namespace {

rt_material_desc make_material(const JVal* m) {   // scene-loader.js:143-173, materials.js constructors
    rt_material_desc d{};
    d.type = RT_MAT_LAMBERTIAN;
    d.albedo[0] = d.albedo[1] = d.albedo[2] = 0.8;
    if (!truthy(m) || !truthy(m->get("type"))) return d;
    const std::string t = type_of(m->get("type"), "material");
    if (t == "lambertian") {
        const V c = parse_vec3(m->get("color"));
        d.albedo[0] = c.x; d.albedo[1] = c.y; d.albedo[2] = c.z;
    } else if (t == "metal") {
        const V c = parse_vec3(m->get("color"));
        d.type = RT_MAT_METAL;
        d.albedo[0] = c.x; d.albedo[1] = c.y; d.albedo[2] = c.z;
        const JVal* r = m->get("roughness");
        const double rough = r ? num(r) : 0.0;
        d.roughness = rough != rough ? NAN : (rough < 1 ? rough : 1.0);   // Math.min(roughness, 1)
    } else if (t == "dielectric") {
        d.type = RT_MAT_DIELECTRIC;
        d.albedo[0] = d.albedo[1] = d.albedo[2] = 0;
        const JVal* ior = m->get("ior");
        d.ior = ior ? num(ior) : 1.5;
    } else if (t == "emissive") {
        d.type = RT_MAT_EMISSIVE;
        d.albedo[0] = d.albedo[1] = d.albedo[2] = 0;
        const V c = parse_vec3(m->get("color"));
        const JVal* in = m->get("intensity");
        const double inten = in ? num(in) : 1.0;
        const V e = vmul(c, inten);                 // color.mul(intensity), materials.js:95
        d.emission[0] = e.x; d.emission[1] = e.y; d.emission[2] = e.z;
    }
    return d;
}

void push_triangle(rt_json_scene& s, V v0, V v1, V v2) {   // geometry.js:138-146
    const V n = vnorm(vcross(vsub(v1, v0), vsub(v2, v0)));
    const double t[12] = {v0.x, v0.y, v0.z, v1.x, v1.y, v1.z, v2.x, v2.y, v2.z, n.x, n.y, n.z};
    s.triangles.insert(s.triangles.end(), t, t + 12);
}

bool is_index(const JVal& x) {
    return x.t == JVal::Num && x.n >= 0 && std::floor(x.n) == x.n && std::isfinite(x.n);
}

void create_object(rt_json_scene& s, const JVal& o) {      // scene-loader.js:90-137
    if (!truthy(o.get("type"))) return;                    // "Object has no type" -> skipped
    const JVal* mj = o.get("material");
    rt_material_desc mat;
    if (truthy(mj)) {
        mat = make_material(mj);
    } else {
        mat = rt_material_desc{};
        mat.type = RT_MAT_LAMBERTIAN;
        mat.albedo[0] = mat.albedo[1] = mat.albedo[2] = 0.8;
    }
    const std::string t = type_of(o.get("type"), "object");
    rt_object_desc d{};
    if (t == "sphere") {
        d.type = RT_OBJ_SPHERE;
        const V c = parse_vec3(o.get("center"));
        const JVal* r = o.get("radius");
        d.g[0] = c.x; d.g[1] = c.y; d.g[2] = c.z;
        d.g[3] = truthy(r) ? num(r) : 1.0;                 // radius || 1.0
    } else if (t == "plane") {
        d.type = RT_OBJ_PLANE;
        const V p = parse_vec3(o.get("point")), n = vnorm(parse_vec3(o.get("normal")));   // geometry.js:52
        d.g[0] = p.x; d.g[1] = p.y; d.g[2] = p.z; d.g[3] = n.x; d.g[4] = n.y; d.g[5] = n.z;
    } else if (t == "box") {
        d.type = RT_OBJ_BOX;
        const V a = parse_vec3(o.get("min")), b = parse_vec3(o.get("max"));
        d.g[0] = a.x; d.g[1] = a.y; d.g[2] = a.z; d.g[3] = b.x; d.g[4] = b.y; d.g[5] = b.z;
    } else if (t == "triangle") {
        d.type = RT_OBJ_TRIANGLE;
        d.first = (int32_t)(s.triangles.size() / 12);
        d.count = 1;
        push_triangle(s, parse_vec3(o.get("v0")), parse_vec3(o.get("v1")), parse_vec3(o.get("v2")));
    } else if (t == "mesh") {
        const JVal* vs = o.get("vertices");
        const JVal* is = o.get("indices");
        if (!truthy(vs) || !truthy(is)) return;            // "Mesh is missing vertices or indices"
        if (vs->t != JVal::Arr) throw LoadError{"mesh vertices is not an array"};   // .map throws
        std::vector<V> verts;
        for (const JVal& v : vs->a) verts.push_back(parse_vec3(&v));
        d.type = RT_OBJ_MESH;
        d.first = (int32_t)(s.triangles.size() / 12);
        if (is->t == JVal::Arr) {                          // geometry.js:193-237
            const size_t nv = verts.size();
            for (size_t i = 0; i < is->a.size(); i += 3) {
                if (i + 2 >= is->a.size()) continue;       // incomplete triangle
                const JVal* idx[3] = {&is->a[i], &is->a[i + 1], &is->a[i + 2]};
                bool skip = false;
                for (const JVal* x : idx) skip |= x->t == JVal::Num && x->n >= (double)nv;   // idx >= vertices.length
                if (skip) continue;
                V tv[3];
                for (int k = 0; k < 3; ++k) tv[k] = is_index(*idx[k]) ? verts[(size_t)idx[k]->n] : V{0, 0, 0};
                push_triangle(s, tv[0], tv[1], tv[2]);
            }
        }
        d.count = (int32_t)(s.triangles.size() / 12) - d.first;
    } else {
        return;                                            // "Unknown object type"
    }
    d.material = (int32_t)s.materials.size();
    s.materials.push_back(mat);
    s.objects.push_back(d);
}

Camera create_camera(const JVal& cam, double aspect) {     // scene-loader.js:205-262
    static const JVal d_pos = [] { JVal v; v.t = JVal::Arr; for (double x : {0.0, 0.0, 5.0}) { JVal e; e.t = JVal::Num; e.n = x; v.a.push_back(e); } return v; }();
    static const JVal d_at = [] { JVal v; v.t = JVal::Arr; for (double x : {0.0, 0.0, 0.0}) { JVal e; e.t = JVal::Num; e.n = x; v.a.push_back(e); } return v; }();
    static const JVal d_up = [] { JVal v; v.t = JVal::Arr; for (double x : {0.0, 1.0, 0.0}) { JVal e; e.t = JVal::Num; e.n = x; v.a.push_back(e); } return v; }();
    const V position = parse_vec3(js_or(cam.get("position"), &d_pos));
    V look_at = parse_vec3(js_or(cam.get("lookAt"), &d_at));
    const V up = parse_vec3(js_or(cam.get("up"), &d_up));
    const JVal* fj = cam.get("fov");
    const double fov = fj ? num(fj) : 45;
    const JVal* aj = cam.get("aperture");
    const double aperture = aj ? num(aj) : 0.0;
    if (vlen(vsub(position, look_at)) < 1.0) {
        const V direction = vmul(vnorm(vsub(position, look_at)), -1);
        look_at = vadd(position, vmul(direction, 100));
    }
    const JVal* fd = cam.get("focusDist");
    const double focus = fd ? num(fd) : vlen(vsub(position, look_at));
    const JVal* ty = cam.get("type");
    std::string type = "perspective";
    if (truthy(ty))   // camera.js compares type with === only: a non-string type is neither kind
        type = ty->t == JVal::Str ? ty->s : std::string("\x01non-string");
    const JVal* as = cam.get("aspect");
    const double final_aspect = truthy(as) ? num(as) : aspect;
    return make_camera(position, look_at, up, fov, final_aspect, aperture, focus, type);
}

Camera setup_camera(const Camera& c, int32_t w, int32_t h) {   // ray-tracer.js:439-474
    const V look_at = vsub(c.origin, vmul(c.w, c.focus_dist));
    return make_camera(c.origin, look_at, c.v, js_or_num(c.fov, 45), (double)w / (double)h,
                       js_or_num(c.aperture, 0.0), js_or_num(c.focus_dist, 10.0),
                       c.perspective ? "perspective" : (c.orthographic ? "orthographic" : "other"));
}

void keyed_permutation(uint32_t seed, int32_t* perm) {     // noise.js:6-18 from the keyed perm stream
    const uint32_t pkey = rt::pixel_key(rt::host_seed_mix(seed), 0xFFFFFFFFu);
    rt::Rng<double> g{rt::sample_key(pkey, 0xFFFFFFFFu), 0};
    int p[256];
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int i = 255; i >= 0; --i) {
        const int j = (int)std::floor(g.next() * (i + 1));
        std::swap(p[i], p[j]);
    }
    for (int i = 0; i < 512; ++i) perm[i] = p[i & 255];
}

}  // namespace

extern "C" {

int rt_json_scene_load(const char* json, size_t len, int32_t width, int32_t height, uint32_t seed,
                       rt_json_scene** out) {
    if (!json || !out) return rt::set_error(RT_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (width <= 0 || height <= 0) return rt::set_error(RT_ERR_INVALID, "width/height must be positive");
    Parser ps{json, json + len, {}};
    JVal root;
    if (!ps.value(root)) return rt::set_error(RT_ERR_INVALID, ps.err.c_str());
    ps.ws();
    if (ps.p != ps.end) return rt::set_error(RT_ERR_INVALID, "JSON: trailing characters");
    if (root.t != JVal::Obj) return rt::set_error(RT_ERR_INVALID, "scene JSON is not an object");
    std::unique_ptr<rt_json_scene> s(new rt_json_scene());
    try {
        s->width = width;
        s->height = height;
        const JVal* cam = root.get("camera");
        bool resized = false;
        if (truthy(cam) && truthy(cam->get("resolution"))) {   // scene-loader.js:24-33
            const JVal* res = cam->get("resolution");
            const double w = res->t == JVal::Arr && res->a.size() > 0 ? num(&res->a[0]) : NAN;
            const double h = res->t == JVal::Arr && res->a.size() > 1 ? num(&res->a[1]) : NAN;
            if (!(w >= 1 && h >= 1 && w < 65536 && h < 65536)) throw LoadError{"camera.resolution is not a valid size"};
            s->width = (int32_t)w;
            s->height = (int32_t)h;
            resized = true;
        }
        rt_scene_desc& d = s->desc;
        d.abi_version = RT_ABI_VERSION;
        d.background = RT_BG_GRADIENT;                       // world.js:12
        d.sky_intensity = 1.0;
        d.solid_color[0] = d.solid_color[1] = d.solid_color[2] = 0.1;
        const JVal* bg = root.get("background");
        if (truthy(bg)) {                                    // scene-loader.js:37-56
            const JVal* t = bg->get("type");
            const std::string ty = t && t->t == JVal::Str ? t->s : std::string();
            if (ty == "solid" || ty == "hdri") d.background = RT_BG_NAN;   // bound factories -> NaN radiance
            else if (ty == "procedural_sky") d.background = RT_BG_PROCEDURAL_SKY;
            else d.background = RT_BG_GRADIENT;
            const JVal* in = bg->get("intensity");
            if (in) d.sky_intensity = num(in);
        }
        const JVal* objs = root.get("objects");
        if (truthy(objs) && objs->t == JVal::Arr)
            for (const JVal& o : objs->a) {
                if (o.t == JVal::Null) throw LoadError{"object is null"};   // objData.type on null throws
                create_object(*s, o);
            }
        // lights (scene-loader.js:69-76) are parsed but never rendered; _createLight calls
        // lightData.type.toLowerCase() (:187), which throws for a truthy non-string type: the load fails
        const JVal* lights = root.get("lights");
        if (truthy(lights) && lights->t == JVal::Arr)
            for (const JVal& l : lights->a) {
                const JVal* lt = l.t == JVal::Obj ? l.get("type") : nullptr;
                if (truthy(lt) && lt->t != JVal::Str) throw LoadError{"light.type is not a string"};
            }
        Camera c;
        if (truthy(cam)) {
            // aspect from the loader's width/height, which a resolution entry already replaced
            c = create_camera(*cam, (double)s->width / (double)s->height);
        } else {                                             // RayTracer constructor camera
            c = make_camera({3, 2, 2}, {0, 0, -1}, {0, 1, 0}, 45, (double)width / (double)height, 0.0, 10.0,
                            "perspective");
        }
        if (resized) c = setup_camera(c, s->width, s->height);   // resizeCanvas -> setupCamera
        rt_camera_desc& cd = d.camera;
        const V* src[7] = {&c.origin, &c.llc, &c.horizontal, &c.vertical, &c.u, &c.v, &c.w};
        double* dst[7] = {cd.origin, cd.lower_left, cd.horizontal, cd.vertical, cd.u, cd.v, cd.w};
        for (int k = 0; k < 7; ++k) { dst[k][0] = src[k]->x; dst[k][1] = src[k]->y; dst[k][2] = src[k]->z; }
        cd.lens_radius = c.lens_radius;
        cd.type = c.orthographic ? RT_CAM_ORTHOGRAPHIC : RT_CAM_PERSPECTIVE;
        keyed_permutation(seed, d.perm);
        d.num_objects = (int32_t)s->objects.size();
        d.objects = s->objects.data();
        d.num_materials = (int32_t)s->materials.size();
        d.materials = s->materials.data();
        d.num_triangles = (int32_t)(s->triangles.size() / 12);
        d.triangles = s->triangles.data();
    } catch (const LoadError& e) {
        return rt::set_error(RT_ERR_INVALID, e.msg.c_str());
    } catch (const std::bad_alloc&) {
        return rt::set_error(RT_ERR_NOMEM, "out of host memory");
    }
    *out = s.release();
    return RT_OK;
}

const rt_scene_desc* rt_json_scene_desc(const rt_json_scene* scene) { return scene ? &scene->desc : nullptr; }

void rt_json_scene_size(const rt_json_scene* scene, int32_t* width, int32_t* height) {
    if (!scene) return;
    if (width) *width = scene->width;
    if (height) *height = scene->height;
}

void rt_json_scene_destroy(rt_json_scene* scene) { delete scene; }

}  // extern "C"
