// tri_exit_check.cpp — TEST INFRASTRUCTURE: checks tri_exit_bound (pt_core.h leaves_tri_hull, scene_pack.h
// build_tri_exit) on the CPU.  Rays are made to hit a triangle A as the kernel makes them (the binary64 test's
// t, point = o + d t), leave it at grazing to steep angles, and whenever the check lets the next segment
// skip the triangle walk, the binary64 test (triangle_candidate) of EVERY triangle must reject the ray.
// usage: tri_exit_check <mesh> <rays> <seed> [mutation]
//   mesh: sphere (config 5's 176 x 142 UV sphere, radius 1.2), sphere_off (the same, off the origin),
//         cube, torus (not convex), bowl (an open half sphere), grid (coplanar triangles), pair (a sphere and
//         a cube beside it in one scene)
//   mutation: 0 none; 1 C from A's own vertices only; 2 the sides' bounds swapped
// prints: rays=.. skips=.. violations=.. hits_not_skipped=.. exit_faces=..
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../blenderraytracer_amd/csrc/pt_path.h"
#include "../../blenderraytracer_amd/csrc/scene_pack.h"

using namespace rt;

static void add_tri(std::vector<double>& T, const double* a, const double* b, const double* c) {
    const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    const double l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);   // geometry.js:143-145 (0/0: NaN)
    for (int k = 0; k < 3; ++k) n[k] /= l;
    T.insert(T.end(), {a[0], a[1], a[2], b[0], b[1], b[2], c[0], c[1], c[2], n[0], n[1], n[2]});
}

// a (nu x nv) grid of quads over (s, t) in [0,1]^2 mapped by f, two triangles each
template <class F>
static void grid_mesh(std::vector<double>& T, int nu, int nv, F f) {
    for (int j = 0; j < nv; ++j)
        for (int i = 0; i < nu; ++i) {
            double p00[3], p10[3], p01[3], p11[3];
            f((double)i / nu, (double)j / nv, p00);
            f((double)(i + 1) / nu, (double)j / nv, p10);
            f((double)i / nu, (double)(j + 1) / nv, p01);
            f((double)(i + 1) / nu, (double)(j + 1) / nv, p11);
            add_tri(T, p00, p10, p11);
            add_tri(T, p00, p11, p01);
        }
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s mesh rays seed [mutation]\n", argv[0]); return 2; }
    const std::string mesh = argv[1];
    const long rays = atol(argv[2]);
    std::mt19937_64 rng((unsigned long long)atoll(argv[3]));
    const int mutation = argc > 4 ? atoi(argv[4]) : 0;
    std::vector<double> T;
    const double pi = 3.14159265358979323846;
    if (mesh == "sphere" || mesh == "sphere_off" || mesh == "bowl") {
        const double c[3] = {mesh == "sphere_off" ? 3.0 : 0.0, mesh == "sphere_off" ? 1.0 : 0.0, mesh == "sphere_off" ? 2.0 : 0.0};
        const bool bowl = mesh == "bowl";
        grid_mesh(T, 176, bowl ? 71 : 142, [&](double s, double t, double* p) {
            const double th = t * (bowl ? pi / 2 : pi), ph = s * 2 * pi;
            p[0] = c[0] + 1.2 * std::sin(th) * std::cos(ph);
            p[1] = c[1] + 1.2 * std::cos(th);
            p[2] = c[2] + 1.2 * std::sin(th) * std::sin(ph);
        });
    } else if (mesh == "pair") {          // the UV sphere and a cube beside it: bounds over both objects' vertices
        grid_mesh(T, 88, 71, [&](double s, double t, double* p) {
            const double th = t * pi, ph = s * 2 * pi;
            p[0] = 1.2 * std::sin(th) * std::cos(ph); p[1] = 1.2 * std::cos(th); p[2] = 1.2 * std::sin(th) * std::sin(ph);
        });
        const double v[8][3] = {{2.5, -.5, -.5}, {3.5, -.5, -.5}, {3.5, .5, -.5}, {2.5, .5, -.5}, {2.5, -.5, .5}, {3.5, -.5, .5}, {3.5, .5, .5}, {2.5, .5, .5}};
        const int f[12][3] = {{0, 2, 1}, {0, 3, 2}, {4, 5, 6}, {4, 6, 7}, {0, 1, 5}, {0, 5, 4},
                              {3, 6, 2}, {3, 7, 6}, {0, 4, 7}, {0, 7, 3}, {1, 2, 6}, {1, 6, 5}};
        for (auto& q : f) add_tri(T, v[q[0]], v[q[1]], v[q[2]]);
    } else if (mesh == "torus") {
        grid_mesh(T, 96, 48, [&](double s, double t, double* p) {
            const double a = s * 2 * pi, b = t * 2 * pi, r = 1.0 + 0.4 * std::cos(b);
            p[0] = r * std::cos(a); p[1] = 0.4 * std::sin(b); p[2] = r * std::sin(a);
        });
    } else if (mesh == "grid") {
        grid_mesh(T, 64, 64, [&](double s, double t, double* p) { p[0] = 4 * s - 2; p[1] = -1; p[2] = 4 * t - 2; });
    } else if (mesh == "cube") {
        const double v[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1}, {-1, -1, 1}, {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}};
        const int f[12][3] = {{0, 2, 1}, {0, 3, 2}, {4, 5, 6}, {4, 6, 7}, {0, 1, 5}, {0, 5, 4},
                              {3, 6, 2}, {3, 7, 6}, {0, 4, 7}, {0, 7, 3}, {1, 2, 6}, {1, 6, 5}};
        for (auto& q : f) add_tri(T, v[q[0]], v[q[1]], v[q[2]]);
    } else {
        fprintf(stderr, "unknown mesh %s\n", mesh.c_str());
        return 2;
    }
    const int nt = (int)(T.size() / 12);
    rt_material_desc mat{};
    mat.type = RT_MAT_METAL;
    rt_object_desc obj{};
    obj.type = RT_OBJ_MESH;
    obj.first = 0;
    obj.count = nt;
    rt_scene_desc d{};
    d.abi_version = RT_ABI_VERSION;
    d.num_objects = 1;
    d.objects = &obj;
    d.num_materials = 1;
    d.materials = &mat;
    d.num_triangles = nt;
    d.triangles = T.data();
    HostScene hs;
    std::string err;
    if (!pack_host(d, hs, err)) { fprintf(stderr, "%s\n", err.c_str()); return 2; }
    build_bvhs(hs);
    HostRecords<double> rec;
    make_records(hs, d, rec);
    long exit_faces = 0;
    for (int i = 0; i < nt; ++i) exit_faces += std::isfinite(hs.tri_exit[2 * i]) + std::isfinite(hs.tri_exit[2 * i + 1]);
    if (mutation == 1) {                  // only A's own vertices: blind to the rest of the mesh
        for (int i = 0; i < nt; ++i)
            for (int s = 0; s < 2; ++s) {
                const double* t = &hs.tris[12 * (size_t)i];
                const double N[3] = {s ? -t[9] : t[9], s ? -t[10] : t[10], s ? -t[11] : t[11]};
                const double p0 = N[0] * t[0] + N[1] * t[1] + N[2] * t[2];
                hs.tri_exit[2 * i + s] = std::max(p0, std::max(p0 + N[0] * t[3] + N[1] * t[4] + N[2] * t[5],
                                                               p0 + N[0] * t[6] + N[1] * t[7] + N[2] * t[8])) + 1e-12;
            }
    } else if (mutation == 2) {
        for (int i = 0; i < nt; ++i) std::swap(hs.tri_exit[2 * i], hs.tri_exit[2 * i + 1]);
    }
    SceneView<double> v{};
    v.tris = rec.tris.data();
    v.tri_exit = hs.tri_exit.data();
    fill_view_constants(v, hs, d);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto unit = [&](double* r) {
        double l;
        do {
            for (int k = 0; k < 3; ++k) r[k] = 2 * U(rng) - 1;
            l = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        } while (l > 1 || l < 1e-6);
        l = std::sqrt(l);
        for (int k = 0; k < 3; ++k) r[k] /= l;
    };
    long made = 0, skips = 0, viol = 0, hits_ns = 0;
    for (long attempt = 0; made < rays && attempt < 20 * rays; ++attempt) {
        const int a = (int)(U(rng) * nt) % nt;
        const TriRec<double>& A = rec.tris[a];
        if (!std::isfinite(A.nx)) continue;
        // a point on A: interior, on an edge or at a vertex
        double u = U(rng), w = U(rng);
        if (u + w > 1) { u = 1 - u; w = 1 - w; }
        const int kind = (int)(U(rng) * 4);
        if (kind == 1) w = 0;
        else if (kind == 2) { u = 0; w = 0; }
        else if (kind == 3) w = 1 - u;
        const double P[3] = {A.v0x + u * A.e1x + w * A.e2x, A.v0y + u * A.e1y + w * A.e2y, A.v0z + u * A.e1z + w * A.e2z};
        // an incoming ray from a random side, hitting A through the binary64 test
        const double side = U(rng) < 0.5 ? 1.0 : -1.0;   // the side it comes from: N = side n
        const double N[3] = {side * A.nx, side * A.ny, side * A.nz};
        double din[3];
        unit(din);
        const double dn = din[0] * N[0] + din[1] * N[1] + din[2] * N[2];
        if (dn > 0) for (int k = 0; k < 3; ++k) din[k] = -din[k];
        const double L = 0.5 + 3 * U(rng);
        const V3<double> o{P[0] - L * din[0], P[1] - L * din[1], P[2] - L * din[2]}, di{din[0], din[1], din[2]};
        double t;
        if (!triangle_candidate(A, o, di, 0.001, t)) continue;
        const V3<double> p = o + di * t;      // hit_record's point (math.js:41)
        // the exit: angle g = N.d from 1 down to 1e-14 (log-uniform), or a metal-like reflection
        double tg[3];
        unit(tg);
        const double tn = tg[0] * N[0] + tg[1] * N[1] + tg[2] * N[2];
        for (int k = 0; k < 3; ++k) tg[k] -= tn * N[k];
        const double tl = std::sqrt(tg[0] * tg[0] + tg[1] * tg[1] + tg[2] * tg[2]);
        if (!(tl > 1e-3)) continue;
        const double g = std::pow(10.0, -14.0 * U(rng)) * (U(rng) < 0.1 ? -1.0 : 1.0);
        const double s = std::sqrt(std::max(0.0, 1 - g * g)), m = 0.2 + 1.8 * U(rng);
        const V3<double> dout{m * (g * N[0] + s * tg[0] / tl), m * (g * N[1] + s * tg[1] / tl), m * (g * N[2] + s * tg[2] / tl)};
        ++made;
        const bool skip = leaves_tri_hull(v, a, p, dout);
        bool hit = false;
        for (int k = 0; k < nt && !hit; ++k) {
            double tk;
            hit = triangle_candidate(rec.tris[k], p, dout, 0.001, tk);
        }
        skips += skip;
        viol += skip && hit;
        hits_ns += !skip && hit;
    }
    printf("rays=%ld skips=%ld violations=%ld hits_not_skipped=%ld exit_faces=%ld triangles=%d\n", made, skips, viol,
           hits_ns, exit_faces, nt);
    return 0;
}
