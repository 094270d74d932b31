// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as product).
//
// Drives the *reference's own* hot path, compiled from the unmodified headers under
// /root/reference (include/render.hpp, lib/obj_norms.hpp, lib/bvh/*.hpp), so that
// fixtures and the CPU baseline come from the reference itself.  static.cpp does not
// compile upstream (static.cpp:130 passes nullptr for tri_norms, render.hpp:88), and
// the README's ./render CLI (README.md:11) does not exist, so this harness reproduces
// static.cpp's sequence (static.cpp:76-147) with the obj_norms loader and CLI-set
// camera / rotation / size.
//
// Build: oracle/Makefile (outputs only into oracle/_ref/).  Never copies reference source.
//
// Modes (combinable):
//   default        render() once per rep (render.hpp:87), time it, print JSON summary
//   --out f.ppm    write the P6 PPM exactly like static.cpp:135-147
//   --float f.bin  dump the float RGB framebuffer (3*W*H f32, render.hpp layout)
//   --records f    per-pixel {i,j,prim,t,u,v,shadow,r,g,b} for every pixel, replicated
//                  from render.hpp:105-150 with the reference traverser directly
//   --stats        node-pair visits / triangle tests per ray type via the Statistics
//                  overload (single_ray_traverser.hpp:132-135,161-163)
//   --orbit ax ay az step count   apply anim.cpp:76-88's camera/sun Transform (transform.hpp)
//                  `count` times before rendering (eye, dir, sun rotate; up does not)
//   --orbit-views s1,s2,...   one render per listed step (degrees, applied once to the base
//                  camera + sun about --orbit's axis): bench.py's timed orbit frames; with --out f
//                  the PPMs are f.<k>.ppm and every view prints its own JSON line
//   --dump p       write p.tri48 (rotated Triangle[]), p.norm36, p.nodes32, p.prim64
//   --primary-only render.hpp:123-125 (commented-out normal visualisation) as the
//                  primary-rays-only mode: pixel = |normalize(tri.n)|
//
// Built twice more with -DREF_SCALAR=double (_ref/ref_render_f64{,_exact}): the whole
// sequence as render<double> (anim.cpp's -d mode, anim.cpp:146-155) -- load_from_file<double>,
// rotate_triangles<double>, BinnedSahBuilder<Bvh<double>,16>, render<double>.  Command-line
// numbers are then parsed with strtod (double literals, as anim.cpp writes its camera).
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cstdint>
#include <string>
#include <vector>
#include <chrono>
#include <fstream>
#include <sstream>
#include <algorithm>

#include <bvh/bvh.hpp>
#include <bvh/binned_sah_builder.hpp>
#include <bvh/single_ray_traverser.hpp>
#include <bvh/primitive_intersectors.hpp>
#include <bvh/triangle.hpp>

#include "render.hpp"
#include "obj_norms.hpp"
#include "transform.hpp"

#ifndef REF_SCALAR
#define REF_SCALAR float
#endif
using Scalar   = REF_SCALAR;
using Vector3  = bvh::Vector3<Scalar>;
using Triangle = bvh::Triangle<Scalar>;
using Bvh      = bvh::Bvh<Scalar>;

[[maybe_unused]] static void hexf(char* buf, float f) {
    uint32_t u; std::memcpy(&u, &f, 4); std::sprintf(buf, "\"0x%08x\"", u);
}
[[maybe_unused]] static void hexf(char* buf, double f) {
    uint64_t u; std::memcpy(&u, &f, 8); std::sprintf(buf, "\"0x%016llx\"", (unsigned long long)u);
}
static Scalar num(const char* s) { return sizeof(Scalar) == 8 ? Scalar(std::strtod(s, nullptr)) : Scalar(std::strtof(s, nullptr)); }

struct Args {
    std::string obj;
    Vector3 eye{0.f, -15.f, 2.f}, dir{0.f, 1.f, 0.f}, up{0.f, 0.f, 1.f}, sun{-50.f, -20.f, 0.f};
    Scalar fov = 60.f;
    int rot_axis = -1; Scalar rot_deg = 0.f;
    size_t W = 1920, H = 1080;
    std::string out, fout, records, dump;
    int reps = 1;
    bool stats = false, primary_only = false, robust = false;
    int proc = 0;  // >0: procedural heightfield with proc x proc vertices instead of an OBJ
    Vector3 orbit_axis{0.f, 1.f, 0.f};
    Scalar orbit_step = 0.f; int orbit_count = 0;   // --orbit: anim.cpp camera/sun rotations
    std::vector<std::string> orbit_views;             // --orbit-views: one render per listed step_deg
};

static Vector3 v3(char** a) { return Vector3(num(a[0]), num(a[1]), num(a[2])); }

static bool parse(int argc, char** argv, Args& a) {
    for (int i = 1; i < argc; ++i) {
        std::string s = argv[i];
        auto need = [&](int n) { if (i + n >= argc) { std::fprintf(stderr, "missing value for %s\n", s.c_str()); std::exit(2); } };
        if (s == "--eye")      { need(3); a.eye = v3(argv + i + 1); i += 3; }
        else if (s == "--dir") { need(3); a.dir = v3(argv + i + 1); i += 3; }
        else if (s == "--up")  { need(3); a.up  = v3(argv + i + 1); i += 3; }
        else if (s == "--sun") { need(3); a.sun = v3(argv + i + 1); i += 3; }
        else if (s == "--fov") { need(1); a.fov = num(argv[++i]); }
        else if (s == "--rotate") { need(2); char c = argv[i + 1][0]; a.rot_axis = c == 'x' ? 0 : c == 'y' ? 1 : 2; a.rot_deg = num(argv[i + 2]); i += 2; }
        else if (s == "--size") { need(2); a.W = std::strtoul(argv[i + 1], nullptr, 10); a.H = std::strtoul(argv[i + 2], nullptr, 10); i += 2; }
        else if (s == "--out") { need(1); a.out = argv[++i]; }
        else if (s == "--float") { need(1); a.fout = argv[++i]; }
        else if (s == "--records") { need(1); a.records = argv[++i]; }
        else if (s == "--dump") { need(1); a.dump = argv[++i]; }
        else if (s == "--reps") { need(1); a.reps = std::atoi(argv[++i]); }
        else if (s == "--stats") a.stats = true;
        else if (s == "--robust") a.robust = true;
        else if (s == "--primary-only") a.primary_only = true;
        else if (s == "--proc") { need(1); a.proc = std::atoi(argv[++i]); }
        else if (s == "--orbit-views") { need(1); std::stringstream ss(argv[++i]); std::string t;
                                          while (std::getline(ss, t, ',')) if (!t.empty()) a.orbit_views.push_back(t); }
        else if (s == "--orbit") { need(5); a.orbit_axis = v3(argv + i + 1); a.orbit_step = num(argv[i + 4]); a.orbit_count = std::atoi(argv[i + 5]); i += 5; }
        else if (s[0] == '-') { std::fprintf(stderr, "unknown flag %s\n", s.c_str()); return false; }
        else a.obj = s;
    }
    return !a.obj.empty() || a.proc > 0;
}

// Procedural heightfield (SURVEY.md §8(d) C5 definition), emitted as OBJ text into a
// stream so it goes through the reference loader (obj_norms.hpp:57-118) unchanged.
// Vertex coordinates are printed with %.9g so they round-trip exactly through strtof.
// The mesh is an INPUT, defined by SURVEY.md's formula, not by the reference's flags: z is
// computed without FMA contraction in both builds (the reference-flag build would otherwise
// fuse 400x + 300y and the final sum, giving _ref/ref_render a different mesh).
__attribute__((optimize("fp-contract=off")))
static std::string proc_obj(int n) {
    std::string s;
    s.reserve(size_t(n) * n * 40 + size_t(n) * n * 2 * 30);
    char buf[128];
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double x = double(i) / double(n - 1), y = double(j) / double(n - 1);
            double z = 0.05 * (std::sin(40.0 * x) + std::cos(37.0 * y)) + 0.01 * std::sin(400.0 * x + 300.0 * y);
            std::snprintf(buf, sizeof buf, "v %.9g %.9g %.9g\n", (float)x, (float)y, (float)z);
            s += buf;
        }
    for (int j = 0; j + 1 < n; ++j)
        for (int i = 0; i + 1 < n; ++i) {
            long a = long(j) * n + i + 1, b = a + 1, c = a + n + 1, d = a + n;
            std::snprintf(buf, sizeof buf, "f %ld %ld %ld\nf %ld %ld %ld\n", a, b, c, a, c, d);
            s += buf;
        }
    return s;
}

struct PixelRecord {          // little-endian, every pixel: 40 B (float); double: natural alignment, 72 B
    uint32_t i, j;
    int32_t  prim;            // -1 on primary miss
    Scalar   t, u, v;
    int32_t  shadow;          // 1 if the shadow ray hit something, 0 if lit, -1 if no shadow ray
    Scalar   r, g, b;
};

int main(int argc, char** argv) {
    Args a;
    if (!parse(argc, argv, a)) {
        std::fprintf(stderr, "usage: ref_render <obj>|--proc N [--eye x y z] [--dir x y z] [--up x y z] [--fov f] [--sun x y z] "
                             "[--rotate x|y|z deg] [--orbit ax ay az step_deg count] [--size W H] [--out f.ppm] [--float f] [--records f] [--dump p] [--reps n] [--stats] [--primary-only]\n");
        return 2;
    }
    std::vector<Triangle> triangles;
    std::vector<std::array<Vector3, 3>> tri_norms;
    auto t_load0 = std::chrono::high_resolution_clock::now();
    if (a.proc > 0) {
        std::istringstream is(proc_obj(a.proc));
        auto p = obj::load_from_stream<Scalar>(is);
        triangles = std::move(p.first); tri_norms = std::move(p.second);
    } else {
        auto p = obj::load_from_file<Scalar>(a.obj);          // obj_norms.hpp:120
        triangles = std::move(p.first); tri_norms = std::move(p.second);
    }
    auto t_load1 = std::chrono::high_resolution_clock::now();
    if (triangles.empty()) { std::fprintf(stderr, "The given scene is empty or cannot be loaded\n"); return 1; }

    if (a.rot_axis == 0) rotate_triangles<0>(a.rot_deg, triangles.data(), triangles.size());   // render.hpp:25
    else if (a.rot_axis == 1) rotate_triangles<1>(a.rot_deg, triangles.data(), triangles.size());
    else if (a.rot_axis == 2) rotate_triangles<2>(a.rot_deg, triangles.data(), triangles.size());

    // BVH build exactly as static.cpp:100-107
    Bvh bvh;
    auto t_b0 = std::chrono::high_resolution_clock::now();
    auto bb = bvh::compute_bounding_boxes_and_centers(triangles.data(), triangles.size());
    auto global_bbox = bvh::compute_bounding_boxes_union(bb.first.get(), triangles.size());
    bvh::BinnedSahBuilder<Bvh, 16> builder(bvh);
    builder.build(global_bbox, bb.first.get(), bb.second.get(), triangles.size());
    auto t_b1 = std::chrono::high_resolution_clock::now();

    if (!a.dump.empty()) {
        auto wr = [&](const std::string& suf, const void* p, size_t n) {
            std::ofstream f(a.dump + suf, std::ios::binary); f.write((const char*)p, n); };
        const std::string w = sizeof(Scalar) == 8 ? "64" : "";      // .tri48 .norm36 .nodes32 | .tri96 .norm72 .nodes64
        wr(w.empty() ? ".tri48" : ".tri96", triangles.data(), triangles.size() * sizeof(Triangle));
        wr(w.empty() ? ".norm36" : ".norm72", tri_norms.data(), tri_norms.size() * sizeof(std::array<Vector3, 3>));
        wr(w.empty() ? ".nodes32" : ".nodes64", bvh.nodes.get(), bvh.node_count * sizeof(Bvh::Node));
        std::vector<uint64_t> pi(bvh.primitive_indices.get(), bvh.primitive_indices.get() + triangles.size());
        wr(".prim64", pi.data(), pi.size() * 8);
    }

    // --orbit-views s1,s2,...: one render per view, the base camera + sun rotated ONCE by s_k degrees
    // about the orbit axis (bench.py's step_views frames); PPMs go to <out>.<k>.ppm, one JSON line each.
    const Vector3 base_sun = a.sun;
    const std::string base_out = a.out;
    const size_t n_views = a.orbit_views.empty() ? 1 : a.orbit_views.size();
    for (size_t view_k = 0; view_k < n_views; ++view_k) {
    a.sun = base_sun;
    if (!a.orbit_views.empty()) {
        a.orbit_step = num(a.orbit_views[view_k].c_str()); a.orbit_count = 1;
        if (!base_out.empty()) a.out = base_out + "." + std::to_string(view_k) + ".ppm";
    }
    Camera<Scalar> camera{a.eye, a.dir, a.up, a.fov};
    if (a.orbit_count > 0) {
        // anim.cpp:76-88: the reference's own Transform applied orbit_count times
        constexpr Scalar pi = Scalar(3.14159265359);
        auto t_cam = Transform<Scalar>().rotate(a.orbit_axis, a.orbit_step / 180.0f * pi);
        auto t_sun = Transform<Scalar>().rotate(a.orbit_axis, a.orbit_step / 180.0f * pi);
        for (int k = 0; k < a.orbit_count; ++k) {
            camera.eye = t_cam(camera.eye);
            camera.dir = t_cam(camera.dir);
            a.sun = t_sun(a.sun);
        }
    }
    const size_t W = a.W, H = a.H;
    std::vector<Scalar> pixels(3 * W * H);

    // Camera basis, restated from render.hpp:91-97 purely to PRINT it (pinned as hex in fixtures).
    auto dir = bvh::normalize(camera.dir);
    auto image_u = bvh::normalize(bvh::cross(dir, camera.up));
    auto image_v = bvh::normalize(bvh::cross(image_u, dir));
    auto image_w = std::tan(camera.fov * Scalar(3.14159265 * (1.0 / 180.0) * 0.5));
    auto ratio = Scalar(H) / Scalar(W);
    image_u = image_u * image_w;
    image_v = image_v * image_w * ratio;

    std::pair<int, int> rh{0, 0};
    std::vector<double> times;
    if (!a.primary_only && !a.robust) {
        for (int r = 0; r < std::max(1, a.reps); ++r) {
            auto t0 = std::chrono::high_resolution_clock::now();
            rh = render(camera, a.sun, bvh, triangles.data(), tri_norms.data(), pixels.data(), W, H);   // render.hpp:87
            auto t1 = std::chrono::high_resolution_clock::now();
            times.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        }
    }

    // Replicated per-pixel loop (render.hpp:105-150) with the reference traverser, used for
    // records / stats / primary-only mode; cross-checked against render()'s framebuffer.
    bvh::ClosestPrimitiveIntersector<Bvh, Triangle, false> intersector(bvh, triangles.data());
    // --robust: the same loop with the library's RobustNodeIntersector (node_intersectors.hpp:
    // 54-79, T. Ize) in place of render()'s default FastNodeIntersector -- the loop is pinned
    // to render() itself by loop_vs_render_mismatch == 0 in the default mode.
    bvh::SingleRayTraverser<Bvh> fast_traverser(bvh);
    bvh::SingleRayTraverser<Bvh, 64, bvh::RobustNodeIntersector<Bvh>> robust_traverser(bvh);
    const bool need_loop = a.stats || !a.records.empty() || a.primary_only || a.robust;
    size_t prim_pairs = 0, prim_tests = 0, sh_pairs = 0, sh_tests = 0, n_sh = 0, loop_hits = 0, loop_rays = 0;
    size_t mismatch = 0;
    std::vector<PixelRecord> recs;
    auto replicated_loop = [&](auto& traverser) {
        using Stats = typename std::decay_t<decltype(traverser)>::Statistics;
        if (!a.records.empty()) recs.resize(W * H);
        std::vector<Scalar> px2(3 * W * H);
        #pragma omp parallel for collapse(2) reduction(+: prim_pairs, prim_tests, sh_pairs, sh_tests, n_sh, loop_hits, loop_rays)
        for (size_t i = 0; i < W; ++i) {
            for (size_t j = 0; j < H; ++j) {
                size_t index = 3 * (W * j + i);
                PixelRecord rec{uint32_t(i), uint32_t(j), -1, 0.f, 0.f, 0.f, -1, 0.f, 0.f, 0.f};
                auto u = 2 * (i + Scalar(0.5)) / Scalar(W) - Scalar(1);
                auto v = 2 * (j + Scalar(0.5)) / Scalar(H) - Scalar(1);
                auto view = bvh::normalize(image_u * u + image_v * v + dir);
                bvh::Ray<Scalar> ray(camera.eye, view);
                Stats st;
                auto hit = traverser.traverse(ray, intersector, st);
                prim_pairs += st.traversal_steps; prim_tests += st.intersections;
                loop_rays++;
                Scalar c0 = 0, c1 = 0, c2 = 0;
                if (hit) {
                    loop_hits++;
                    auto ind = hit->primitive_index;
                    auto tri = triangles[ind];
                    auto normal = bvh::normalize(tri.n);
                    auto hu = hit->intersection.u, hv = hit->intersection.v;
                    rec.prim = int32_t(ind); rec.t = hit->intersection.t; rec.u = hu; rec.v = hv;
                    if (a.primary_only) {
                        c0 = std::fabs(normal[0]); c1 = std::fabs(normal[1]); c2 = std::fabs(normal[2]);
                    } else {
                        Vector3 p = (hu * tri.p0 + hv * tri.p1() + (1 - hu - hv) * tri.p2());
                        Scalar scale = -0.00001;
                        p = p + scale * normal;
                        Vector3 sun_line = bvh::normalize(a.sun - p);
                        bvh::Ray<Scalar> sray(p, sun_line);
                        Stats st2;
                        auto shit = traverser.traverse(sray, intersector, st2);
                        sh_pairs += st2.traversal_steps; sh_tests += st2.intersections; n_sh++;
                        loop_rays++;
                        if (!shit) {
                            auto c = smooth_shading(sun_line, tri_norms[ind], view, hu, hv);
                            c0 = c[0]; c1 = c[1]; c2 = c[2];
                            rec.shadow = 0;
                        } else {
                            loop_hits++;
                            rec.shadow = 1;
                        }
                    }
                }
                px2[index] = c0; px2[index + 1] = c1; px2[index + 2] = c2;
                rec.r = c0; rec.g = c1; rec.b = c2;
                if (!recs.empty()) recs[W * j + i] = rec;
            }
        }
        if (a.primary_only || a.robust) { pixels = px2; rh = {int(loop_rays), int(loop_hits)}; }
        else mismatch = size_t(std::count_if(pixels.begin(), pixels.end(), [&, k = size_t(0)](Scalar x) mutable {
            uint64_t p = 0, q = 0; Scalar y = px2[k++]; std::memcpy(&p, &x, sizeof x); std::memcpy(&q, &y, sizeof y); return p != q; }));
    };
    if (need_loop) {
        if (a.robust) replicated_loop(robust_traverser);
        else replicated_loop(fast_traverser);
    }

    if (!a.records.empty()) {
        std::ofstream f(a.records, std::ios::binary);
        f.write((const char*)recs.data(), recs.size() * sizeof(PixelRecord));
    }
    if (!a.fout.empty()) {
        std::ofstream f(a.fout, std::ios::binary);
        f.write((const char*)pixels.data(), pixels.size() * sizeof(Scalar));
    }
    if (!a.out.empty()) {   // static.cpp:135-147
        std::ofstream out(a.out, std::ofstream::binary);
        out << "P6 " << W << " " << H << " " << 255 << "\n";
        for (size_t j = H; j > 0; --j) {
            for (size_t i = 0; i < W; ++i) {
                size_t index = 3 * (W * (j - 1) + i);
                uint8_t pixel[3] = {
                    static_cast<uint8_t>(std::max(std::min(pixels[index    ] * 255, Scalar(255)), Scalar(0))),
                    static_cast<uint8_t>(std::max(std::min(pixels[index + 1] * 255, Scalar(255)), Scalar(0))),
                    static_cast<uint8_t>(std::max(std::min(pixels[index + 2] * 255, Scalar(255)), Scalar(0)))
                };
                out.write(reinterpret_cast<char*>(pixel), 3);
            }
        }
    }

    std::sort(times.begin(), times.end());
    double med = times.empty() ? 0.0 : times[times.size() / 2];
    double best = times.empty() ? 0.0 : times[0];
    char h[15][24];
    hexf(h[9], camera.eye[0]); hexf(h[10], camera.eye[1]); hexf(h[11], camera.eye[2]);
    hexf(h[12], a.sun[0]); hexf(h[13], a.sun[1]); hexf(h[14], a.sun[2]);
    hexf(h[0], dir[0]); hexf(h[1], dir[1]); hexf(h[2], dir[2]);
    hexf(h[3], image_u[0]); hexf(h[4], image_u[1]); hexf(h[5], image_u[2]);
    hexf(h[6], image_v[0]); hexf(h[7], image_v[1]); hexf(h[8], image_v[2]);
    int threads = 1;
#ifdef _OPENMP
    threads = omp_get_max_threads();
#endif
    std::printf("{\"n_tri\": %zu, \"n_nodes\": %zu, \"W\": %zu, \"H\": %zu, \"rays\": %d, \"hits\": %d, "
                "\"render_ms_median\": %.4f, \"render_ms_best\": %.4f, \"reps\": %zu, \"threads\": %d, "
                "\"load_ms\": %.3f, \"build_ms\": %.3f, "
                "\"basis_dir\": [%s, %s, %s], \"basis_u\": [%s, %s, %s], \"basis_v\": [%s, %s, %s], "
                "\"eye\": [%s, %s, %s], \"sun\": [%s, %s, %s]",
                triangles.size(), bvh.node_count, W, H, rh.first, rh.second, med, best, times.size(), threads,
                std::chrono::duration<double, std::milli>(t_load1 - t_load0).count(),
                std::chrono::duration<double, std::milli>(t_b1 - t_b0).count(),
                h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12], h[13], h[14]);
    if (need_loop)
        std::printf(", \"loop_rays\": %zu, \"loop_hits\": %zu, \"loop_vs_render_mismatch\": %zu, "
                    "\"primary_pairs\": %zu, \"primary_tests\": %zu, \"shadow_rays\": %zu, \"shadow_pairs\": %zu, \"shadow_tests\": %zu",
                    loop_rays, loop_hits, mismatch, prim_pairs, prim_tests, n_sh, sh_pairs, sh_tests);
    std::printf("}\n");
    std::fflush(stdout);
    }   // views
    return 0;
}
