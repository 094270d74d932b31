// render_cli.cpp -- the `./render <obj> --eye ... --rotate ...` CLI of README.md:11.
//
// The reference documents this CLI but never built it (include/CMakeLists.txt:1 comments the
// target out; static.cpp:21-24 ignores argv).  This is its MI355X implementation: the
// static.cpp sequence (load :76, rotate :83-88, BVH :100-107, render :130, PPM :135-147) with
// the hot path on the GPU through libceres_hip.so.  Defaults follow static.cpp:39-47,72-73.
//
//   render <obj> [--eye x y z] [--dir x y z] [--up x y z] [--fov deg] [--sun x y z]
//                [--rotate x|y|z deg] [--size W H] [-o|--out file.ppm] [--primary-only]
//                [--proc N] [--device D] [--bench reps] [--json]
//                [--orbit ax ay az step_deg count] [--frames N] [--gpu-bvh] [--double|-d]
//                [--gpus N] [--row-block R] [--robust] [--qbvh] [--exact | --fma] [--cpu [--threads T]]
//
// Arithmetic (float and double pipelines): --fma (the default) computes every step as the reference's own
// CMake build does (CMakeLists.txt:11-13, g++ -O3 -mavx2 -mfma: GCC contracts a*b+c into FMA at
// the sites listed in oracle/contraction_sites.txt) -- the scene (normals, rotation, SAH costs),
// the camera basis, the orbit and the kernels (CERES_ARITH_FMA + CERES_MODE_FMA), so the PPM is
// the one that build writes.  --exact is the contraction-free reference (-ffp-contract=off).
//
// --robust traverses with the library's RobustNodeIntersector (node_intersectors.hpp:54-79,
// T. Ize's padded-inverse slab test) instead of render()'s FastNodeIntersector.
//
// --gpus N splits every frame over N GPUs of this node in one process: rows
// are dealt in blocks of R (default 8) rows round-robin to ranks on devices D, D+1, ... (mod
// the device count, so N > devices reuses devices -- the test mode on a one-GPU box), each
// rank with its own scene copy; the RGB8 rows are gathered peer-to-peer over xGMI to the first
// device and assembled there (ceres_render_multi_f32).  The PPM is identical to --gpus 1.
//
// --double (anim.cpp's -d, anim.cpp:146-155) runs the whole sequence as render<double>:
// numbers parsed with strtod, double mesh / BVH / camera, the double GPU kernel.
// --gpu-bvh builds the same BinnedSahBuilder BVH with the gfx950 builder (bvh_build.hip).
//
// --orbit / --frames are the anim.cpp:76-125 driver without Magick++: the camera eye, dir and
// the sun are rotated by step_deg about the axis (transform.hpp:67-112) `count` times before
// the first frame, and once more per further frame; N frames are written as
// <out-stem>_000.ppm ... (one file when N = 1), "Total Rays" summed like anim.cpp:127.
//
// --cpu renders on the host cores instead (ceres_render_cpu_f32 / _f64: the product's CPU path, the
// same images, rays and hits, float or --double; one process; --threads T, default the OpenMP default) --
// SURVEY.md §7 step 3's "config 1 works with no GPU".  It is only ever chosen by the flag:
//
// Exit status: 0 on success, 1 on a load/render error (message on stderr), 2 on bad usage.
// There is no CPU fallback: without --cpu and without a gfx950 device the render step fails.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <cctype>
#include <type_traits>

#include "ceres_render.h"

namespace {

// Every number is kept as float (strtof, render<float>) and as double (strtod: the double
// literals of anim.cpp's -d mode); --double selects the double pipeline.
template <class S> struct Num {
    S eye[3] = {0, -15, 2}, dir[3] = {0, 1, 0}, up[3] = {0, 0, 1}, sun[3] = {-50, -20, 0};
    S fov = 60, rot_deg = 0, orbit_axis[3] = {0, 1, 0}, orbit_step = 0;
};

struct Opts {
    std::string obj, out = "render.ppm";
    Num<float> f;
    Num<double> d;
    int rot_axis = -1;
    size_t W = 1920, H = 1080;
    int mode = CERES_MODE_FULL, proc = 0, device = 0, bench = 0, gpus = 1, row_block = 16;
    bool json = false, gpu_bvh = false, f64 = false;
    int arith = CERES_ARITH_FMA;                   // --fma (default) / --exact
    int orbit_count = 0, frames = 1;
    bool cpu = false;                              // --cpu: ceres_render_cpu_f32 on the host cores
    int threads = 0;                               // --threads (0: the OpenMP default)
};

int usage() {
    std::fprintf(stderr,
                 "usage: render <obj> [--eye x y z] [--dir x y z] [--up x y z] [--fov deg] [--sun x y z]\n"
                 "              [--rotate x|y|z deg] [--size W H] [-o out.ppm] [--primary-only] [--proc N]\n"
                 "              [--device D] [--bench reps] [--json] [--orbit ax ay az step_deg count] [--frames N]\n"
                 "              [--gpu-bvh] [--double] [--gpus N] [--row-block R] [--robust] [--qbvh] [--exact|--fma]\n"
                 "              [--cpu [--threads T]]\n");
    return 2;
}

bool parse(int argc, char** argv, Opts& o) {
    // one number into both precisions; the whole string must convert
    auto num = [](const char* s, float* f, double* d) {
        char* e1; char* e2;
        *f = std::strtof(s, &e1);
        *d = std::strtod(s, &e2);
        return *e1 == '\0' && *e2 == '\0';
    };
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto have = [&](int n) { return i + n < argc; };
        auto vec = [&](float* v, double* w) {
            if (!have(3)) return false;
            bool ok = num(argv[i + 1], v, w) && num(argv[i + 2], v + 1, w + 1) && num(argv[i + 3], v + 2, w + 2);
            i += 3;
            return ok;
        };
        if (a == "--eye") { if (!vec(o.f.eye, o.d.eye)) return false; }
        else if (a == "--dir") { if (!vec(o.f.dir, o.d.dir)) return false; }
        else if (a == "--up") { if (!vec(o.f.up, o.d.up)) return false; }
        else if (a == "--sun") { if (!vec(o.f.sun, o.d.sun)) return false; }
        else if (a == "--fov") { if (!have(1) || !num(argv[++i], &o.f.fov, &o.d.fov)) return false; }
        else if (a == "--rotate") {
            if (!have(2)) return false;
            const char c = argv[i + 1][0];
            o.rot_axis = c == 'x' ? 0 : c == 'y' ? 1 : c == 'z' ? 2 : -2;
            if (o.rot_axis == -2 || argv[i + 1][1] != '\0' || !num(argv[i + 2], &o.f.rot_deg, &o.d.rot_deg)) return false;
            i += 2;
        } else if (a == "--size") {
            if (!have(2)) return false;
            o.W = std::strtoul(argv[i + 1], nullptr, 10); o.H = std::strtoul(argv[i + 2], nullptr, 10); i += 2;
            if (!o.W || !o.H) return false;
        } else if (a == "-o" || a == "--out") { if (!have(1)) return false; o.out = argv[++i]; }
        else if (a == "--primary-only") o.mode = (o.mode & CERES_MODE_ROBUST) | CERES_MODE_PRIMARY;
        else if (a == "--robust") o.mode |= CERES_MODE_ROBUST;             // RobustNodeIntersector traversal
        else if (a == "--qbvh") o.mode |= CERES_MODE_QBVH4;                // compressed shadow BVH4 (not exact)
        else if (a == "--exact") o.arith = CERES_ARITH_EXACT;              // the -ffp-contract=off reference
        else if (a == "--fma") o.arith = CERES_ARITH_FMA;                  // the reference's CMake build
        else if (a == "--proc") { if (!have(1)) return false; o.proc = std::atoi(argv[++i]); }
        else if (a == "--device") { if (!have(1)) return false; o.device = std::atoi(argv[++i]); }
        else if (a == "--gpus") { if (!have(1)) return false; o.gpus = std::atoi(argv[++i]); if (o.gpus < 1) return false; }
        else if (a == "--row-block") { if (!have(1)) return false; o.row_block = std::atoi(argv[++i]); if (o.row_block < 1) return false; }
        else if (a == "--bench") { if (!have(1)) return false; o.bench = std::atoi(argv[++i]); }
        else if (a == "--json") o.json = true;
        else if (a == "--cpu") o.cpu = true;
        else if (a == "--threads") { if (!have(1)) return false; o.threads = std::atoi(argv[++i]); if (o.threads < 0) return false; }
        else if (a == "--gpu-bvh") o.gpu_bvh = true;
        else if (a == "--double" || a == "-d") o.f64 = true;                   // anim.cpp:146-147
        else if (a == "--orbit") {
            if (!vec(o.f.orbit_axis, o.d.orbit_axis) || !have(2) || !num(argv[i + 1], &o.f.orbit_step, &o.d.orbit_step)) return false;
            o.orbit_count = std::atoi(argv[i + 2]); i += 2;
            if (o.orbit_count < 0) return false;
        } else if (a == "--frames") { if (!have(1)) return false; o.frames = std::atoi(argv[++i]); if (o.frames < 1) return false; }
        else if (a == "-h" || a == "--help") return false;
        else if (!a.empty() && a[0] == '-' && a.size() > 1 && !std::isdigit((unsigned char)a[1])) { std::fprintf(stderr, "unknown flag %s\n", a.c_str()); return false; }
        else if (o.obj.empty()) o.obj = a;
        else return false;
    }
    return !o.obj.empty() || o.proc > 0;
}

// The C ABI per precision (render<float> / render<double>).
template <class S> struct Api;
template <> struct Api<float> {
    using Node = uint32_t;
    static int load(const char* p, float** t, float** n, size_t* c, int ar) { return ceres_obj_load_arith(p, t, n, c, ar); }
    static int proc(int k, float** t, float** n, size_t* c, int ar) { return ceres_proc_mesh_arith(k, t, n, c, ar); }
    static int rotate(float* t, size_t c, int ax, float deg, int ar) { return ceres_rotate_triangles_arith(t, c, ax, deg, ar); }
    static int bvh(const float* t, size_t c, Node** nodes, size_t* m, uint64_t** prim, bool gpu, int dev, int ar) {
        return gpu ? ceres_bvh_build_gpu_arith(t, c, nodes, m, prim, dev, ar) : ceres_bvh_build_arith(t, c, nodes, m, prim, ar);
    }
    static ceres_scene* scene(const float* t, size_t c, const float* n, const Node* nodes, size_t m, const uint64_t* prim, int dev) {
        return ceres_scene_create(t, c, n, nodes, m, prim, dev, 0);
    }
    static int orbit(const Num<float>& v, size_t W, size_t H, uint32_t k, float* b, float* s, int ar) {
        return ceres_orbit_cameras_arith(v.eye, v.dir, v.up, v.sun, v.fov, W, H, v.orbit_axis, v.orbit_step, k, 0, b, s,
                                         nullptr, ar);
    }
    static int render(ceres_scene* sc, const float* b, const float* s, int mode, uint8_t* rgb, size_t W, size_t H, ceres_stats* st) {
        return ceres_render_f32(sc, b, s, mode, nullptr, rgb, W, H, st);
    }
    static int render_multi(ceres_scene* const* sc, uint32_t n, uint32_t rb, const float* b, const float* s, int mode,
                            uint8_t* rgb, size_t W, size_t H, ceres_stats* st) {
        return ceres_render_multi_f32(sc, n, rb, b, s, mode, nullptr, rgb, W, H, st);
    }
    static ceres_cpu_scene* cpu_scene(const float* t, size_t c, const float* n, const Node* nodes, size_t m, const uint64_t* prim) {
        return ceres_cpu_scene_create(t, c, n, nodes, m, prim);
    }
    static int render_cpu(const ceres_cpu_scene* cs, const float* b, const float* s, int mode, uint8_t* rgb, size_t W, size_t H,
                          ceres_stats* st, int threads) {
        return ceres_render_cpu_f32(cs, b, s, mode, nullptr, rgb, W, H, st, threads);
    }
};
template <> struct Api<double> {
    using Node = uint64_t;
    // render<double> in either arithmetic (--fma: anim.cpp -d as the reference's CMake build compiles it)
    static int load(const char* p, double** t, double** n, size_t* c, int ar) { return ceres_obj_load_f64_arith(p, t, n, c, ar); }
    static int proc(int k, double** t, double** n, size_t* c, int ar) { return ceres_proc_mesh_f64_arith(k, t, n, c, ar); }
    static int rotate(double* t, size_t c, int ax, double deg, int ar) { return ceres_rotate_triangles_f64_arith(t, c, ax, deg, ar); }
    static int bvh(const double* t, size_t c, Node** nodes, size_t* m, uint64_t** prim, bool gpu, int, int ar) {
        if (gpu) { std::fprintf(stderr, "error: --gpu-bvh builds single-precision BVHs only\n"); return CERES_EUNSUPPORTED; }
        return ceres_bvh_build_f64_arith(t, c, nodes, m, prim, ar);
    }
    static ceres_scene* scene(const double* t, size_t c, const double* n, const Node* nodes, size_t m, const uint64_t* prim, int dev) {
        return ceres_scene_create_f64(t, c, n, nodes, m, prim, dev, 0);
    }
    static int orbit(const Num<double>& v, size_t W, size_t H, uint32_t k, double* b, double* s, int ar) {
        return ceres_orbit_cameras_f64_arith(v.eye, v.dir, v.up, v.sun, v.fov, W, H, v.orbit_axis, v.orbit_step, k, 0, b, s,
                                             nullptr, ar);
    }
    static int render(ceres_scene* sc, const double* b, const double* s, int mode, uint8_t* rgb, size_t W, size_t H, ceres_stats* st) {
        return ceres_render_f64(sc, b, s, mode, nullptr, rgb, W, H, st);
    }
    static int render_multi(ceres_scene* const*, uint32_t, uint32_t, const double*, const double*, int, uint8_t*, size_t,
                            size_t, ceres_stats*) {
        std::fprintf(stderr, "error: --gpus > 1 renders single precision only\n");
        return CERES_EUNSUPPORTED;
    }
    static ceres_cpu_scene* cpu_scene(const double* t, size_t c, const double* n, const Node* nodes, size_t m,
                                      const uint64_t* prim) {
        return ceres_cpu_scene_create_f64(t, c, n, nodes, m, prim);
    }
    static int render_cpu(const ceres_cpu_scene* cs, const double* b, const double* s, int mode, uint8_t* rgb, size_t W,
                          size_t H, ceres_stats* st, int threads) {
        return ceres_render_cpu_f64(cs, b, s, mode, nullptr, rgb, W, H, st, threads);
    }
};

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

template <class S, class Render>
int frames_loop(const Opts& o, const Num<S>& v, Render&& render, const char* where);

template <class S>
int run(const Opts& o, const Num<S>& v) {
    using A = Api<S>;
    S* tri = nullptr; S* norm = nullptr; size_t n_tri = 0;
    const int rc_load = o.proc ? A::proc(o.proc, &tri, &norm, &n_tri, o.arith) : A::load(o.obj.c_str(), &tri, &norm, &n_tri, o.arith);
    if (rc_load != CERES_OK) { std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1; }
    if (n_tri == 0) { std::fprintf(stderr, "The given scene is empty or cannot be loaded\n"); return 1; }   // static.cpp:77-80
    if (o.rot_axis >= 0) A::rotate(tri, n_tri, o.rot_axis, v.rot_deg, o.arith);

    std::printf("Building BVH ( using BinnedSahBuilder%s )...\n", o.gpu_bvh ? " on the GPU" : "");
    const double t0 = now_s();
    typename A::Node* nodes = nullptr; uint64_t* prim = nullptr; size_t n_nodes = 0;
    const int rc_bvh = A::bvh(tri, n_tri, &nodes, &n_nodes, &prim, o.gpu_bvh, o.device, o.arith);
    if (rc_bvh != CERES_OK) { std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1; }
    std::printf("%g\n", now_s() - t0);
    std::printf("BVH of %zu node(s) and %zu reference(s)\n", n_nodes, n_tri);

    if (o.cpu) {
        ceres_cpu_scene* cs = A::cpu_scene(tri, n_tri, norm, nodes, n_nodes, prim);
        ceres_free(nodes); ceres_free(prim); ceres_free(tri); ceres_free(norm);
        if (!cs) { std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1; }
        const int rc = frames_loop(o, v, [&](const S* basis, const S* sun, uint8_t* rgb, ceres_stats* st) {
            return A::render_cpu(cs, basis, sun, o.mode, rgb, o.W, o.H, st, o.threads);
        }, "CPU");
        ceres_cpu_scene_destroy(cs);
        return rc;
    }
    ceres_scene* scene = A::scene(tri, n_tri, norm, nodes, n_nodes, prim, o.device);
    // --gpus N: one scene copy per further rank, on the next devices (mod the device count)
    std::vector<ceres_scene*> ranks(1, scene);
    if (scene && o.gpus > 1) {
        const int ndev = ceres_device_count();
        for (int r = 1; r < o.gpus && ndev > 0; ++r) {
            ceres_scene* sr = A::scene(tri, n_tri, norm, nodes, n_nodes, prim, (o.device + r) % ndev);
            if (!sr) break;
            ranks.push_back(sr);
        }
    }
    ceres_free(nodes); ceres_free(prim); ceres_free(tri); ceres_free(norm);
    auto destroy = [&] { for (auto* sr : ranks) ceres_scene_destroy(sr); };
    if (!scene || int(ranks.size()) != o.gpus) {
        std::fprintf(stderr, "error: %s\n", ceres_last_error());
        destroy();
        return 1;
    }
    auto render = [&](const S* basis, const S* sun, uint8_t* rgb, ceres_stats* st) {
        return o.gpus > 1 ? A::render_multi(ranks.data(), uint32_t(o.gpus), uint32_t(o.row_block), basis, sun, o.mode, rgb,
                                            o.W, o.H, st)
                          : A::render(scene, basis, sun, o.mode, rgb, o.W, o.H, st);
    };
    const int rc = frames_loop(o, v, render, "HIP");
    destroy();
    return rc;
}

// The frame loop of static.cpp / anim.cpp (render :130 / :104-110, PPM :135-147, "Total Rays"
// anim.cpp:127) over `render`; `where` names the render path in the progress lines.
template <class S, class Render>
int frames_loop(const Opts& o, const Num<S>& v, Render&& render, const char* where) {
    using A = Api<S>;

    // frame poses: count + k orbit rotations for frame k (count = 0, frames = 1: the plain camera)
    const uint32_t n_pose = uint32_t(o.orbit_count + o.frames);
    std::vector<S> bases(12 * size_t(n_pose)), suns(3 * size_t(n_pose));
    if (A::orbit(v, o.W, o.H, n_pose, bases.data(), suns.data(), o.arith) != CERES_OK) {
        std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1;
    }
    std::vector<uint8_t> rgb(3 * o.W * o.H);
    ceres_stats st{};
    unsigned long long tot_rays = 0;
    std::vector<double> ms, e2e;
    for (int k = 0; k < o.frames; ++k) {
        const S* basis = bases.data() + 12 * size_t(o.orbit_count + k);
        const S* sun = suns.data() + 3 * size_t(o.orbit_count + k);
        if (o.cpu) std::printf("Rendering image %d (%zux%zu) on the %s%s...\n", k, o.W, o.H, where,
                               o.threads ? (" with " + std::to_string(o.threads) + " threads").c_str() : "");
        else if (o.gpus > 1) std::printf("Rendering image %d (%zux%zu) on %d %s ranks from device %d...\n", k, o.W, o.H, o.gpus, where, o.device);
        else std::printf("Rendering image %d (%zux%zu) on %s device %d...\n", k, o.W, o.H, where, o.device);
        const double t1 = now_s();
        int rc = render(basis, sun, rgb.data(), &st);
        const double t2 = now_s();
        if (rc != CERES_OK) { std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1; }
        std::printf("%g\n", t2 - t1);
        std::printf("Rays: %llu\tHits: %llu\n", (unsigned long long)st.rays, (unsigned long long)st.hits);   // anim.cpp:109
        tot_rays += st.rays;
        for (int r = 0; r < o.bench; ++r) {
            ceres_stats s2{};
            const double b1 = now_s();
            rc = render(basis, sun, rgb.data(), &s2);
            e2e.push_back((now_s() - b1) * 1e3);          // the whole call: launch + kernel + RGB8 copy to the host
            if (rc != CERES_OK) { std::fprintf(stderr, "error: %s\n", ceres_last_error()); return 1; }
            ms.push_back(s2.ms);
        }
        std::string path = o.out;
        if (o.frames > 1) {
            char suffix[16];
            std::snprintf(suffix, sizeof suffix, "_%03d", k);
            const size_t dot = path.rfind('.');
            const size_t slash = path.rfind('/');
            if (dot == std::string::npos || (slash != std::string::npos && dot < slash)) path += suffix;
            else path.insert(dot, suffix);
        }
        if (FILE* f = std::fopen(path.c_str(), "wb")) {              // static.cpp:135-147
            std::fprintf(f, "P6 %zu %zu %d\n", o.W, o.H, 255);
            std::fwrite(rgb.data(), 1, rgb.size(), f);
            std::fclose(f);
        } else {
            std::fprintf(stderr, "error: cannot write %s\n", path.c_str());
            return 1;
        }
    }
    if (o.frames > 1) std::printf("Total Rays: %llu\n", tot_rays);   // anim.cpp:127
    if (o.json) {
        double med = 0, e2e_med = 0;
        if (!ms.empty()) { std::sort(ms.begin(), ms.end()); med = ms[ms.size() / 2]; }
        if (!e2e.empty()) { std::sort(e2e.begin(), e2e.end()); e2e_med = e2e[e2e.size() / 2]; }
        std::printf("{\"rays\": %llu, \"hits\": %llu, \"W\": %zu, \"H\": %zu, \"device_ms\": %.4f, \"bench_median_ms\": %.4f, "
                    "\"mrays_per_s\": %.3f, \"e2e_ms\": %.4f}\n",
                    (unsigned long long)st.rays, (unsigned long long)st.hits, o.W, o.H, st.ms, med,
                    med > 0 ? double(st.rays) / (med * 1e3) : 0.0, e2e_med);
    }
    if (o.json && o.cpu)                                              // the reference's Statistics, all rays
        std::printf("{\"node_pairs\": %llu, \"tri_tests\": %llu, \"primary_rays\": %llu, \"shadow_rays\": %llu}\n",
                    (unsigned long long)st.node_pairs, (unsigned long long)st.tri_tests,
                    (unsigned long long)st.primary_rays, (unsigned long long)st.shadow_rays);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    Opts o;
    if (!parse(argc, argv, o)) return usage();
    if (o.arith == CERES_ARITH_FMA) o.mode |= CERES_MODE_FMA;
    if (o.cpu && (o.gpus > 1 || o.gpu_bvh || (o.mode & CERES_MODE_QBVH4))) {
        std::fprintf(stderr, "error: --cpu renders in one process on the host (not with --gpus, --gpu-bvh, --qbvh)\n");
        return 2;
    }
    return o.f64 ? run<double>(o, o.d) : run<float>(o, o.f);
}
