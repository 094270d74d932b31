// dropin_bench -- end-to-end cost of the drop-in boundary, the way the reference's callers pay it.
//
// static.cpp:76-133 / anim.cpp:93-110 call render<float>() (render.hpp:86-89) with a caller-owned
// host float framebuffer (3*W*H floats) and time that call.  This program does exactly that
// through include/ceres/render.hpp (scene cached after the first call, as anim.cpp's frames reuse
// it), and reports the wall time per call (e2e) beside the kernel's own device time
// (ceres_render_f32 stats.ms) and the PPM sha-independent checks the test harness needs.
//
// hash_ms: the per-call content hash of the caller's arrays alone (render.hpp's scene check,
// ceres_content_hash over nodes, primitive_indices, triangles and tri_norms); the
// dropin_bench_trust build defines CERES_DROPIN_TRUST_UNCHANGED and skips it.
//
// usage: dropin_bench <obj> | --proc N  [--size W H] [--rotate x|y|z deg] [--eye x y z] [--dir x y z]
//                     [--up x y z] [--sun x y z] [--reps N] [--out f.ppm]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ceres/render.hpp"

int main(int argc, char** argv) {
    std::string obj;
    size_t W = 1920, H = 1080;
    int rot_axis = -1, reps = 50, proc = 0;
    float rot_deg = 0.f;
    float eye[3] = {0.f, -15.f, 2.f}, dir[3] = {0.f, 1.f, 0.f}, up[3] = {0.f, 0.f, 1.f}, sun[3] = {-50.f, -20.f, 0.f};
    std::string out;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto v3 = [&](float* d) { for (int k = 0; k < 3; ++k) d[k] = std::strtof(argv[++i], nullptr); };
        if (a == "--size") { W = std::strtoul(argv[++i], nullptr, 10); H = std::strtoul(argv[++i], nullptr, 10); }
        else if (a == "--rotate") { const char c = argv[++i][0]; rot_axis = c == 'x' ? 0 : c == 'y' ? 1 : 2; rot_deg = std::strtof(argv[++i], nullptr); }
        else if (a == "--eye") v3(eye);
        else if (a == "--dir") v3(dir);
        else if (a == "--up") v3(up);
        else if (a == "--sun") v3(sun);
        else if (a == "--reps") reps = std::atoi(argv[++i]);
        else if (a == "--proc") proc = std::atoi(argv[++i]);
        else if (a == "--out") out = argv[++i];
        else obj = a;
    }
    float *tri = nullptr, *norm = nullptr;
    size_t n_tri = 0;
    const int lrc = proc ? ceres_proc_mesh(proc, &tri, &norm, &n_tri) : ceres_obj_load(obj.c_str(), &tri, &norm, &n_tri);
    if (lrc != CERES_OK || n_tri == 0) {
        std::fprintf(stderr, "cannot load %s: %s\n", proc ? "the procedural mesh" : obj.c_str(), ceres_last_error());
        return 1;
    }
    std::vector<ceres::HostTriangle> triangles(n_tri);
    std::memcpy(triangles.data(), tri, n_tri * 48);
    std::vector<std::array<ceres::vec3<float>, 3>> tri_norms(n_tri);
    std::memcpy(tri_norms.data(), norm, n_tri * 36);
    ceres_free(tri);
    ceres_free(norm);
    if (rot_axis == 0) rotate_triangles<0>(rot_deg, triangles.data(), n_tri);          // static.cpp:76-98
    if (rot_axis == 1) rotate_triangles<1>(rot_deg, triangles.data(), n_tri);
    if (rot_axis == 2) rotate_triangles<2>(rot_deg, triangles.data(), n_tri);
    uint32_t* nodes32 = nullptr;
    uint64_t* prim64 = nullptr;
    size_t n_nodes = 0;
    if (ceres_bvh_build(reinterpret_cast<const float*>(triangles.data()), n_tri, &nodes32, &n_nodes, &prim64) != CERES_OK) {
        std::fprintf(stderr, "bvh build: %s\n", ceres_last_error());
        return 1;
    }
    ceres::HostBvh bvh;                                                                 // static.cpp:100-107
    bvh.node_count = n_nodes;
    bvh.nodes.reset(new ceres::HostBvh::Node[n_nodes]);
    std::memcpy(bvh.nodes.get(), nodes32, n_nodes * 32);
    bvh.primitive_indices.reset(new size_t[n_tri]);
    std::memcpy(bvh.primitive_indices.get(), prim64, n_tri * 8);
    ceres_free(nodes32);
    ceres_free(prim64);

    Camera<float> camera{ceres::vec3<float>(eye[0], eye[1], eye[2]), ceres::vec3<float>(dir[0], dir[1], dir[2]),
                         ceres::vec3<float>(up[0], up[1], up[2]), 60.f};
    const ceres::vec3<float> sun_position(sun[0], sun[1], sun[2]);
    std::vector<float> pixels(3 * W * H);                                               // static.cpp:127
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    auto [rays, hits] = render(camera, sun_position, bvh, triangles.data(), tri_norms.data(), pixels.data(), W, H);
    const double first_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    std::vector<double> e2e;
    for (int r = 0; r < reps; ++r) {
        auto a = clk::now();
        auto rh = render(camera, sun_position, bvh, triangles.data(), tri_norms.data(), pixels.data(), W, H);
        e2e.push_back(std::chrono::duration<double, std::milli>(clk::now() - a).count());
        if (rh.first != rays || rh.second != hits) { std::fprintf(stderr, "rays/hits changed between calls\n"); return 1; }
    }
    // the kernel alone: the same scene through the C ABI, device time from HIP events
    float basis[12];
    std::memcpy(basis, eye, sizeof eye);
    if (ceres_camera_basis(eye, dir, up, 60.f, W, H, basis + 3) != CERES_OK) return 1;
    ceres_scene* sc = ceres::detail::cache().scene;
    std::vector<double> dev;
    for (int r = 0; r < std::max(5, reps / 2); ++r) {
        ceres_stats st{};
        if (ceres_render_f32(sc, basis, sun, CERES_MODE_FULL, nullptr, nullptr, W, H, &st) != CERES_OK) {
            std::fprintf(stderr, "render: %s\n", ceres_last_error());
            return 1;
        }
        dev.push_back(st.ms);
    }
    if (!out.empty()) {                                                                // static.cpp:135-147
        FILE* f = std::fopen(out.c_str(), "wb");
        if (!f) return 1;
        std::fprintf(f, "P6 %zu %zu %d\n", W, H, 255);
        for (size_t j = H; j > 0; --j)
            for (size_t i = 0; i < W; ++i) {
                const size_t k = 3 * (W * (j - 1) + i);
                unsigned char px[3];
                for (int c = 0; c < 3; ++c) px[c] = static_cast<unsigned char>(std::max(std::min(pixels[k + c] * 255.f, 255.f), 0.f));
                std::fwrite(px, 1, 3, f);
            }
        std::fclose(f);
    }
    std::vector<double> hash;
    for (int r = 0; r < 5; ++r) {
        auto a = clk::now();
        uint64_t h = ceres_content_hash(bvh.nodes.get(), n_nodes * 32) ^ ceres_content_hash(bvh.primitive_indices.get(), n_tri * 8);
        h ^= ceres_content_hash(triangles.data(), n_tri * 48) ^ ceres_content_hash(tri_norms.data(), n_tri * 36);
        hash.push_back(std::chrono::duration<double, std::milli>(clk::now() - a).count());
        volatile uint64_t sink = h;
        (void)sink;
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
    auto mn = [](const std::vector<double>& v) { return v.empty() ? 0.0 : *std::min_element(v.begin(), v.end()); };
    std::printf("{\"W\": %zu, \"H\": %zu, \"rays\": %d, \"hits\": %d, \"reps\": %d, \"first_call_ms\": %.3f, "
                "\"e2e_ms_median\": %.4f, \"e2e_ms_min\": %.4f, \"device_ms_median\": %.4f, \"float_bytes\": %zu, "
                "\"hash_ms_median\": %.3f, \"hashed_bytes\": %zu, \"trust_unchanged\": %d, \"e2e_mrays_per_s\": %.2f}\n",
                W, H, rays, hits, reps, first_ms, med(e2e), mn(e2e), med(dev), 3 * W * H * sizeof(float), med(hash),
                n_nodes * 32 + n_tri * (8 + 48 + 36),
#ifdef CERES_DROPIN_TRUST_UNCHANGED
                1,
#else
                0,
#endif
                med(e2e) > 0 ? rays / (med(e2e) * 1e3) : 0.0);
    return 0;
}
