// host_sanitize.cpp -- drives the product's HOST code (scene_host.cpp: OBJ loader, rotation,
// binned-SAH BVH build, camera basis, orbit, BVH2 -> GPU relayout and the exact BVH4 collapse,
// float and double) under AddressSanitizer + UndefinedBehaviorSanitizer ("run
// host code under -fsanitize=address,undefined").  Built and run by tests/test_host_sanitizers.py:
//   g++ -fsanitize=address,undefined -fno-sanitize-recover=all ... host_sanitize.cpp scene_host.cpp
// usage: host_sanitize <obj> ...   (prints one line per mesh; any sanitizer report aborts)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"

namespace ceres {
// render_hip.hip defines the per-thread error buffer in the real library
char* error_buffer() {
    static thread_local char buf[kErrorBufferSize] = "";
    return buf;
}
}  // namespace ceres

using namespace ceres;

static int check_float(const char* what, float* tri, float* norm, size_t n) {
    if (n == 0) { std::printf("%s: empty (%s)\n", what, error_buffer()); return 0; }
    if (ceres_rotate_triangles(tri, n, 0, 90.0f) != CERES_OK) return 1;
    uint32_t* nodes = nullptr; uint64_t* prim = nullptr; size_t n_nodes = 0;
    if (ceres_bvh_build(tri, n, &nodes, &n_nodes, &prim) != CERES_OK) return 1;
    std::vector<SiblingPair> pairs; std::vector<Tri48> leaf; std::vector<uint32_t> orig;
    uint32_t depth = 0, rlc = 0, rlf = 0;
    if (relayout_bvh(reinterpret_cast<const RefNode*>(nodes), n_nodes, prim, n, reinterpret_cast<const Tri48*>(tri),
                     pairs, leaf, orig, depth, rlc, rlf) != CERES_OK) return 1;
    std::vector<Node4> n4; uint32_t stack4 = 0, nc = 0;
    if (!rlc && build_shadow_bvh4(pairs, n4, stack4, nc) != CERES_OK) return 1;   // as ceres_scene_create
    const float eye[3] = {0, -15, 2}, dir[3] = {0, 1, 0}, up[3] = {0, 0, 1}, sun[3] = {-50, -20, 0}, ax[3] = {0, 0, 1};
    float basis[9], b12[12 * 3], s3[9], d3[9];
    if (ceres_camera_basis(eye, dir, up, 60.f, 333, 217, basis) != CERES_OK) return 1;
    if (ceres_orbit_cameras(eye, dir, up, sun, 60.f, 333, 217, ax, 45.f, 3, 1, b12, s3, d3) != CERES_OK) return 1;
    std::printf("%s: %zu tris, %zu nodes, %zu pairs, depth %u, %zu nodes4 (stack %u)\n", what, n, n_nodes, pairs.size(),
                depth, n4.size(), stack4);
    ceres_free(nodes); ceres_free(prim);
    return 0;
}

static int check_double(const char* what, double* tri, double* norm, size_t n) {
    (void)norm;
    if (n == 0) return 0;
    if (ceres_rotate_triangles_f64(tri, n, 1, -145.0) != CERES_OK) return 1;
    uint64_t* nodes = nullptr; uint64_t* prim = nullptr; size_t n_nodes = 0;
    if (ceres_bvh_build_f64(tri, n, &nodes, &n_nodes, &prim) != CERES_OK) return 1;
    std::vector<SiblingPair64> pairs; std::vector<Tri96> leaf; std::vector<uint32_t> orig;
    uint32_t depth = 0, rlc = 0, rlf = 0;
    if (relayout_bvh64(reinterpret_cast<const RefNode64*>(nodes), n_nodes, prim, n, reinterpret_cast<const Tri96*>(tri),
                       pairs, leaf, orig, depth, rlc, rlf) != CERES_OK) return 1;
    std::printf("%s (double): %zu tris, %zu nodes, depth %u\n", what, n, n_nodes, depth);
    ceres_free(nodes); ceres_free(prim);
    return 0;
}

int main(int argc, char** argv) {
    int bad = 0;
    for (int i = 1; i < argc; ++i) {
        float* t = nullptr; float* nm = nullptr; size_t n = 0;
        const int rc = ceres_obj_load(argv[i], &t, &nm, &n);
        if (rc == CERES_OK) bad |= check_float(argv[i], t, nm, n);
        else std::printf("%s: load error %d (%s)\n", argv[i], rc, error_buffer());
        ceres_free(t); ceres_free(nm);
        double* td = nullptr; double* nd = nullptr; size_t m = 0;
        if (ceres_obj_load_f64(argv[i], &td, &nd, &m) == CERES_OK) bad |= check_double(argv[i], td, nd, m);
        ceres_free(td); ceres_free(nd);
    }
    float* t = nullptr; float* nm = nullptr; size_t n = 0;
    if (ceres_proc_mesh(101, &t, &nm, &n) != CERES_OK) return 1;
    bad |= check_float("proc 101", t, nm, n);
    ceres_free(t); ceres_free(nm);
    // argument errors come back as codes, not crashes
    if (ceres_bvh_build(nullptr, 0, nullptr, nullptr, nullptr) == CERES_OK) bad = 1;
    // an unreadable file is an empty mesh, as in obj_norms.hpp:123-126 (the caller then stops,
    // static.cpp:77-80)
    if (ceres_obj_load("/nonexistent/x.obj", &t, &nm, &n) != CERES_OK || n != 0) bad = 1;
    ceres_free(t); ceres_free(nm);
    std::printf(bad ? "FAILED\n" : "host code clean\n");
    return bad;
}
