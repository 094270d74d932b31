// render_cpu.cpp -- the product's CPU render path: render<float>() (render.hpp:86-156) on host
// cores, behind `./render --cpu` ("the CLI can run the CPU path, so
// config 1 works with no GPU").  It is chosen explicitly (ceres_render_cpu_f32 / --cpu); nothing
// falls back to it -- without a GPU the device calls still fail loudly.
//
// It walks the product's own scene layout (ceres_types.hpp: 64-B sibling-pair records, leaf-ordered
// triangles, orig[] slot -> original index) in the reference's order, with the same per-ray
// arithmetic the gfx950 kernels compute (render_hip.hip: trace, tri_test, hit_point, shade), so its
// images are the reference's bit for bit in both arithmetics:
//   * CERES_MODE_FMA: GCC's contraction sites of the reference CMake build (CMakeLists.txt:11-13;
//     oracle/contraction_sites.txt) as explicit std::fma; without it every expression is plain (this
//     file is compiled with -ffp-contract=off, so the compiler adds none);
//   * FastNodeIntersector (node_intersectors.hpp:83-103) or, with CERES_MODE_ROBUST, the
//     RobustNodeIntersector (:54-79);
//   * the shadow ray is traced like the reference traces it: the closest-hit traversal
//     (render.hpp:135-136; only whether it hits is used), so the traversal statistics are the
//     reference's Statistics (single_ray_traverser.hpp:83,53) for primary and shadow rays alike.
// Rows are spread over OpenMP threads (render.hpp:103, `omp parallel for`).
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include <omp.h>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "pow24.hpp"

using namespace ceres;

struct ceres_cpu_scene {
    std::vector<SiblingPair> pairs;   // pair k: the two children of an inner node (pairs[0]: the root's)
    std::vector<Tri48> tris;          // leaf order
    std::vector<uint32_t> orig;       // leaf slot -> original triangle index (tri_norms order)
    std::vector<float> norms;         // 9 floats per original triangle (obj_norms.hpp:113-115)
    uint32_t depth = 0, root_leaf_count = 0, root_leaf_first = 0;
};

namespace {

struct V3f { float x, y, z; };
inline V3f operator+(V3f a, V3f b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3f operator-(V3f a, V3f b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3f operator*(V3f a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3f v3(const float* p) { return {p[0], p[1], p[2]}; }

// vector.hpp:134-167 as each build computes it (see render_hip.hip dotA / dotB / crossG): dot "A"
// fma(a2, b2, fma(a0, b0, a1 b1)), Triangle::intersect's v = dot(r, e1) as "B"
// fma(a2, b2, fma(a1, b1, a0 b0)), cross a_j b_k - a_k b_j as fma(a_j, b_k, -(a_k b_j)).
template <bool G> inline float dot_a(V3f a, V3f b) {
    if constexpr (G) return std::fma(a.z, b.z, std::fma(a.x, b.x, a.y * b.y));
    float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z;
    return s;
}
template <bool G> inline float dot_b(V3f a, V3f b) {
    if constexpr (G) return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x));
    return dot_a<false>(a, b);
}
template <bool G> inline V3f cross_g(V3f a, V3f b) {
    if constexpr (G) return {std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)), std::fma(a.x, b.y, -(a.y * b.x))};
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <bool G> inline V3f normalize_g(V3f v) { const float inv = 1.0f / std::sqrt(dot_a<G>(v, v)); return v * inv; }

// The slab constants of a ray and the test of one box (entry e, exit x; hit iff e <= x).
//   fast: inv = safe_inverse(d) (vector.hpp:69-74), s = -o inv, each slab fma(bound, inv, s); the
//         octant's near / far bound is min / max of the two fmas (fma is monotone in the bound);
//   robust: inv = 1 / d, the exit slabs scaled by inv padded by 2 ulps (utilities.hpp:102-106).
// fminf / fmaxf (the non-NaN operand when one is NaN; the sign of a zero result is never observed:
// only comparisons read these values), written out so they inline instead of calling libm
inline float min_nn(float x, float y) { return (x < y || std::isnan(y)) ? x : y; }
inline float max_nn(float x, float y) { return (x > y || std::isnan(y)) ? x : y; }
template <bool R> struct SlabC { float ix, iy, iz, sx, sy, sz; V3f o; };
inline float pad2(float x) { uint32_t b; std::memcpy(&b, &x, 4); b += 2; float y; std::memcpy(&y, &b, 4); return std::isfinite(x) ? y : x; }
template <bool R> inline SlabC<R> slab_of(V3f o, V3f d) {
    SlabC<R> s;
    if constexpr (R) {
        s.ix = 1.0f / d.x; s.iy = 1.0f / d.y; s.iz = 1.0f / d.z;
        s.sx = pad2(s.ix); s.sy = pad2(s.iy); s.sz = pad2(s.iz);
    } else {
        auto safe_inv = [](float x) { return 1.0f / (std::fabs(x) < FLT_EPSILON ? std::copysign(FLT_EPSILON, x) : x); };
        s.ix = safe_inv(d.x); s.iy = safe_inv(d.y); s.iz = safe_inv(d.z);
        s.sx = (-o.x) * s.ix; s.sy = (-o.y) * s.iy; s.sz = (-o.z) * s.iz;
    }
    s.o = o;
    return s;
}
template <bool R> inline bool box_hit(const SlabC<R>& s, const float* b, float tmin, float tmax, float& entry) {
    float e, x;                                   // b: xmin, xmax, ymin, ymax, zmin, zmax
    if constexpr (R) {
        const bool nx = std::signbit(s.ix), ny = std::signbit(s.iy), nz = std::signbit(s.iz);
        const float ex = ((nx ? b[1] : b[0]) - s.o.x) * s.ix, xx = ((nx ? b[0] : b[1]) - s.o.x) * s.sx;
        const float ey = ((ny ? b[3] : b[2]) - s.o.y) * s.iy, xy = ((ny ? b[2] : b[3]) - s.o.y) * s.sy;
        const float ez = ((nz ? b[5] : b[4]) - s.o.z) * s.iz, xz = ((nz ? b[4] : b[5]) - s.o.z) * s.sz;
        e = max_nn(ex, max_nn(ey, max_nn(ez, tmin)));
        x = min_nn(xx, min_nn(xy, min_nn(xz, tmax)));
    } else {
        const float a0 = std::fma(b[0], s.ix, s.sx), a1 = std::fma(b[1], s.ix, s.sx);
        const float b0 = std::fma(b[2], s.iy, s.sy), b1 = std::fma(b[3], s.iy, s.sy);
        const float c0 = std::fma(b[4], s.iz, s.sz), c1 = std::fma(b[5], s.iz, s.sz);
        e = max_nn(min_nn(a0, a1), max_nn(min_nn(b0, b1), max_nn(min_nn(c0, c1), tmin)));
        x = min_nn(max_nn(a0, a1), min_nn(max_nn(b0, b1), min_nn(max_nn(c0, c1), tmax)));
    }
    entry = e;
    return e <= x;
}

// Triangle::intersect (triangle.hpp:95-115): Moller-Trumbore, left-handed normal, IEEE 1 / det.
template <bool G> inline bool tri_hit(const Tri48& tr, V3f o, V3f d, float tmin, float tmax, float& t_out, float& u_out,
                                      float& v_out) {
    const V3f c = v3(tr.p0) - o;
    const V3f r = cross_g<G>(d, c);
    const float inv_det = 1.0f / dot_a<G>(v3(tr.n), d);
    const float u = dot_a<G>(r, v3(tr.e2)) * inv_det;
    const float v = dot_b<G>(r, v3(tr.e1)) * inv_det;
    const float w = 1.0f - u - v;
    if (u >= 0 && v >= 0 && w >= 0) {
        const float t = dot_a<G>(v3(tr.n), c) * inv_det;
        if (t >= tmin && t <= tmax) { t_out = t; u_out = u; v_out = v; return true; }
    }
    return false;
}

struct HitRec { uint32_t slot; float t, u, v; };

// SingleRayTraverser::intersect (single_ray_traverser.hpp:68-126) with a closest-primitive
// intersector over the sibling-pair records: both children's boxes against the step's tmax, left
// leaf then right leaf in leaf order (each accepted hit lowers tmax, the last accepted one wins),
// the far child pushed, ties left.  steps / tests: the reference's Statistics.
template <bool G, bool R>
bool trace_closest(const ceres_cpu_scene& s, V3f o, V3f d, uint32_t* stack, uint32_t cap, HitRec& best, uint64_t& steps,
                   uint64_t& tests, bool& overflow) {
    const float tmin = 0.0f;
    float tmax = FLT_MAX;                                                   // ray.hpp:17-21
    bool have = false;
    auto leaf = [&](uint32_t first, uint32_t count) {                      // intersect_leaf, :43-63
        tests += count;
        for (uint32_t k = first; k < first + count; ++k) {
            float t, u, v;
            if (tri_hit<G>(s.tris[k], o, d, tmin, tmax, t, u, v)) { best = {k, t, u, v}; have = true; tmax = t; }
        }
    };
    if (s.root_leaf_count) {                                                // :72-73
        leaf(s.root_leaf_first, s.root_leaf_count);
        return have;
    }
    const SlabC<R> sl = slab_of<R>(o, d);
    uint32_t sp = 0, cur = 0;
    while (true) {
        ++steps;                                                            // :83
        const SiblingPair& p = s.pairs[cur];
        float el, er;
        const bool hl = box_hit<R>(sl, p.lb, tmin, tmax, el), hr = box_hit<R>(sl, p.rb, tmin, tmax, er);
        if (hl && p.lcount) leaf(p.lfirst, p.lcount);                       // :89-97
        if (hr && p.rcount) leaf(p.rfirst, p.rcount);                       // :99-107
        const bool go_l = hl && !p.lcount, go_r = hr && !p.rcount;
        if (go_l && go_r) {                                                 // :109-115
            const bool swap = el > er;
            if (sp >= cap) { overflow = true; return have; }
            stack[sp++] = swap ? p.lfirst : p.rfirst;
            cur = swap ? p.rfirst : p.lfirst;
        } else if (go_l || go_r) {                                          // :115-117
            cur = go_l ? p.lfirst : p.rfirst;
        } else {                                                            // :118-121
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    return have;
}

// Hit point + self-intersection offset (render.hpp:127-133; p1 = p0 - e1, p2 = p0 + e2).
template <bool G> inline V3f hit_point(const Tri48& tr, V3f normal, float hu, float hv) {
    const V3f p0 = v3(tr.p0), p1 = p0 - v3(tr.e1), p2 = p0 + v3(tr.e2);
    const float scale = -0.00001;
    const float w = 1 - hu - hv;
    if constexpr (G) {
        auto c = [&](float a, float q1, float q2, float n) { return std::fma(n, scale, std::fma(w, q2, std::fma(hv, q1, hu * a))); };
        return {c(p0.x, p1.x, p2.x, normal.x), c(p0.y, p1.y, p2.y, normal.y), c(p0.z, p1.z, p2.z, normal.z)};
    }
    const V3f p = p0 * hu + p1 * hv + p2 * w;
    return p + normal * scale;
}

// smooth_shading (render.hpp:46-84): std::pow(float, 24) is the double pow narrowed to float
// (pow24f, pinned against glibc for every float by tests/test_pow24.py).
template <bool G> inline void shade(V3f sun_line, const float* nrm, V3f view, float u, float v, float c[3]) {
    c[0] = c[1] = c[2] = 0.0f;
    const float amb = 0.2;
    const V3f vneg = view * -1.0f;
    const float w[3] = {u, v, 1 - u - v};
    for (int k = 0; k < 3; ++k) {
        const V3f N{nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]};
        const float lam = std::fabs(dot_a<G>(sun_line, N));
        const float spec = 0.8f * pow24f(dot_a<G>(N, normalize_g<G>(sun_line + vneg)));
        const float base = G ? std::fma(lam, 0.5f, amb) : amb + 0.5f * lam;
        auto clamp01 = [](float x) { return (x < 0.f) ? 0.f : (1.f < x) ? 1.f : x; };   // std::clamp
        auto ch = [&](float k2) { return G ? std::fma(base, k2, spec) : base * k2 + spec; };
        c[0] += w[k] * clamp01(ch(0.5f));
        c[1] += w[k] * clamp01(ch(0.0f));
        c[2] += w[k] * clamp01(ch(0.8f));
    }
}

inline uint8_t quantize(float x) {                                          // static.cpp:141-143
    const float a = x * 255;
    const float m = (255.0f < a) ? 255.0f : a;
    const float q = (m < 0.0f) ? 0.0f : m;
    return static_cast<uint8_t>(static_cast<int>(q));
}

struct Counts { uint64_t primary = 0, shadow = 0, hits = 0, steps = 0, tests = 0; bool overflow = false; };

template <bool G, bool R>
void render_rows(const ceres_cpu_scene& s, const float* b12, const float* sun, bool full, float* pixels, uint8_t* rgb8,
                 size_t W, size_t H, int threads, Counts& tot) {
    const V3f eye = v3(b12), dir = v3(b12 + 3), iu = v3(b12 + 6), iv = v3(b12 + 9), sunp = v3(sun);
    const uint32_t cap = std::max<uint32_t>(1, s.depth);                    // a push per level: <= depth - 1 entries
    uint64_t primary = 0, shadow = 0, hits = 0, steps = 0, tests = 0;
    int overflow = 0;
#pragma omp parallel num_threads(threads > 0 ? threads : omp_get_max_threads()) reduction(+ : primary, shadow, hits, steps, tests) reduction(| : overflow)
    {
        std::vector<uint32_t> stack(cap);
#pragma omp for schedule(dynamic, 1)
        for (long long jj = 0; jj < (long long)H; ++jj) {
            const size_t j = size_t(jj);
            bool ov = false;
            for (size_t i = 0; i < W; ++i) {
                // render.hpp:105-111 (GCC: dir + fma(iv, v, iu u))
                const float u = 2 * (float(i) + 0.5f) / float(W) - 1.0f;
                const float v = 2 * (float(j) + 0.5f) / float(H) - 1.0f;
                const V3f a = G ? V3f{dir.x + std::fma(iv.x, v, iu.x * u), dir.y + std::fma(iv.y, v, iu.y * u),
                                      dir.z + std::fma(iv.z, v, iu.z * u)}
                                : iu * u + iv * v + dir;
                const V3f view = normalize_g<G>(a);
                HitRec h{0, 0.f, 0.f, 0.f};
                ++primary;
                float c[3] = {0.f, 0.f, 0.f};                                // a miss: render.hpp:116-117
                if (trace_closest<G, R>(s, eye, view, stack.data(), cap, h, steps, tests, ov)) {
                    ++hits;
                    const Tri48& tr = s.tris[h.slot];
                    const V3f normal = normalize_g<G>(v3(tr.n));
                    if (!full) {                                             // render.hpp:123-125 (primary only)
                        c[0] = std::fabs(normal.x); c[1] = std::fabs(normal.y); c[2] = std::fabs(normal.z);
                    } else {
                        const V3f p = hit_point<G>(tr, normal, h.u, h.v);
                        const V3f sun_line = normalize_g<G>(sunp - p);       // render.hpp:135
                        HitRec hs{0, 0.f, 0.f, 0.f};
                        ++shadow;
                        if (trace_closest<G, R>(s, p, sun_line, stack.data(), cap, hs, steps, tests, ov))
                            ++hits;                                          // render.hpp:146-149: occluded, RGB 0
                        else
                            shade<G>(sun_line, s.norms.data() + 9 * size_t(s.orig[h.slot]), view, h.u, h.v, c);
                    }
                }
                const size_t px = W * j + i;                                 // render.hpp:107
                if (pixels) { pixels[3 * px] = c[0]; pixels[3 * px + 1] = c[1]; pixels[3 * px + 2] = c[2]; }
                if (rgb8) {                                                  // static.cpp:135-147: top row first
                    uint8_t* q = rgb8 + 3 * (W * (H - 1 - j) + i);
                    q[0] = quantize(c[0]); q[1] = quantize(c[1]); q[2] = quantize(c[2]);
                }
            }
            overflow |= ov ? 1 : 0;
        }
    }
    tot.primary = primary; tot.shadow = shadow; tot.hits = hits; tot.steps = steps; tot.tests = tests;
    tot.overflow = overflow != 0;
}

}  // namespace

extern "C" {

ceres_cpu_scene* ceres_cpu_scene_create(const float* tri48, size_t n_tri, const float* norm36, const void* nodes32,
                                        size_t n_nodes, const uint64_t* prim64) {
    if (!tri48 || !norm36 || !nodes32 || !prim64 || n_tri == 0 || n_nodes == 0) {
        set_error(CERES_EINVAL, "ceres_cpu_scene_create: empty scene or null argument");
        return nullptr;
    }
    if (n_tri > 0xffffffffull || n_nodes > 0xffffffffull) { set_error(CERES_EUNSUPPORTED, "scene too large"); return nullptr; }
    auto* s = new (std::nothrow) ceres_cpu_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    try {
        if (relayout_bvh(static_cast<const RefNode*>(nodes32), n_nodes, prim64, n_tri, reinterpret_cast<const Tri48*>(tri48),
                         s->pairs, s->tris, s->orig, s->depth, s->root_leaf_count, s->root_leaf_first)) {
            delete s;
            return nullptr;
        }
        s->norms.assign(norm36, norm36 + 9 * n_tri);
    } catch (const std::bad_alloc&) {
        delete s;
        set_error(CERES_ENOMEM, "out of host memory");
        return nullptr;
    }
    return s;
}

void ceres_cpu_scene_destroy(ceres_cpu_scene* scene) { delete scene; }

int ceres_render_cpu_f32(const ceres_cpu_scene* scene, const float basis12[12], const float sun[3], int mode, float* pixels,
                         uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats, int threads) {
    if (!scene || !basis12 || !sun || width == 0 || height == 0) return set_error(CERES_EINVAL, "render (cpu): bad argument");
    if (width > 0xffffffu || height > 0xffffffu) return set_error(CERES_EINVAL, "render (cpu): image too large");
    if (mode & CERES_MODE_QBVH4) return set_error(CERES_EUNSUPPORTED, "render (cpu): CERES_MODE_QBVH4 is a GPU mode");
    const int base = mode & ~(CERES_MODE_ROBUST | CERES_MODE_FMA);
    if (base != CERES_MODE_FULL && base != CERES_MODE_PRIMARY) return set_error(CERES_EINVAL, "render (cpu): bad mode %d", mode);
    const bool full = base == CERES_MODE_FULL, g = (mode & CERES_MODE_FMA) != 0, r = (mode & CERES_MODE_ROBUST) != 0;
    const auto t0 = std::chrono::steady_clock::now();
    Counts c;
    if (g && r) render_rows<true, true>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    else if (g) render_rows<true, false>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    else if (r) render_rows<false, true>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    else render_rows<false, false>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    if (c.overflow) return set_error(CERES_ESTACK, "render (cpu): traversal stack overflow");
    if (stats) {
        stats->rays = c.primary + c.shadow;
        stats->hits = c.hits;
        stats->primary_rays = c.primary;
        stats->shadow_rays = c.shadow;
        stats->node_pairs = c.steps;
        stats->tri_tests = c.tests;
        stats->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return CERES_OK;
}

}  // extern "C"
