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
#include <type_traits>
#include <vector>

#include <omp.h>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "pow24.hpp"

using namespace ceres;

struct ceres_cpu_scene {
    bool f64 = false;                 // render<double> (anim.cpp -d): the *64 arrays
    std::vector<SiblingPair> pairs;   // pair k: the two children of an inner node (pairs[0]: the root's)
    std::vector<Tri48> tris;          // leaf order
    std::vector<SiblingPair64> pairs64;
    std::vector<Tri96> tris64;
    std::vector<uint32_t> orig;       // leaf slot -> original triangle index (tri_norms order)
    std::vector<float> norms;         // 9 scalars per original triangle (obj_norms.hpp:113-115)
    std::vector<double> norms64;
    uint32_t depth = 0, root_leaf_count = 0, root_leaf_first = 0;
};

namespace {

// The scene's arrays for one Scalar.
template <class S> struct Arr;
template <> struct Arr<float> {
    static const std::vector<SiblingPair>& pairs(const ceres_cpu_scene& s) { return s.pairs; }
    static const std::vector<Tri48>& tris(const ceres_cpu_scene& s) { return s.tris; }
    static const float* norms(const ceres_cpu_scene& s) { return s.norms.data(); }
    static constexpr float eps = FLT_EPSILON, big = FLT_MAX;
};
template <> struct Arr<double> {
    static const std::vector<SiblingPair64>& pairs(const ceres_cpu_scene& s) { return s.pairs64; }
    static const std::vector<Tri96>& tris(const ceres_cpu_scene& s) { return s.tris64; }
    static const double* norms(const ceres_cpu_scene& s) { return s.norms64.data(); }
    static constexpr double eps = DBL_EPSILON, big = DBL_MAX;
};

template <class S> struct V3 { S x, y, z; };
template <class S> inline V3<S> operator+(V3<S> a, V3<S> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class S> inline V3<S> operator-(V3<S> a, V3<S> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class S> inline V3<S> operator*(V3<S> a, S s) { return {a.x * s, a.y * s, a.z * s}; }
template <class S> inline V3<S> v3(const S* p) { return {p[0], p[1], p[2]}; }

// vector.hpp:134-167 as each build computes it (see render_hip.hip dotA / dotB / crossG, render64.hip
// for double: GCC fuses the double path at the same sites): dot "A" fma(a2, b2, fma(a0, b0, a1 b1)),
// Triangle::intersect's v = dot(r, e1) as "B" fma(a2, b2, fma(a1, b1, a0 b0)), cross a_j b_k - a_k b_j
// as fma(a_j, b_k, -(a_k b_j)).
template <bool G, class S> inline S dot_a(V3<S> a, V3<S> b) {
    if constexpr (G) return std::fma(a.z, b.z, std::fma(a.x, b.x, a.y * b.y));
    S s = a.x * b.x; s += a.y * b.y; s += a.z * b.z;
    return s;
}
template <bool G, class S> inline S dot_b(V3<S> a, V3<S> b) {
    if constexpr (G) return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x));
    return dot_a<false>(a, b);
}
template <bool G, class S> inline V3<S> cross_g(V3<S> a, V3<S> b) {
    if constexpr (G) return {std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)), std::fma(a.x, b.y, -(a.y * b.x))};
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <bool G, class S> inline V3<S> normalize_g(V3<S> v) { const S inv = S(1) / std::sqrt(dot_a<G>(v, v)); return v * inv; }

// fminf / fmaxf (the non-NaN operand when one is NaN; the sign of a zero result is never observed:
// only comparisons read these values), written out so they inline instead of calling libm
template <class S> inline S min_nn(S x, S y) { return (x < y || std::isnan(y)) ? x : y; }
template <class S> inline S max_nn(S x, S y) { return (x > y || std::isnan(y)) ? x : y; }

// The slab constants of a ray and the test of one box (entry e, exit x; hit iff e <= x).
//   fast: inv = safe_inverse(d) (vector.hpp:69-74), s = -o inv, each slab fma(bound, inv, s); the
//         octant's near / far bound is min / max of the two fmas (fma is monotone in the bound);
//   robust (float scenes): inv = 1 / d, the exit slabs scaled by inv padded by 2 ulps
//         (utilities.hpp:102-106).
template <bool R, class S> struct SlabC { S ix, iy, iz, sx, sy, sz; V3<S> o; };
inline float pad2(float x) { uint32_t b; std::memcpy(&b, &x, 4); b += 2; float y; std::memcpy(&y, &b, 4); return std::isfinite(x) ? y : x; }
template <bool R, class S> inline SlabC<R, S> slab_of(V3<S> o, V3<S> d) {
    SlabC<R, S> s;
    if constexpr (R) {
        static_assert(std::is_same<S, float>::value, "robust slabs: float scenes");
        s.ix = 1.0f / d.x; s.iy = 1.0f / d.y; s.iz = 1.0f / d.z;
        s.sx = pad2(s.ix); s.sy = pad2(s.iy); s.sz = pad2(s.iz);
    } else {
        auto safe_inv = [](S x) { return S(1) / (std::fabs(x) < Arr<S>::eps ? std::copysign(Arr<S>::eps, x) : x); };
        s.ix = safe_inv(d.x); s.iy = safe_inv(d.y); s.iz = safe_inv(d.z);
        s.sx = (-o.x) * s.ix; s.sy = (-o.y) * s.iy; s.sz = (-o.z) * s.iz;
    }
    s.o = o;
    return s;
}
template <bool R, class S> inline bool box_hit(const SlabC<R, S>& s, const S* b, S tmin, S tmax, S& entry) {
    S e, x;                                       // b: xmin, xmax, ymin, ymax, zmin, zmax
    if constexpr (R) {
        const bool nx = std::signbit(s.ix), ny = std::signbit(s.iy), nz = std::signbit(s.iz);
        const S ex = ((nx ? b[1] : b[0]) - s.o.x) * s.ix, xx = ((nx ? b[0] : b[1]) - s.o.x) * s.sx;
        const S ey = ((ny ? b[3] : b[2]) - s.o.y) * s.iy, xy = ((ny ? b[2] : b[3]) - s.o.y) * s.sy;
        const S ez = ((nz ? b[5] : b[4]) - s.o.z) * s.iz, xz = ((nz ? b[4] : b[5]) - s.o.z) * s.sz;
        e = max_nn(ex, max_nn(ey, max_nn(ez, tmin)));
        x = min_nn(xx, min_nn(xy, min_nn(xz, tmax)));
    } else {
        const S a0 = std::fma(b[0], s.ix, s.sx), a1 = std::fma(b[1], s.ix, s.sx);
        const S b0 = std::fma(b[2], s.iy, s.sy), b1 = std::fma(b[3], s.iy, s.sy);
        const S c0 = std::fma(b[4], s.iz, s.sz), c1 = std::fma(b[5], s.iz, s.sz);
        e = max_nn(min_nn(a0, a1), max_nn(min_nn(b0, b1), max_nn(min_nn(c0, c1), tmin)));
        x = min_nn(max_nn(a0, a1), min_nn(max_nn(b0, b1), min_nn(max_nn(c0, c1), tmax)));
    }
    entry = e;
    return e <= x;
}

// Triangle::intersect (triangle.hpp:95-115): Moller-Trumbore, left-handed normal, IEEE 1 / det.
template <bool G, class S, class Tri> inline bool tri_hit(const Tri& tr, V3<S> o, V3<S> d, S tmin, S tmax, S& t_out, S& u_out,
                                                         S& v_out) {
    const V3<S> c = v3(tr.p0) - o;
    const V3<S> r = cross_g<G>(d, c);
    const S inv_det = S(1) / dot_a<G>(v3(tr.n), d);
    const S u = dot_a<G>(r, v3(tr.e2)) * inv_det;
    const S v = dot_b<G>(r, v3(tr.e1)) * inv_det;
    const S w = S(1) - u - v;
    if (u >= 0 && v >= 0 && w >= 0) {
        const S t = dot_a<G>(v3(tr.n), c) * inv_det;
        if (t >= tmin && t <= tmax) { t_out = t; u_out = u; v_out = v; return true; }
    }
    return false;
}

template <class S> struct HitRec { uint32_t slot; S t, u, v; };

// SingleRayTraverser::intersect (single_ray_traverser.hpp:68-126) with a closest-primitive
// intersector over the sibling-pair records: both children's boxes against the step's tmax, left
// leaf then right leaf in leaf order (each accepted hit lowers tmax, the last accepted one wins),
// the far child pushed, ties left.  steps / tests: the reference's Statistics.
template <bool G, bool R, class S>
bool trace_closest(const ceres_cpu_scene& s, V3<S> o, V3<S> d, uint32_t* stack, uint32_t cap, HitRec<S>& best, uint64_t& steps,
                   uint64_t& tests, bool& overflow) {
    const auto& pairs = Arr<S>::pairs(s);
    const auto& tris = Arr<S>::tris(s);
    const S tmin = 0;
    S tmax = Arr<S>::big;                                                   // ray.hpp:17-21
    bool have = false;
    auto leaf = [&](uint32_t first, uint32_t count) {                      // intersect_leaf, :43-63
        tests += count;
        for (uint32_t k = first; k < first + count; ++k) {
            S t, u, v;
            if (tri_hit<G>(tris[k], o, d, tmin, tmax, t, u, v)) { best = {k, t, u, v}; have = true; tmax = t; }
        }
    };
    if (s.root_leaf_count) {                                                // :72-73
        leaf(s.root_leaf_first, s.root_leaf_count);
        return have;
    }
    const SlabC<R, S> sl = slab_of<R>(o, d);
    uint32_t sp = 0, cur = 0;
    while (true) {
        ++steps;                                                            // :83
        const auto& p = pairs[cur];
        S el, er;
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
template <bool G, class S, class Tri> inline V3<S> hit_point(const Tri& tr, V3<S> normal, S hu, S hv) {
    const V3<S> p0 = v3(tr.p0), p1 = p0 - v3(tr.e1), p2 = p0 + v3(tr.e2);
    const S scale = -0.00001;
    const S w = 1 - hu - hv;
    if constexpr (G) {
        auto c = [&](S a, S q1, S q2, S n) { return std::fma(n, scale, std::fma(w, q2, std::fma(hv, q1, hu * a))); };
        return {c(p0.x, p1.x, p2.x, normal.x), c(p0.y, p1.y, p2.y, normal.y), c(p0.z, p1.z, p2.z, normal.z)};
    }
    const V3<S> p = p0 * hu + p1 * hv + p2 * w;
    return p + normal * scale;
}

// smooth_shading (render.hpp:46-84).  lambertian and blinn_phong_spec return float and
// std::pow(Scalar, 24) is the double pow narrowed to float (render.hpp:46-54): float scenes use
// pow24f (pinned against glibc for every float by tests/test_pow24.py), double scenes call the pow
// itself; the colour accumulates in float, `c[k] += w * clamp(...)` (double weights for double
// scenes: float(double + double), render64.hip).
template <bool G, class S> inline void shade(V3<S> sun_line, const S* nrm, V3<S> view, S u, S v, float c[3]) {
    c[0] = c[1] = c[2] = 0.0f;
    const float amb = 0.2;
    const V3<S> vneg = view * S(-1);
    const S w[3] = {u, v, 1 - u - v};
    for (int k = 0; k < 3; ++k) {
        const V3<S> N{nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]};
        const float lam = float(std::fabs(dot_a<G>(sun_line, N)));
        const S x = dot_a<G>(N, normalize_g<G>(sun_line + vneg));
        float p24;
        if constexpr (std::is_same<S, float>::value) p24 = pow24f(x);
        else p24 = float(std::pow(x, 24.0));
        const float spec = 0.8f * p24;
        const float base = G ? std::fma(lam, 0.5f, amb) : amb + 0.5f * lam;
        auto clamp01 = [](float y) { return (y < 0.f) ? 0.f : (1.f < y) ? 1.f : y; };   // std::clamp
        auto ch = [&](float k2) { return G ? std::fma(base, k2, spec) : base * k2 + spec; };
        for (int ch_i = 0; ch_i < 3; ++ch_i) {
            const float kk = ch_i == 0 ? 0.5f : ch_i == 1 ? 0.0f : 0.8f;
            if constexpr (std::is_same<S, float>::value) c[ch_i] += w[k] * clamp01(ch(kk));
            else c[ch_i] = float(double(c[ch_i]) + w[k] * double(clamp01(ch(kk))));
        }
    }
}

template <class S> inline uint8_t quantize(S x) {                          // static.cpp:141-143
    const S a = x * 255;
    const S m = (S(255) < a) ? S(255) : a;
    const S q = (m < S(0)) ? S(0) : m;
    return static_cast<uint8_t>(static_cast<int>(q));
}

struct Counts { uint64_t primary = 0, shadow = 0, hits = 0, steps = 0, tests = 0; bool overflow = false; };

template <bool G, bool R, class S>
void render_rows(const ceres_cpu_scene& s, const S* b12, const S* sun, bool full, S* pixels, uint8_t* rgb8,
                 size_t W, size_t H, int threads, Counts& tot) {
    const V3<S> eye = v3(b12), dir = v3(b12 + 3), iu = v3(b12 + 6), iv = v3(b12 + 9), sunp = v3(sun);
    const auto& tris = Arr<S>::tris(s);
    const S* norms = Arr<S>::norms(s);
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
                const S u = 2 * (S(i) + S(0.5)) / S(W) - S(1);
                const S v = 2 * (S(j) + S(0.5)) / S(H) - S(1);
                const V3<S> a = G ? V3<S>{dir.x + std::fma(iv.x, v, iu.x * u), dir.y + std::fma(iv.y, v, iu.y * u),
                                          dir.z + std::fma(iv.z, v, iu.z * u)}
                                  : iu * u + iv * v + dir;
                const V3<S> view = normalize_g<G>(a);
                HitRec<S> h{0, 0, 0, 0};
                ++primary;
                S c[3] = {0, 0, 0};                                          // a miss: render.hpp:116-117
                if (trace_closest<G, R>(s, eye, view, stack.data(), cap, h, steps, tests, ov)) {
                    ++hits;
                    const auto& tr = tris[h.slot];
                    const V3<S> normal = normalize_g<G>(v3(tr.n));
                    if (!full) {                                             // render.hpp:123-125 (primary only)
                        c[0] = std::fabs(normal.x); c[1] = std::fabs(normal.y); c[2] = std::fabs(normal.z);
                    } else {
                        const V3<S> p = hit_point<G>(tr, normal, h.u, h.v);
                        const V3<S> sun_line = normalize_g<G>(sunp - p);     // render.hpp:135
                        HitRec<S> hs{0, 0, 0, 0};
                        ++shadow;
                        if (trace_closest<G, R>(s, p, sun_line, stack.data(), cap, hs, steps, tests, ov)) {
                            ++hits;                                          // render.hpp:146-149: occluded, RGB 0
                        } else {
                            float col[3];
                            shade<G>(sun_line, norms + 9 * size_t(s.orig[h.slot]), view, h.u, h.v, col);
                            c[0] = col[0]; c[1] = col[1]; c[2] = col[2];
                        }
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

template <class S>
int render_cpu(const ceres_cpu_scene* scene, const S* basis12, const S* sun, int mode, S* pixels, uint8_t* rgb8, size_t width,
               size_t height, ceres_stats* stats, int threads) {
    if (!scene || !basis12 || !sun || width == 0 || height == 0) return set_error(CERES_EINVAL, "render (cpu): bad argument");
    if (scene->f64 != std::is_same<S, double>::value)
        return set_error(CERES_EINVAL, "render (cpu): the scene is %s precision", scene->f64 ? "double" : "single");
    if (width > 0xffffffu || height > 0xffffffu) return set_error(CERES_EINVAL, "render (cpu): image too large");
    if (mode & CERES_MODE_QBVH4) return set_error(CERES_EUNSUPPORTED, "render (cpu): CERES_MODE_QBVH4 is a GPU mode");
    if (scene->f64 && (mode & CERES_MODE_ROBUST))
        return set_error(CERES_EUNSUPPORTED, "render (cpu): CERES_MODE_ROBUST takes float scenes");
    const int base = mode & ~(CERES_MODE_ROBUST | CERES_MODE_FMA);
    if (base != CERES_MODE_FULL && base != CERES_MODE_PRIMARY) return set_error(CERES_EINVAL, "render (cpu): bad mode %d", mode);
    const bool full = base == CERES_MODE_FULL, g = (mode & CERES_MODE_FMA) != 0, r = (mode & CERES_MODE_ROBUST) != 0;
    const auto t0 = std::chrono::steady_clock::now();
    Counts c;
    if constexpr (std::is_same<S, float>::value) {
        if (g && r) render_rows<true, true, S>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
        else if (r) render_rows<false, true, S>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    }
    if (!r) {
        if (g) render_rows<true, false, S>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
        else render_rows<false, false, S>(*scene, basis12, sun, full, pixels, rgb8, width, height, threads, c);
    }
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

ceres_cpu_scene* ceres_cpu_scene_create_f64(const double* tri96, size_t n_tri, const double* norm72, const void* nodes64,
                                            size_t n_nodes, const uint64_t* prim64) {
    if (!tri96 || !norm72 || !nodes64 || !prim64 || n_tri == 0 || n_nodes == 0) {
        set_error(CERES_EINVAL, "ceres_cpu_scene_create_f64: empty scene or null argument");
        return nullptr;
    }
    if (n_tri > 0xffffffffull || n_nodes > 0xffffffffull) { set_error(CERES_EUNSUPPORTED, "scene too large"); return nullptr; }
    auto* s = new (std::nothrow) ceres_cpu_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    s->f64 = true;
    try {
        if (relayout_bvh64(static_cast<const RefNode64*>(nodes64), n_nodes, prim64, n_tri, reinterpret_cast<const Tri96*>(tri96),
                           s->pairs64, s->tris64, s->orig, s->depth, s->root_leaf_count, s->root_leaf_first)) {
            delete s;
            return nullptr;
        }
        s->norms64.assign(norm72, norm72 + 9 * n_tri);
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
    return render_cpu<float>(scene, basis12, sun, mode, pixels, rgb8, width, height, stats, threads);
}

int ceres_render_cpu_f64(const ceres_cpu_scene* scene, const double basis12[12], const double sun[3], int mode,
                         double* pixels, uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats, int threads) {
    return render_cpu<double>(scene, basis12, sun, mode, pixels, rgb8, width, height, stats, threads);
}

}  // extern "C"
