// render64.hip -- render<double> (render.hpp:86-156 with Scalar = double; anim.cpp's -d mode,
// anim.cpp:146-155) on gfx950.
//
// The double instantiation keeps the reference's mixed precision exactly: camera basis, rays,
// BVH2 traversal (FastNodeIntersector with a true fma, node_intersectors.hpp:35-47,83-103),
// Moller-Trumbore (triangle.hpp:95-115), hit point, offset and shadow ray in double; the
// shading helpers return float (render.hpp:46-54: lambertian / blinn_phong_spec are declared
// `float`, std::pow(double, int) is a double pow narrowed to float) and smooth_shading
// accumulates `c[k] += u * clamp(...)` as float = float(double + double) (render.hpp:56-84); the
// pixel is the float colour widened to double and quantised in double (static.cpp:141-143).
//
// One kernel, one lane per pixel, 8x8 tiles per wavefront: primary closest-hit traversal in
// the reference's order, then the any-hit shadow ray over the same BVH2 (only the boolean is
// used, render.hpp:139), shading, store.  Records are double-width (112-B sibling pairs, 96-B
// triangles); the stack is u32 in LDS like the float path.  Built without FP contraction;
// IEEE double division and sqrt are correctly rounded on gfx950.
//
// CERES_MODE_FMA (kG = true, round 5): the reference's own CMake build of anim.cpp -d (g++ -O3
// -mavx2 -mfma, CMakeLists.txt:11) fuses the double hot path at the same sites as the float one
// -- GCC's widening_mul dump of the double harness lists the same (file, line, column, FMA kind)
// multiset for render()'s pixel loop, smooth_shading and blinn_phong_spec
// (oracle/contraction_sites.txt) -- so the kernel carries an explicit fma at each: dotA / dotB,
// cross with the first product fused, the primary direction dir + fma(iv, v, iu u), the hit point
// fma(n, -1e-5, fma(w, p2, fma(v, p1, u p0))), lambertian as dotA in double, and the float
// fmaf(lam, 0.5, amb) / fmaf(base, k, spec) of smooth_shading.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "pow24.hpp"
#include "scene_internal.hpp"

#pragma clang fp contract(off)

namespace ceres {
namespace dev64 {

#ifndef CERES64_WG
#define CERES64_WG 64            // workgroup: 64 = one 8x8 tile (a long tile pins only its own LDS), 256 = 16x16
#endif
#ifndef CERES_LANE_QUADS64
#define CERES_LANE_QUADS64 0     // lanes in Morton order over the 8x8 tile (else row-major)
#endif
constexpr int kBlock = CERES64_WG;
constexpr uint32_t kTile = kBlock == 256 ? 16u : 8u;

struct D3 { double x, y, z; };
__device__ __forceinline__ D3 operator+(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ D3 operator-(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ D3 operator*(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ D3 operator*(double s, D3 a) { return {s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ double dot(D3 a, D3 b) { double s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
__device__ __forceinline__ D3 cross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ __forceinline__ D3 normalize(D3 v) { const double inv = 1.0 / sqrt(dot(v, v)); return v * inv; }
__device__ __forceinline__ D3 d3(const double* p) { return {p[0], p[1], p[2]}; }
// GCC's contraction of vector.hpp:134-167 in the reference-flag build (kG; oracle/contraction_sites.txt)
template <bool kG> __device__ __forceinline__ double dotA(D3 a, D3 b) {
    if constexpr (kG) return fma(a.z, b.z, fma(a.x, b.x, a.y * b.y));
    else return dot(a, b);
}
template <bool kG> __device__ __forceinline__ double dotB(D3 a, D3 b) {
    if constexpr (kG) return fma(a.z, b.z, fma(a.y, b.y, a.x * b.x));
    else return dot(a, b);
}
template <bool kG> __device__ __forceinline__ D3 crossG(D3 a, D3 b) {
    if constexpr (kG) return {fma(a.y, b.z, -(a.z * b.y)), fma(a.z, b.x, -(a.x * b.z)), fma(a.x, b.y, -(a.y * b.x))};
    else return cross(a, b);
}
template <bool kG> __device__ __forceinline__ D3 normalizeG(D3 v) { const double inv = 1.0 / sqrt(dotA<kG>(v, v)); return v * inv; }

struct Cam64 { double eye[3], dir[3], iu[3], iv[3], sun[3]; };

struct KParams64 {
    Cam64 cam;
    uint32_t W, H;
    uint32_t stack_entries, root_leaf_count, root_leaf_first;
    const SiblingPair64* pairs;
    const Tri96* tris;
    const uint32_t* orig;
    const double* norms;
    double* pixels;          // 3*W*H, row 0 at the bottom (render.hpp:107)
    uint8_t* rgb8;           // PPM body, rows top-down
    Shard* shards;
    int32_t* rec_prim;       // optional per-pixel records, pixel = j*W + i
    double* rec_tuv;
    int8_t* rec_shadow;
    const uint32_t* tile_order;  // block -> tile, centre first and XCD-balanced (frame_tile_order)
    uint32_t tiles_x;
};

struct TriD { D3 p0, e1, e2, n; };
__device__ __forceinline__ TriD load_tri(const Tri96* t) {
    const double2* q = reinterpret_cast<const double2*>(t);
    const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5];
    return {{a.x, a.y, b.x}, {b.y, c.x, c.y}, {d.x, d.y, e.x}, {e.y, f.x, f.y}};
}

// Triangle<double>::intersect (triangle.hpp:95-115)
template <bool kG>
__device__ __forceinline__ bool tri_test(const TriD& tr, D3 o, D3 d, double tmin, double tmax, double& t_out, double& u_out,
                                         double& v_out) {
    const D3 c = tr.p0 - o;
    const D3 r = crossG<kG>(d, c);
    const double inv_det = 1.0 / dotA<kG>(tr.n, d);
    const double u = dotA<kG>(r, tr.e2) * inv_det;
    const double v = dotB<kG>(r, tr.e1) * inv_det;
    const double w = 1.0 - u - v;
    if (u >= 0 && v >= 0 && w >= 0) {
        const double t = dotA<kG>(tr.n, c) * inv_det;
        if (t >= tmin && t <= tmax) { t_out = t; u_out = u; v_out = v; return true; }
    }
    return false;
}

struct Hit { uint32_t slot; double t, u, v; };

// single_ray_traverser.hpp:68-126 in double (the float trace() of render_hip.hip: the same
// visiting order, octant-free monotone slab test, near-first ties left; any-hit returns at the
// first accepted triangle).
template <bool kAnyHit, bool kG>
__device__ bool trace(const KParams64& P, D3 o, D3 d, uint32_t* stk, Hit& best, bool& overflow) {
    const double tmin = 0.0;
    double tmax = DBL_MAX;                                          // ray.hpp:17-21
    bool have = false;
    if (P.root_leaf_count) {
        for (uint32_t k = P.root_leaf_first; k < P.root_leaf_first + P.root_leaf_count; ++k) {
            double t, u, v;
            if (tri_test<kG>(load_tri(P.tris + k), o, d, tmin, tmax, t, u, v)) {
                best = {k, t, u, v}; have = true;
                if (kAnyHit) return true;
                tmax = t;
            }
        }
        return have;
    }
    auto safe_inv = [](double x) { return 1.0 / (fabs(x) < DBL_EPSILON ? copysign(DBL_EPSILON, x) : x); };   // vector.hpp:69-74
    const double ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
    const double sx = (-o.x) * ix, sy = (-o.y) * iy, sz = (-o.z) * iz;
    uint32_t sp = 0, cur = 0;
    while (true) {
        const double2* q = reinterpret_cast<const double2*>(P.pairs + cur);
        const double2 A = q[0], B = q[1], C = q[2], D = q[3], E = q[4], F = q[5];
        const uint4 L = reinterpret_cast<const uint4*>(q)[6];
        const double l0 = fma(A.x, ix, sx), l1 = fma(A.y, ix, sx);
        const double l2 = fma(B.x, iy, sy), l3 = fma(B.y, iy, sy);
        const double l4 = fma(C.x, iz, sz), l5 = fma(C.y, iz, sz);
        const double r0 = fma(D.x, ix, sx), r1 = fma(D.y, ix, sx);
        const double r2 = fma(E.x, iy, sy), r3 = fma(E.y, iy, sy);
        const double r4 = fma(F.x, iz, sz), r5 = fma(F.y, iz, sz);
        const double le = fmax(fmin(l0, l1), fmax(fmin(l2, l3), fmax(fmin(l4, l5), tmin)));
        const double lx = fmin(fmax(l0, l1), fmin(fmax(l2, l3), fmin(fmax(l4, l5), tmax)));
        const double re = fmax(fmin(r0, r1), fmax(fmin(r2, r3), fmax(fmin(r4, r5), tmin)));
        const double rx = fmin(fmax(r0, r1), fmin(fmax(r2, r3), fmin(fmax(r4, r5), tmax)));
        const bool hit_l = le <= lx, hit_r = re <= rx;
        uint32_t k = 0, k_end = 0, k2 = 0, k2_end = 0;
        if (hit_l && L.x) { k = L.y; k_end = L.y + L.x; }
        if (hit_r && L.z) { k2 = L.w; k2_end = L.w + L.z; }
        while (k < k_end || k2 < k2_end) {
            const uint32_t idx = k < k_end ? k++ : k2++;
            double t, u, v;
            if (tri_test<kG>(load_tri(P.tris + idx), o, d, tmin, tmax, t, u, v)) {
                best = {idx, t, u, v}; have = true;
                if (kAnyHit) return true;
                tmax = t;
            }
        }
        const bool go_l = hit_l && !L.x, go_r = hit_r && !L.z;
        if (go_l && go_r) {
            const bool swap = le > re;
            if (sp >= P.stack_entries) { overflow = true; return have; }
            stk[sp * kBlock] = swap ? L.y : L.w;
            ++sp;
            cur = swap ? L.w : L.y;
        } else if (go_l || go_r) {
            cur = go_l ? L.y : L.w;
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * kBlock];
        }
    }
    return have;
}

// (float)std::pow(x, 24) for a double x: x^24 in double-double, rounded to double (the
// correctly rounded pow), then narrowed to float as blinn_phong_spec's return type does.
__device__ __forceinline__ float pow24_from_double(double x) {
    if (!(fabs(x) <= 1e12)) return isnan(x) ? float(x) : INFINITY;   // |x|^24 overflows float long before
    double h2 = x * x, l2 = fma(x, x, -h2);
    double h4, l4, h8, l8, h16, l16, h24, l24;
    dd_square(h2, l2, h4, l4);
    dd_square(h4, l4, h8, l8);
    dd_square(h8, l8, h16, l16);
    dd_mul(h16, l16, h8, l8, h24, l24);
    return float(h24 + l24);
}

// smooth_shading<double> (render.hpp:46-84): float helpers, double weights, float accumulators
template <bool kG>
__device__ __forceinline__ void shade(D3 sun_line, const double* nrm, D3 view, double u, double v, float c[3]) {
    c[0] = c[1] = c[2] = 0.0f;
    const float amb = 0.2;
    const D3 vneg = view * -1.0;
    const double w[3] = {u, v, 1 - u - v};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const D3 N{nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]};
        const float lam = float(fabs(kG ? dotA<true>(sun_line, N) : sun_line.x * N.x + sun_line.y * N.y + sun_line.z * N.z));   // lambertian
        const float spec = 0.8f * pow24_from_double(dotA<kG>(N, normalizeG<kG>(sun_line + vneg)));  // blinn_phong_spec
        const float base = kG ? __builtin_fmaf(lam, 0.5f, amb) : amb + 0.5f * lam;
        auto clamp01 = [](float x) { return (x < 0.f) ? 0.f : (1.f < x) ? 1.f : x; };          // std::clamp
        auto ch = [&](float k) { return kG ? __builtin_fmaf(base, k, spec) : base * k + spec; };
        c[0] = float(double(c[0]) + w[k] * double(clamp01(ch(0.5f))));
        c[1] = float(double(c[1]) + w[k] * double(clamp01(ch(0.0f))));
        c[2] = float(double(c[2]) + w[k] * double(clamp01(ch(0.8f))));
    }
}

__device__ __forceinline__ uint8_t quantize(double x) {              // static.cpp:141-143 with Scalar = double
    const double a = x * 255;
    const double m = (255.0 < a) ? 255.0 : a;
    const double q = (m < 0.0) ? 0.0 : m;
    return static_cast<uint8_t>(static_cast<int>(q));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// 1-D grid over the frame's kTile x kTile tiles in tile_order (as the float path: expensive tiles
// first, every XCD an unbiased share); each wavefront an 8x8 tile (of its workgroup's 16x16
// pixels when kBlock = 256)
template <int kMode, bool kG>
__global__ __launch_bounds__(kBlock) void ceres_render64(const KParams64 P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t* stk = lds + tid;
    const uint32_t t = __builtin_amdgcn_readfirstlane(P.tile_order[blockIdx.x]);
    const uint32_t tby = t / P.tiles_x, tbx = t - tby * P.tiles_x;
#if CERES_LANE_QUADS64
    // lanes in Morton order over the wavefront's 8x8 tile (quads = 2x2 pixel blocks)
    const uint32_t lx = (lane & 1u) | ((lane >> 1) & 2u) | ((lane >> 2) & 4u), ly = ((lane >> 1) & 1u) | ((lane >> 2) & 2u) | ((lane >> 3) & 4u);
#else
    const uint32_t lx = lane & 7u, ly = lane >> 3;
#endif
    const uint32_t i = tbx * kTile + (kBlock == 256 ? (wave & 1u) * 8u : 0u) + lx;
    const uint32_t j = tby * kTile + (kBlock == 256 ? (wave >> 1) * 8u : 0u) + ly;
    const bool valid = i < P.W && j < P.H;
    bool overflow = false;
    uint32_t n_hit = 0, n_shadow = 0, n_occ = 0;
    if (valid) {
        const Cam64& c = P.cam;
        // render.hpp:109-113
        const double u = 2 * (double(i) + 0.5) / double(P.W) - 1.0;
        const double v = 2 * (double(j) + 0.5) / double(P.H) - 1.0;
        D3 a;
        if constexpr (kG)                                            // GCC: dir + fma(iv, v, iu u)
            a = D3{c.dir[0] + fma(c.iv[0], v, c.iu[0] * u), c.dir[1] + fma(c.iv[1], v, c.iu[1] * u),
                   c.dir[2] + fma(c.iv[2], v, c.iu[2] * u)};
        else a = d3(c.iu) * u + d3(c.iv) * v + d3(c.dir);
        const D3 view = normalizeG<kG>(a);
        Hit h{};
        const bool hit = trace<false, kG>(P, d3(c.eye), view, stk, h, overflow);
        double px[3] = {0.0, 0.0, 0.0};
        int8_t shadow_rec = -1;
        if (hit) {
            n_hit = 1;
            const TriD tri = load_tri(P.tris + h.slot);
            const D3 normal = normalizeG<kG>(tri.n);
            if (kMode == CERES_MODE_PRIMARY) {                        // render.hpp:123-125
                px[0] = fabs(normal.x); px[1] = fabs(normal.y); px[2] = fabs(normal.z);
            } else {
                const D3 p1 = tri.p0 - tri.e1, p2 = tri.p0 + tri.e2;   // p1(), p2()
                const double scale = -0.00001;
                D3 p;
                if constexpr (kG) {                                  // GCC: fma(n, scale, fma(w, p2, fma(v, p1, u p0)))
                    const double w = 1 - h.u - h.v;
                    auto cp = [&](double a0, double q1, double q2, double n) { return fma(n, scale, fma(w, q2, fma(h.v, q1, h.u * a0))); };
                    p = D3{cp(tri.p0.x, p1.x, p2.x, normal.x), cp(tri.p0.y, p1.y, p2.y, normal.y), cp(tri.p0.z, p1.z, p2.z, normal.z)};
                } else {
                    p = h.u * tri.p0 + h.v * p1 + (1 - h.u - h.v) * p2;   // render.hpp:129 (permuted weights)
                    p = p + scale * normal;
                }
                const D3 sun_line = normalizeG<kG>(d3(c.sun) - p);     // render.hpp:135
                Hit h2;
                n_shadow = 1;
                const bool blocked = trace<true, kG>(P, p, sun_line, stk, h2, overflow);
                shadow_rec = blocked ? 1 : 0;
                if (blocked) {
                    n_occ = 1;
                } else {
                    float col[3];
                    shade<kG>(sun_line, P.norms + 9 * size_t(P.orig[h.slot]), view, h.u, h.v, col);
                    px[0] = col[0]; px[1] = col[1]; px[2] = col[2];
                }
            }
        }
        const size_t pix = size_t(j) * P.W + i;
        if (P.pixels) { double* q = P.pixels + 3 * pix; q[0] = px[0]; q[1] = px[1]; q[2] = px[2]; }
        if (P.rgb8) {
            uint8_t* q = P.rgb8 + 3 * (size_t(P.H - 1 - j) * P.W + i);
            q[0] = quantize(px[0]); q[1] = quantize(px[1]); q[2] = quantize(px[2]);
        }
        if (P.rec_prim) {
            P.rec_prim[pix] = hit ? int32_t(P.orig[h.slot]) : -1;
            P.rec_tuv[3 * pix] = hit ? h.t : 0.0; P.rec_tuv[3 * pix + 1] = hit ? h.u : 0.0; P.rec_tuv[3 * pix + 2] = hit ? h.v : 0.0;
            P.rec_shadow[pix] = shadow_rec;
        }
    }
    const uint32_t wh = wave_sum(n_hit + n_occ), ws = wave_sum(n_shadow);
    const uint32_t shard = blockIdx.x * (kBlock / 64) + wave;
    if (lane == 0) {
        Shard& sh = P.shards[shard % kShards];
        if (ws) atomicAdd(&sh.queued, ws);
        if (wh) atomicAdd(&sh.hits, (unsigned long long)wh);
    }
    if (__ballot(overflow) && lane == 0) atomicOr(&P.shards[shard % kShards].error, 1u);
}

}  // namespace dev64
}  // namespace ceres

using namespace ceres;
using namespace ceres::dev64;

namespace {

#define HIP64_TRY(expr)                                                                       \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return set_error(CERES_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <typename T>
void dfree64(T*& p) { if (p) { (void)hipFree(p); p = nullptr; } }

// one render into device buffers; counters summed from the shards on the host
int render64(ceres_scene* s, const double basis12[12], const double sun[3], int mode, size_t W, size_t H, double* d_px,
             uint8_t* d_rgb, int32_t* d_prim, double* d_tuv, int8_t* d_sh, ceres_stats* st) {
    if (!s || !basis12 || !sun) return set_error(CERES_EINVAL, "ceres_render_f64: null argument");
    if (!s->f64) return set_error(CERES_EINVAL, "scene is single precision: use ceres_render_f32");
    const bool gfma = (mode & CERES_MODE_FMA) != 0;                 // the reference CMake build's FMA contraction
    mode &= ~CERES_MODE_FMA;
    if (mode != CERES_MODE_FULL && mode != CERES_MODE_PRIMARY) return set_error(CERES_EINVAL, "bad mode %d", mode);
    if (W == 0 || H == 0 || W > 65535u * kTile || H > 65535u * kTile) return set_error(CERES_EINVAL, "bad frame size %zux%zu", W, H);
    HIP64_TRY(hipSetDevice(s->device));
    KParams64 P{};
    std::memcpy(P.cam.eye, basis12, 3 * sizeof(double));
    std::memcpy(P.cam.dir, basis12 + 3, 3 * sizeof(double));
    std::memcpy(P.cam.iu, basis12 + 6, 3 * sizeof(double));
    std::memcpy(P.cam.iv, basis12 + 9, 3 * sizeof(double));
    std::memcpy(P.cam.sun, sun, 3 * sizeof(double));
    P.W = uint32_t(W); P.H = uint32_t(H);
    P.stack_entries = s->stack_entries;
    P.root_leaf_count = s->root_leaf_count; P.root_leaf_first = s->root_leaf_first;
    P.pairs = s->d_pairs64; P.tris = s->d_tris64; P.orig = s->d_orig; P.norms = s->d_norms64;
    P.pixels = d_px; P.rgb8 = d_rgb; P.shards = s->d_shards;
    P.rec_prim = d_prim; P.rec_tuv = d_tuv; P.rec_shadow = d_sh;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP64_TRY(hipEventCreate(&e0));
    HIP64_TRY(hipEventCreate(&e1));
    HIP64_TRY(hipMemsetAsync(s->d_shards, 0, sizeof(Shard) * kShards, s->stream));
    s->shards_dirty = true;
    const uint32_t tx = (uint32_t(W) + kTile - 1) / kTile, ty = (uint32_t(H) + kTile - 1) / kTile;
    if (int rc = frame_tile_order(s, W, H, kTile, s->stream, &P.tile_order)) return rc;
    P.tiles_x = tx;
    const dim3 grid(tx * ty), block(kBlock);
    const size_t lds = size_t(s->stack_entries) * kBlock * 4;
    HIP64_TRY(hipEventRecord(e0, s->stream));
    if (mode == CERES_MODE_PRIMARY && gfma) hipLaunchKernelGGL((ceres_render64<CERES_MODE_PRIMARY, true>), grid, block, lds, s->stream, P);
    else if (mode == CERES_MODE_PRIMARY) hipLaunchKernelGGL((ceres_render64<CERES_MODE_PRIMARY, false>), grid, block, lds, s->stream, P);
    else if (gfma) hipLaunchKernelGGL((ceres_render64<CERES_MODE_FULL, true>), grid, block, lds, s->stream, P);
    else hipLaunchKernelGGL((ceres_render64<CERES_MODE_FULL, false>), grid, block, lds, s->stream, P);
    HIP64_TRY(hipGetLastError());
    HIP64_TRY(hipEventRecord(e1, s->stream));
    std::vector<Shard> sh(kShards);
    HIP64_TRY(hipMemcpyAsync(sh.data(), s->d_shards, sizeof(Shard) * kShards, hipMemcpyDeviceToHost, s->stream));
    HIP64_TRY(hipStreamSynchronize(s->stream));
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    uint64_t shadow = 0, hits = 0;
    uint32_t err = 0;
    for (const Shard& x : sh) { shadow += x.queued; hits += x.hits; err |= x.error; }
    if (st) {
        st->primary_rays = uint64_t(W) * H; st->shadow_rays = shadow;
        st->rays = st->primary_rays + shadow; st->hits = hits;
        st->node_pairs = st->tri_tests = 0; st->ms = ms;
    }
    if (err) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

}  // namespace

extern "C" {

// Scene for render<double>: the reference's own double arrays (Triangle<double>[], tri_norms,
// Bvh<double> nodes + primitive_indices), re-laid as double sibling pairs in depth-first order.
ceres_scene* ceres_scene_create_f64(const double* tri96, size_t n_tri, const double* norm72, const void* nodes64,
                                    size_t n_nodes, const uint64_t* prim64, int device, uint32_t flags) {
    if (!tri96 || !norm72 || !nodes64 || !prim64 || n_tri == 0 || n_nodes == 0) {
        set_error(CERES_EINVAL, "ceres_scene_create_f64: empty scene or null argument");
        return nullptr;
    }
    if (n_tri > 0xffffffffull || n_nodes > 0xffffffffull) { set_error(CERES_EUNSUPPORTED, "scene too large"); return nullptr; }
    std::vector<SiblingPair64> pairs;
    std::vector<Tri96> leaf;
    std::vector<uint32_t> orig;
    uint32_t depth = 0, rlc = 0, rlf = 0;
    if (relayout_bvh64(static_cast<const RefNode64*>(nodes64), n_nodes, prim64, n_tri, reinterpret_cast<const Tri96*>(tri96),
                       pairs, leaf, orig, depth, rlc, rlf))
        return nullptr;
    auto* s = new (std::nothrow) ceres_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    s->f64 = true;
    s->device = device; s->flags = flags; s->n_tri = n_tri; s->n_pairs = pairs.size();
    s->depth = depth; s->root_leaf_count = rlc; s->root_leaf_first = rlf;
    s->stack_entries = std::max<uint32_t>(1, depth);
    auto fail = [&]() -> ceres_scene* { scene_release(s); delete s; return nullptr; };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { set_error(CERES_EHIP, "no HIP device available"); return fail(); }
    if (device < 0 || device >= ndev) { set_error(CERES_EINVAL, "device %d out of range (%d devices)", device, ndev); return fail(); }
    auto body = [&]() -> int {
        HIP64_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIP64_TRY(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_error(CERES_EHIP, "device %d is %s, this build targets gfx950 only", device, prop.gcnArchName);
        s->num_cus = prop.multiProcessorCount;
        HIP64_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        HIP64_TRY(hipMalloc(&s->d_pairs64, pairs.size() * sizeof(SiblingPair64)));
        HIP64_TRY(hipMalloc(&s->d_tris64, n_tri * sizeof(Tri96)));
        HIP64_TRY(hipMalloc(&s->d_orig, n_tri * sizeof(uint32_t)));
        HIP64_TRY(hipMalloc(&s->d_norms64, n_tri * 72));
        HIP64_TRY(hipMalloc(&s->d_shards, sizeof(Shard) * kShards));
        HIP64_TRY(hipMemcpy(s->d_pairs64, pairs.data(), pairs.size() * sizeof(SiblingPair64), hipMemcpyHostToDevice));
        HIP64_TRY(hipMemcpy(s->d_tris64, leaf.data(), n_tri * sizeof(Tri96), hipMemcpyHostToDevice));
        HIP64_TRY(hipMemcpy(s->d_orig, orig.data(), n_tri * sizeof(uint32_t), hipMemcpyHostToDevice));
        HIP64_TRY(hipMemcpy(s->d_norms64, norm72, n_tri * 72, hipMemcpyHostToDevice));
        return CERES_OK;
    };
    if (body()) return fail();
    return s;
}

// render<double>() with host buffers (render.hpp:86-156, Scalar = double): pixels (3*W*H
// doubles, bottom row first) and/or the RGB8 PPM body; rays/hits in stats.
int ceres_render_f64(ceres_scene* s, const double basis12[12], const double sun[3], int mode, double* pixels,
                     uint8_t* rgb8, size_t W, size_t H, ceres_stats* stats) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    HIP64_TRY(hipSetDevice(s->device));
    const size_t n = W * H;
    double* dp = nullptr;
    uint8_t* dr = nullptr;
    auto cleanup = [&] { dfree64(dp); dfree64(dr); };
    if ((pixels && hipMalloc(&dp, n * 24) != hipSuccess) || (rgb8 && hipMalloc(&dr, n * 3) != hipSuccess)) {
        cleanup();
        return set_error(CERES_ENOMEM, "ceres_render_f64: device allocation failed");
    }
    int rc = render64(s, basis12, sun, mode, W, H, dp, dr, nullptr, nullptr, nullptr, stats);
    if (!rc && ((pixels && hipMemcpy(pixels, dp, n * 24, hipMemcpyDeviceToHost) != hipSuccess) ||
                (rgb8 && hipMemcpy(rgb8, dr, n * 3, hipMemcpyDeviceToHost) != hipSuccess)))
        rc = set_error(CERES_EHIP, "ceres_render_f64: copy back failed");
    cleanup();
    return rc;
}

// Per-pixel hit records of render<double> (pixel = j*W + i): original triangle (-1 on a miss),
// t / u / v (double), shadow (-1 none, 0 lit, 1 occluded).
int ceres_render_records_f64(ceres_scene* s, const double basis12[12], const double sun[3], int mode, size_t W, size_t H,
                             int32_t* prim, double* tuv, int8_t* shadow, ceres_stats* stats) {
    if (!s || !prim || !tuv || !shadow) return set_error(CERES_EINVAL, "ceres_render_records_f64: null argument");
    HIP64_TRY(hipSetDevice(s->device));
    const size_t n = W * H;
    int32_t* dp = nullptr;
    double* dt = nullptr;
    int8_t* ds = nullptr;
    auto cleanup = [&] { dfree64(dp); dfree64(dt); dfree64(ds); };
    if (hipMalloc(&dp, n * 4) != hipSuccess || hipMalloc(&dt, n * 24) != hipSuccess || hipMalloc(&ds, n) != hipSuccess) {
        cleanup();
        return set_error(CERES_ENOMEM, "ceres_render_records_f64: device allocation failed");
    }
    int rc = render64(s, basis12, sun, mode, W, H, nullptr, nullptr, dp, dt, ds, stats);
    if (!rc && (hipMemcpy(prim, dp, n * 4, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(tuv, dt, n * 24, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(shadow, ds, n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = set_error(CERES_EHIP, "ceres_render_records_f64: copy back failed");
    cleanup();
    return rc;
}

}  // extern "C"
