// render_hip.hip -- the CERES hot path as hand-written HIP for gfx950 (MI355X) + its C ABI.
//
// Replaces render<float>() of include/render.hpp:86-156 (iracigt/ceres-raytracer): per-pixel
// primary rays (render.hpp:105-113), BVH2 traversal (single_ray_traverser.hpp:68-126) with the
// fast slab test (node_intersectors.hpp:35-47,83-103), Moller-Trumbore (triangle.hpp:95-115),
// the offset shadow ray (render.hpp:119-138) and smooth Blinn-Phong shading (render.hpp:46-84),
// plus the PPM quantiser of static.cpp:135-147.
//
// Two kernels per frame (DESIGN.md "Kernels"):
//   ceres_primary  one lane per pixel, 8x8 pixel tile per wavefront (coherent primary rays),
//                  closest-hit traversal; misses / primary-only pixels are written directly;
//                  hits are COMPACTED into a sharded shadow-ray queue with a wave __ballot +
//                  popcount prefix (one atomic per workgroup), so no lane idles on pixels
//                  that missed while other lanes trace 28-node-pair shadow rays.
//   ceres_shadow   one lane per queued shadow ray (dense waves), any-hit traversal (only the
//                  boolean matters, render.hpp:139 -- result-identical to the reference's
//                  closest-hit with tmax = FLT_MAX), then smooth shading of lit pixels.
// The traversal stack lives in LDS ([entries][threads], lane-contiguous = bank-conflict
// free), sized from the BVH depth at scene creation (<= 63 entries for max_depth 64).
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32 div/sqrt, explicit
// fmaf only where the reference calls fast_multiply_add, std::pow in double -- so every
// float matches the reference compiled without contraction bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "pow24.hpp"

#pragma clang fp contract(off)


namespace ceres {

char* error_buffer() {
    static thread_local char buf[kErrorBufferSize] = "";
    return buf;
}

namespace dev {

constexpr int kBlock = 256;            // 4 wavefronts of 64 lanes
constexpr int kWaves = kBlock / 64;

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(F3 a, F3 b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
__device__ __forceinline__ F3 cross(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ __forceinline__ F3 normalize(F3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
__device__ __forceinline__ float rmax(float x, float y) { return x > y ? x : y; }   // robust_max, utilities.hpp:57-67
__device__ __forceinline__ float rmin(float x, float y) { return x < y ? x : y; }

struct TriV { F3 p0, e1, e2, n; };
__device__ __forceinline__ TriV load_tri(const Tri48* t) {
    const float4* q = reinterpret_cast<const float4*>(t);
    const float4 a = q[0], b = q[1], c = q[2];
    return {{a.x, a.y, a.z}, {a.w, b.x, b.y}, {b.z, b.w, c.x}, {c.y, c.z, c.w}};
}

// Per-ray traversal state; the hit is "last accepted wins" like intersect_leaf (:54-60).
struct Hit { uint32_t slot; float t, u, v; };

// Triangle::intersect (triangle.hpp:95-115, left-handed normal): on an accepted hit updates
// best / tmax (closest hit keeps the LAST accepted hit with t <= tmax, intersect_leaf :54-60).
__device__ __forceinline__ bool tri_test(const TriV& tr, F3 o, F3 d, float tmin, float tmax, float& t_out,
                                         float& u_out, float& v_out) {
    const F3 c = tr.p0 - o;
    const F3 r = cross(d, c);
    const float inv_det = 1.0f / dot(tr.n, d);
    const float u = dot(r, tr.e2) * inv_det;
    const float v = dot(r, tr.e1) * inv_det;
    const float w = 1.0f - u - v;
    if (u >= 0 && v >= 0 && w >= 0) {
        const float t = dot(tr.n, c) * inv_det;
        if (t >= tmin && t <= tmax) { t_out = t; u_out = u; v_out = v; return true; }
    }
    return false;
}

// Eager BVH2 traversal, single_ray_traverser.hpp:68-126 with FastNodeIntersector
// (node_intersectors.hpp:35-47,83-103).  Exactly the reference's visiting order: both
// children's slab tests use the tmax from before this step's leaves; left leaf triangles,
// then right leaf triangles, are tested in leaf order; the far child is pushed, ties go left.
//
// Slab test restatement: the reference picks the entry/exit bound per axis by the ray octant
// and evaluates fma(bound, inv, -o*inv).  fma is monotone in `bound`, so for inv >= 0 (octant
// 0, including d = +0 -> inv = +1/eps) fma(min) <= fma(max) and for inv < 0 (d = -0 included)
// the reverse: the octant-selected entry is min(fma(lo), fma(hi)) and the exit is the max,
// bit for bit, without per-ray selects.  robust_max(x, y) = x > y ? x : y equals fmaxf(x, y)
// whenever y is not NaN (y is tmin / tmax / a previous robust_max -- never NaN) up to the
// sign of zero, which no comparison below can observe; likewise robust_min and fminf.  The
// slab values themselves are finite for |coordinates| < 4e31 (|inv| <= 1/FLT_EPSILON).
// Diagnostic section clocks (stats builds only): wave-uniform s_memtime sums per trace().
struct Stamps { unsigned long long box = 0, leaf = 0, next = 0, iters = 0; };
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

template <bool kAnyHit, bool kStats, int kStride = kBlock, bool kPF = false>
__device__ __forceinline__ bool trace(const KParams& P, F3 o, F3 d, uint32_t* stk, Hit& best,
                                      uint32_t& n_pairs, uint32_t& n_tests, bool& overflow, Stamps* ss = nullptr) {
    const float tmin = 0.0f;
    float tmax = FLT_MAX;                                           // ray.hpp:17-21
    bool have = false;
    if (P.root_leaf_count) {                                          // root is a leaf, :72-73
        if (kStats) n_tests += P.root_leaf_count;
        for (uint32_t k = P.root_leaf_first; k < P.root_leaf_first + P.root_leaf_count; ++k) {
            float t, u, v;
            if (tri_test(load_tri(P.tris + k), o, d, tmin, tmax, t, u, v)) {
                best = {k, t, u, v}; have = true;
                if (kAnyHit) return true;
                tmax = t;
            }
        }
        return have;
    }
    auto safe_inv = [](float x) { return 1.0f / (fabsf(x) < FLT_EPSILON ? copysignf(FLT_EPSILON, x) : x); };   // vector.hpp:69-74
    const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
    const float sx = (-o.x) * ix, sy = (-o.y) * iy, sz = (-o.z) * iz;
    uint32_t sp = 0;
    uint32_t cur = 0;                                                 // pair of the root's children (:81)
    unsigned long long c0 = 0, c1 = 0, c2 = 0;
    while (true) {                                                    // :82-123
        if (kStats) ++n_pairs;
        if (kStats && ss) c0 = stamp();
        const float4* q = reinterpret_cast<const float4*>(P.pairs + cur);
        const float4 A = q[0], B = q[1], C = q[2];
        const uint4 L = reinterpret_cast<const uint4*>(q)[3];
        // left bounds A.x A.y | A.z A.w | B.x B.y ; right bounds B.z B.w | C.x C.y | C.z C.w
        const float l0 = __builtin_fmaf(A.x, ix, sx), l1 = __builtin_fmaf(A.y, ix, sx);
        const float l2 = __builtin_fmaf(A.z, iy, sy), l3 = __builtin_fmaf(A.w, iy, sy);
        const float l4 = __builtin_fmaf(B.x, iz, sz), l5 = __builtin_fmaf(B.y, iz, sz);
        const float r0 = __builtin_fmaf(B.z, ix, sx), r1 = __builtin_fmaf(B.w, ix, sx);
        const float r2 = __builtin_fmaf(C.x, iy, sy), r3 = __builtin_fmaf(C.y, iy, sy);
        const float r4 = __builtin_fmaf(C.z, iz, sz), r5 = __builtin_fmaf(C.w, iz, sz);
        const float le = fmaxf(fminf(l0, l1), fmaxf(fminf(l2, l3), fmaxf(fminf(l4, l5), tmin)));
        const float lx = fminf(fmaxf(l0, l1), fminf(fmaxf(l2, l3), fminf(fmaxf(l4, l5), tmax)));
        const float re = fmaxf(fminf(r0, r1), fmaxf(fminf(r2, r3), fmaxf(fminf(r4, r5), tmin)));
        const float rx = fminf(fmaxf(r0, r1), fminf(fmaxf(r2, r3), fminf(fmaxf(r4, r5), tmax)));
        const bool hit_l = le <= lx, hit_r = re <= rx;
        if (kStats && ss) { volatile bool keep = hit_l | hit_r; (void)keep; c1 = stamp(); }
        // leaves of this step, left then right (intersect_leaf on each, :89-107), one loop so a
        // wavefront runs max(left + right) trips rather than max(left) + max(right)
        uint32_t k = 0, k_end = 0, k2 = 0, k2_end = 0;
        if (hit_l && L.x) { k = L.y; k_end = L.y + L.x; }
        if (hit_r && L.z) { k2 = L.w; k2_end = L.w + L.z; }
        if (kStats) n_tests += (k_end - k) + (k2_end - k2);
        while (k < k_end || k2 < k2_end) {
            const uint32_t idx = k < k_end ? k++ : k2++;
            float t, u, v;
            if (tri_test(load_tri(P.tris + idx), o, d, tmin, tmax, t, u, v)) {
                best = {idx, t, u, v}; have = true;
                if (kAnyHit) { if (kStats && ss) { ss->box += c1 - c0; ss->iters++; } return true; }
                tmax = t;
            }
        }
        if (kStats && ss) { c2 = stamp(); ss->box += c1 - c0; ss->leaf += c2 - c1; ss->iters++; }
        const bool go_l = hit_l && !L.x, go_r = hit_r && !L.z;
        if (go_l && go_r) {                                           // near first, ties left (:109-115)
            const bool swap = le > re;
            if (sp >= P.stack_entries) { overflow = true; return have; }
            stk[sp * kStride] = swap ? L.y : L.w;
            ++sp;
            cur = swap ? L.w : L.y;
        } else if (go_l || go_r) {
            cur = go_l ? L.y : L.w;                                   // :115-117
        } else {
            if (sp == 0) { if (kStats && ss) ss->next += stamp() - c2; break; }   // :118-121
            --sp;
            cur = stk[sp * kStride];
        }
        if (kStats && ss) ss->next += stamp() - c2;
    }
    return have;
}

__device__ __forceinline__ uint8_t quantize(float x) {               // static.cpp:141-143
    const float a = x * 255;
    const float m = (255.0f < a) ? 255.0f : a;                       // std::min(a, 255)
    const float q = (m < 0.0f) ? 0.0f : m;                           // std::max(m, 0)
    return static_cast<uint8_t>(static_cast<int>(q));
}

__device__ __forceinline__ void store_pixel(const KParams& P, uint32_t lr, uint32_t i, float c0, float c1, float c2) {
    if (P.pixels) {
        float* q = P.pixels + 3 * (size_t(lr) * P.W + i);
        q[0] = c0; q[1] = c1; q[2] = c2;
    }
    if (P.rgb8) {
        uint8_t* q = P.rgb8 + 3 * (size_t(P.local_rows - 1 - lr) * P.W + i);
        q[0] = quantize(c0); q[1] = quantize(c1); q[2] = quantize(c2);
    }
}

__device__ __forceinline__ uint32_t global_row(const KParams& P, uint32_t lr) {
    return ((lr / P.row_block) * P.world + P.rank) * P.row_block + lr % P.row_block;
}

// Primary ray direction of pixel (i, j), render.hpp:109-111.
__device__ __forceinline__ F3 primary_dir(const KParams& P, uint32_t i, uint32_t j) {
    const float u = 2 * (float(i) + 0.5f) / float(P.W) - 1.0f;
    const float v = 2 * (float(j) + 0.5f) / float(P.H) - 1.0f;
    const F3 iu{P.iu[0], P.iu[1], P.iu[2]}, iv{P.iv[0], P.iv[1], P.iv[2]}, dir{P.dir[0], P.dir[1], P.dir[2]};
    return normalize(iu * u + iv * v + dir);
}

// smooth_shading, render.hpp:46-84 (pow in double: std::pow(float, int) promotes).
__device__ __forceinline__ void shade(F3 sun_line, const float* nrm, F3 view, float u, float v, float c[3]) {
    c[0] = c[1] = c[2] = 0.0f;
    const float amb = 0.2;
    const F3 vneg = view * -1.0f;
    const float w[3] = {u, v, 1 - u - v};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const F3 N{nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]};
        const float diffuse = 0.5f * fabsf(sun_line.x * N.x + sun_line.y * N.y + sun_line.z * N.z);
        const float spec = 0.8f * pow24f(dot(N, normalize(sun_line + vneg)));   // == (float)std::pow(double, 24)
        const float base = amb + diffuse;
        auto clamp01 = [](float x) { return (x < 0.f) ? 0.f : (1.f < x) ? 1.f : x; };   // std::clamp
        c[0] += w[k] * clamp01(base * 0.5f + spec);
        c[1] += w[k] * clamp01(base * 0.0f + spec);
        c[2] += w[k] * clamp01(base * 0.8f + spec);
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// ---------------------------------------------------------------- primary kernel
// kBS threads per workgroup (64: one 8x8 tile per workgroup; 256: 16x16 pixels as 2x2 wave
// tiles).  Every wavefront is independent: no workgroup barrier, one queue atomic per wave.
template <int kMode, bool kStats, int kBS, bool kPF>
__device__ __forceinline__ void primary_tile(const KParams& P, uint32_t* stk, uint32_t lane, uint32_t wave_id,
                                             uint32_t i, uint32_t lr) {
    const bool active = i < P.W && lr < P.local_rows;
    bool hit = false, job = false;
    Hit h{0, 0.f, 0.f, 0.f};
    uint32_t n_pairs = 0, n_tests = 0;
    bool overflow = false;
    F3 shadow_o{0.f, 0.f, 0.f};
    if (active) {
        const uint32_t j = global_row(P, lr);
        const F3 eye{P.eye[0], P.eye[1], P.eye[2]};
        const F3 view = primary_dir(P, i, j);
        hit = trace<false, kStats, kBS, kPF>(P, eye, view, stk, h, n_pairs, n_tests, overflow);
        if (P.rec_prim) {
            const size_t px = size_t(lr) * P.W + i;
            P.rec_prim[px] = hit ? int32_t(P.orig[h.slot]) : -1;
            P.rec_tuv[3 * px] = hit ? h.t : 0.f; P.rec_tuv[3 * px + 1] = hit ? h.u : 0.f; P.rec_tuv[3 * px + 2] = hit ? h.v : 0.f;
            P.rec_shadow[px] = -1;
        }
        if (!hit) {
            store_pixel(P, lr, i, 0.f, 0.f, 0.f);                    // render.hpp:116-117
        } else {
            const TriV tr = load_tri(P.tris + h.slot);
            const F3 normal = normalize(tr.n);
            if (kMode == CERES_MODE_PRIMARY) {                       // render.hpp:123-125
                store_pixel(P, lr, i, fabsf(normal.x), fabsf(normal.y), fabsf(normal.z));
            } else {                                                 // render.hpp:127-133
                const F3 p1 = tr.p0 - tr.e1, p2 = tr.p0 + tr.e2;
                F3 p = tr.p0 * h.u + p1 * h.v + p2 * (1 - h.u - h.v);
                const float scale = -0.00001;
                p = p + normal * scale;
                shadow_o = p;
                job = true;
            }
        }
    }
    // wave-level compaction of the shadow rays: ballot + popcount prefix, one atomic per wave
    const uint32_t shard = wave_id % kShards;
    const unsigned long long jm = __ballot(job);
    const uint32_t nh = __popcll(__ballot(hit));
    uint32_t base = 0;
    if (lane == 0) {
        if (jm) base = atomicAdd(&P.shards[shard].queued, uint32_t(__popcll(jm)));
        if (nh) atomicAdd(&P.shards[shard].hits, (unsigned long long)nh);
    }
    if (jm) {
        base = __shfl(base, 0, 64);
        if (job) {
            const uint32_t off = base + __popcll(jm & ((1ull << lane) - 1ull));
            float4* q = reinterpret_cast<float4*>(P.jobs + size_t(shard) * P.shard_capacity + off);
            q[0] = make_float4(__uint_as_float(lr * P.W + i), __uint_as_float(h.slot), h.u, h.v);
            q[1] = make_float4(shadow_o.x, shadow_o.y, shadow_o.z, 0.f);
        }
    }
    if (kStats) {
        const uint32_t wp = wave_sum(n_pairs), wt = wave_sum(n_tests);
        if (lane == 0) {
            atomicAdd(&P.shards[shard].pairs, (unsigned long long)wp);
            atomicAdd(&P.shards[shard].tests, (unsigned long long)wt);
        }
    }
    if (overflow) atomicOr(&P.shards[shard].error, 1u);
}


template <int kMode, bool kStats, int kBS, bool kPF>
__global__ __launch_bounds__(kBS) void ceres_primary(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* stk = lds + tid;                                       // [entries][kBS]
    if (kBS == 64) {
        // one wavefront per workgroup; tiles_per_wave 8x8 tiles, interleaved over the grid
        const uint32_t n_tiles = P.tiles_x * P.tiles_y;
        for (uint32_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
            const uint32_t ty = t / P.tiles_x, tx = t - ty * P.tiles_x;
            primary_tile<kMode, kStats, kBS, kPF>(P, stk, lane, t, tx * 8 + (lane & 7), ty * 8 + (lane >> 3));
        }
    } else {
        const uint32_t i = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
        const uint32_t lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
        primary_tile<kMode, kStats, kBS, kPF>(P, stk, lane, (blockIdx.y * gridDim.x + blockIdx.x) * (kBS / 64) + wave, i, lr);
    }
}

// ---------------------------------------------------------------- shadow kernel
template <bool kStats, int kBS, bool kPF>
__global__ __launch_bounds__(kBS) void ceres_shadow(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* stk = lds + tid;
    // per-shard job prefix, read by every wave from the shard counters (scalar loads)
    uint32_t pre[kShards + 1];
    pre[0] = 0;
#pragma unroll
    for (int s = 0; s < kShards; ++s) pre[s + 1] = pre[s] + __builtin_amdgcn_readfirstlane(P.shards[s].queued);
    const uint32_t total = pre[kShards];
    const F3 sun{P.sun[0], P.sun[1], P.sun[2]};
    uint32_t occluded = 0, n_pairs = 0, n_tests = 0;
    bool overflow = false;
    unsigned long long t_begin = 0;
    Stamps stamps;
    if (kStats) t_begin = __builtin_amdgcn_s_memrealtime();
    for (uint32_t g = blockIdx.x * kBS + tid; g < total; g += gridDim.x * kBS) {
        uint32_t s = 0;                                              // shard holding global job g
#pragma unroll
        for (uint32_t step = 16; step > 0; step >>= 1)
            if (pre[s + step] <= g) s += step;
        const float4* q = reinterpret_cast<const float4*>(P.jobs + size_t(s) * P.shard_capacity + (g - pre[s]));
        const float4 J0 = q[0], J1 = q[1];
        const uint32_t pix = __float_as_uint(J0.x), slot = __float_as_uint(J0.y);
        const float hu = J0.z, hv = J0.w;
        const F3 o{J1.x, J1.y, J1.z};
        const F3 sun_line = normalize(sun - o);                      // render.hpp:135
        Hit h2{0, 0.f, 0.f, 0.f};
        const bool blocked = trace<true, kStats, kBS, kPF>(P, o, sun_line, stk, h2, n_pairs, n_tests, overflow,
                                                           kStats ? &stamps : nullptr);
        const uint32_t lr = pix / P.W, i = pix - lr * P.W;
        if (P.rec_shadow) P.rec_shadow[pix] = blocked ? 1 : 0;
        if (blocked) {                                               // render.hpp:147-150
            ++occluded;
            store_pixel(P, lr, i, 0.f, 0.f, 0.f);
        } else {                                                     // render.hpp:139-146
            const F3 view = primary_dir(P, i, global_row(P, lr));
            float c[3];
            shade(sun_line, P.norms + 9 * size_t(P.orig[slot]), view, hu, hv, c);
            store_pixel(P, lr, i, c[0], c[1], c[2]);
        }
    }
    const uint32_t wo = wave_sum(occluded);
    const uint32_t shard = (blockIdx.x * (kBS / 64) + wave) % kShards;
    if (lane == 0 && wo) atomicAdd(&P.shards[shard].hits, (unsigned long long)wo);
    if (kStats) {
        const uint32_t wp = wave_sum(n_pairs), wt = wave_sum(n_tests);
        uint32_t mp = n_pairs;                                       // max chain in the wave
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mp = max(mp, __shfl_xor(mp, off, 64));
        if (lane == 0) {
            atomicAdd(&P.shards[shard].pairs, (unsigned long long)wp);
            atomicAdd(&P.shards[shard].tests, (unsigned long long)wt);
            if (P.wave_log) {                                        // diagnostic wave timeline
                unsigned long long* w = P.wave_log + 8 * size_t(blockIdx.x * (kBS / 64) + wave);
                uint32_t xcc = 0, hw = 0;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                w[0] = t_begin; w[1] = __builtin_amdgcn_s_memrealtime(); w[2] = mp; w[3] = stamps.iters;
                w[4] = stamps.box; w[5] = stamps.leaf; w[6] = stamps.next; w[7] = wp;
            }
        }
    }
    if (overflow) atomicOr(&P.shards[shard].error, 1u);
}

// ---------------------------------------------------------------- persistent frame kernel
// One launch per frame.  Each wavefront is an independent worker with a private LDS region:
//   [stack: entries x 64 lanes][shadow-ray queue: 7 x 128 words (pixel, slot, u, v, px, py, pz)]
// Loop: fetch a chunk of 8x8 tiles (dynamic, sharded counters); trace the tile's primary rays
// (one pixel per lane, closest hit); write misses; COMPACT the hits' shadow rays into the
// wave's LDS queue with __ballot + popcount prefix; whenever >= 64 are queued, trace a FULL
// wavefront of shadow rays (any-hit) and shade them.  The queue is flushed when the work runs
// out.  No global queue, no block barriers, no second launch; shadow rays stay coherent
// (they come from the same tiles) and waves stay dense.
constexpr int kFrameBlock = 128;          // 2 independent wavefronts per workgroup
constexpr int kQueue = 128;               // shadow-ray queue capacity per wavefront
constexpr int kQueueWords = 7 * kQueue;
constexpr int kChunkTiles = 2;            // tiles per dynamic fetch
constexpr int kTileShards = 16;           // tile counters (bands of the tile grid)

__device__ __forceinline__ uint32_t band_begin(uint32_t s, uint32_t n_chunks) {
    return uint32_t((uint64_t(n_chunks) * s) / kTileShards);
}

// Lane 0 claims the next chunk: its own band first, then the others (skipping drained ones).
__device__ __forceinline__ uint32_t fetch_chunk(const KParams& P, uint32_t home, uint32_t lane) {
    uint32_t got = 0xffffffffu;
    if (lane == 0) {
        uint32_t dead = __hip_atomic_load(&P.shards[0].exhausted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t k = 0; k < kTileShards; ++k) {
            const uint32_t s = (home + k) % kTileShards;
            if (dead & (1u << s)) continue;
            const uint32_t b0 = band_begin(s, P.n_chunks), b1 = band_begin(s + 1, P.n_chunks);
            const uint32_t v = atomicAdd(&P.shards[s].tiles, 1u);
            if (v < b1 - b0) { got = b0 + v; break; }
            atomicOr(&P.shards[0].exhausted, 1u << s);
        }
    }
    return __builtin_amdgcn_readfirstlane(__shfl(got, 0, 64));
}

template <bool kStats>
__device__ __forceinline__ void shade_queued(const KParams& P, uint32_t* q, uint32_t base, uint32_t count,
                                             uint32_t lane, uint32_t* stk, uint32_t& occluded, uint32_t& traced,
                                             uint32_t& n_pairs, uint32_t& n_tests, bool& overflow) {
    if (lane >= count) return;
    const uint32_t e = base + lane;
    const uint32_t pix = q[e], slot = q[kQueue + e];
    const float hu = __uint_as_float(q[2 * kQueue + e]), hv = __uint_as_float(q[3 * kQueue + e]);
    const F3 o{__uint_as_float(q[4 * kQueue + e]), __uint_as_float(q[5 * kQueue + e]), __uint_as_float(q[6 * kQueue + e])};
    const F3 sun{P.sun[0], P.sun[1], P.sun[2]};
    const F3 sun_line = normalize(sun - o);                          // render.hpp:135
    Hit h2{0, 0.f, 0.f, 0.f};
    const bool blocked = trace<true, kStats, 64>(P, o, sun_line, stk, h2, n_pairs, n_tests, overflow);
    ++traced;
    const uint32_t lr = pix / P.W, i = pix - lr * P.W;
    if (P.rec_shadow) P.rec_shadow[pix] = blocked ? 1 : 0;
    if (blocked) {                                                   // render.hpp:147-150
        ++occluded;
        store_pixel(P, lr, i, 0.f, 0.f, 0.f);
    } else {                                                         // render.hpp:139-146
        const F3 view = primary_dir(P, i, global_row(P, lr));
        float c[3];
        shade(sun_line, P.norms + 9 * size_t(P.orig[slot]), view, hu, hv, c);
        store_pixel(P, lr, i, c[0], c[1], c[2]);
    }
}

template <int kMode, bool kStats>
__global__ __launch_bounds__(kFrameBlock) void ceres_frame(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63, wslot = threadIdx.x >> 6;
    const uint32_t per_wave = P.stack_entries * 64 + kQueueWords;
    uint32_t* base = lds + wslot * per_wave;
    uint32_t* stk = base + lane;                                     // entry k of this lane at stk[k * 64]
    uint32_t* q = base + P.stack_entries * 64;
    const uint32_t wave_id = blockIdx.x * (kFrameBlock / 64) + wslot;
    const uint32_t home = wave_id % kTileShards;
    const F3 eye{P.eye[0], P.eye[1], P.eye[2]};
    uint32_t qn = 0;                                                 // queued shadow rays (wave-uniform)
    uint32_t hits = 0, occluded = 0, traced = 0, n_pairs = 0, n_tests = 0;
    bool overflow = false;
    // diagnostic stamps (stats build only): wall clock (100 MHz) + shader-clock fetch time
    unsigned long long t_begin = 0, fetch_clk = 0, n_chunk = 0, n_batch = 0;
    if (kStats) t_begin = __builtin_amdgcn_s_memrealtime();
    auto fetch = [&]() {
        unsigned long long c0 = 0;
        if (kStats) c0 = __builtin_amdgcn_s_memtime();
        const uint32_t r = fetch_chunk(P, home, lane);
        if (kStats) { fetch_clk += __builtin_amdgcn_s_memtime() - c0; ++n_chunk; }
        return r;
    };
    for (uint32_t chunk = fetch(); chunk < P.n_chunks; chunk = fetch()) {
#pragma unroll 1
        for (uint32_t t = chunk * kChunkTiles; t < (chunk + 1) * kChunkTiles && t < P.tiles_x * P.tiles_y; ++t) {
            const uint32_t ty = t / P.tiles_x, tx = t - ty * P.tiles_x;
            const uint32_t i = tx * 8 + (lane & 7), lr = ty * 8 + (lane >> 3);
            bool job = false;
            Hit h{0, 0.f, 0.f, 0.f};
            F3 so{0.f, 0.f, 0.f};
            if (i < P.W && lr < P.local_rows) {
                const F3 view = primary_dir(P, i, global_row(P, lr));
                const bool hit = trace<false, kStats, 64>(P, eye, view, stk, h, n_pairs, n_tests, overflow);
                if (P.rec_prim) {
                    const size_t px = size_t(lr) * P.W + i;
                    P.rec_prim[px] = hit ? int32_t(P.orig[h.slot]) : -1;
                    P.rec_tuv[3 * px] = hit ? h.t : 0.f; P.rec_tuv[3 * px + 1] = hit ? h.u : 0.f; P.rec_tuv[3 * px + 2] = hit ? h.v : 0.f;
                    P.rec_shadow[px] = -1;
                }
                if (!hit) {
                    store_pixel(P, lr, i, 0.f, 0.f, 0.f);            // render.hpp:116-117
                } else {
                    ++hits;
                    const TriV tr = load_tri(P.tris + h.slot);
                    const F3 normal = normalize(tr.n);
                    if (kMode == CERES_MODE_PRIMARY) {               // render.hpp:123-125
                        store_pixel(P, lr, i, fabsf(normal.x), fabsf(normal.y), fabsf(normal.z));
                    } else {                                         // render.hpp:127-133
                        const F3 p1 = tr.p0 - tr.e1, p2 = tr.p0 + tr.e2;
                        F3 p = tr.p0 * h.u + p1 * h.v + p2 * (1 - h.u - h.v);
                        const float scale = -0.00001;
                        so = p + normal * scale;
                        job = true;
                    }
                }
            }
            if (kMode == CERES_MODE_FULL) {
                const unsigned long long m = __ballot(job);
                if (job) {                                           // append to the wave's LDS queue
                    const uint32_t e = qn + __popcll(m & ((1ull << lane) - 1ull));
                    q[e] = lr * P.W + i; q[kQueue + e] = h.slot;
                    q[2 * kQueue + e] = __float_as_uint(h.u); q[3 * kQueue + e] = __float_as_uint(h.v);
                    q[4 * kQueue + e] = __float_as_uint(so.x); q[5 * kQueue + e] = __float_as_uint(so.y);
                    q[6 * kQueue + e] = __float_as_uint(so.z);
                }
                qn += __popcll(m);
                __builtin_amdgcn_wave_barrier();
                if (qn >= 64) {                                      // a full wavefront of shadow rays
                    qn -= 64;
                    if (kStats) ++n_batch;
                    shade_queued<kStats>(P, q, qn, 64, lane, stk, occluded, traced, n_pairs, n_tests, overflow);
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
    }
    if (kMode == CERES_MODE_FULL && qn > 0)
        shade_queued<kStats>(P, q, 0, qn, lane, stk, occluded, traced, n_pairs, n_tests, overflow);
    // one set of counter atomics per wavefront
    const uint32_t wh = wave_sum(hits + occluded), wq = wave_sum(traced);
    const uint32_t shard = wave_id % kShards;
    if (lane == 0) {
        if (wh) atomicAdd(&P.shards[shard].hits, (unsigned long long)wh);
        if (wq) atomicAdd(&P.shards[shard].queued, wq);
    }
    if (kStats) {
        const uint32_t wp = wave_sum(n_pairs), wt = wave_sum(n_tests);
        if (lane == 0) {
            atomicAdd(&P.shards[shard].pairs, (unsigned long long)wp);
            atomicAdd(&P.shards[shard].tests, (unsigned long long)wt);
            if (P.wave_log) {
                unsigned long long* w = P.wave_log + 8 * size_t(wave_id);
                uint32_t xcc = 0, hw = 0;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                w[0] = t_begin; w[1] = __builtin_amdgcn_s_memrealtime(); w[2] = n_chunk; w[3] = n_batch;
                w[4] = fetch_clk; w[5] = wp; w[6] = (unsigned long long)xcc << 32 | hw; w[7] = wave_sum(traced);
            }
        }
    }
    if (overflow) atomicOr(&P.shards[shard].error, 1u);
}

// ---------------------------------------------------------------- counters
__global__ void ceres_finalize(const Shard* shards, uint64_t primary_rays, uint64_t* out) {
    if (threadIdx.x != 0) return;
    unsigned long long q = 0, h = 0, p = 0, t = 0;
    uint32_t err = 0;
    for (int s = 0; s < kShards; ++s) { q += shards[s].queued; h += shards[s].hits; p += shards[s].pairs; t += shards[s].tests; err |= shards[s].error; }
    out[0] = primary_rays + q; out[1] = h; out[2] = primary_rays; out[3] = q;
    out[4] = p; out[5] = t; out[6] = err; out[7] = 0;
}

}  // namespace dev
}  // namespace ceres

// =====================================================================================
// host side: scene upload + launch glue (C ABI)
// =====================================================================================
using namespace ceres;

struct ceres_scene {
    int device = 0;
    uint32_t flags = 0;
    size_t n_tri = 0, n_pairs = 0;
    uint32_t depth = 0, stack_entries = 1, root_leaf_count = 0, root_leaf_first = 0;
    SiblingPair* d_pairs = nullptr;
    Tri48* d_tris = nullptr;
    uint32_t* d_orig = nullptr;
    float* d_norms = nullptr;
    Shard* d_shards = nullptr;
    uint64_t* d_counters = nullptr;
    ShadowJob* d_jobs = nullptr;
    size_t jobs_cap = 0;
    float* d_pixels = nullptr;
    uint8_t* d_rgb8 = nullptr;
    size_t px_cap = 0;
    hipStream_t stream = nullptr;
    int num_cus = 256;
    unsigned long long* d_wave_log = nullptr;   // stats scenes: per-wave diagnostic records
    size_t wave_log_waves = 0, last_grid_waves = 0;
    int variant = 0;                   // kVariantTwoPass (default); kVariantWave / kVariantFrame via CERES_KERNEL
    int frame_blocks_per_cu[4] = {0, 0, 0, 0};
    uint32_t tiles_per_wave = 1;       // primary kernel (wave variant): 8x8 tiles per wavefront
    bool pf_primary = false, pf_shadow = false; // (reserved variant bit, currently identical code)
    // optional per-kernel device timing (bench.py roofline leg)
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<hipEvent_t> ev_used;   // triples: start, after primary, after shadow
};

namespace {

constexpr int kVariantTwoPass = 0, kVariantWave = 1, kVariantFrame = 2;

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return set_error(CERES_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <typename T>
void dfree(T*& p) { if (p) { (void)hipFree(p); p = nullptr; } }

void scene_release(ceres_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    dfree(s->d_pairs); dfree(s->d_tris); dfree(s->d_orig); dfree(s->d_norms);
    dfree(s->d_shards); dfree(s->d_counters); dfree(s->d_wave_log); dfree(s->d_jobs); dfree(s->d_pixels); dfree(s->d_rgb8);
    for (auto e : s->ev_pool) (void)hipEventDestroy(e);
    for (auto e : s->ev_used) if (e) (void)hipEventDestroy(e);
    s->ev_pool.clear(); s->ev_used.clear();
    if (s->stream) (void)hipStreamDestroy(s->stream);
    s->stream = nullptr;
}

size_t local_rows_of(size_t H, uint32_t rb, uint32_t rank, uint32_t world) {
    const size_t nblocks = (H + rb - 1) / rb;
    size_t rows = 0;
    for (size_t b = rank; b < nblocks; b += world) rows += std::min<size_t>(rb, H - b * rb);
    return rows;
}

// Re-lay the reference BVH (nodes32 + prim64) as depth-first SiblingPair records and the
// triangles in leaf order.  Validates the structure (ranges, cycles) on the way.
int relayout(const RefNode* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri48* tris,
             std::vector<SiblingPair>& pairs, std::vector<Tri48>& leaf_tris, std::vector<uint32_t>& orig,
             uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first) {
    leaf_tris.resize(n_tri);
    orig.resize(n_tri);
    for (size_t k = 0; k < n_tri; ++k) {
        if (prim[k] >= n_tri) return set_error(CERES_EINVAL, "primitive_indices[%zu] = %llu out of range", k, (unsigned long long)prim[k]);
        leaf_tris[k] = tris[prim[k]];
        orig[k] = uint32_t(prim[k]);
    }
    auto check_leaf = [&](const RefNode& n) -> bool {
        return size_t(n.first_child_or_primitive) + n.primitive_count <= n_tri;
    };
    depth = 0;
    root_leaf_count = root_leaf_first = 0;
    if (nodes[0].primitive_count) {
        if (!check_leaf(nodes[0])) return set_error(CERES_EINVAL, "root leaf range out of bounds");
        root_leaf_count = nodes[0].primitive_count;
        root_leaf_first = nodes[0].first_child_or_primitive;
        pairs.assign(1, SiblingPair{});
        return CERES_OK;
    }
    // pre-order DFS over inner nodes; each inner node's children become one record
    struct Item { uint32_t node, pair, level; };
    pairs.clear();
    pairs.reserve(n_nodes / 2 + 1);
    std::vector<Item> st;
    if (size_t(nodes[0].first_child_or_primitive) + 1 >= n_nodes) return set_error(CERES_EINVAL, "root child index out of range");
    pairs.emplace_back();
    st.push_back({0, 0, 1});
    size_t visited = 0;
    while (!st.empty()) {
        const Item it = st.back(); st.pop_back();
        if (++visited > n_nodes) return set_error(CERES_EINVAL, "BVH has a cycle");
        const RefNode& n = nodes[it.node];
        const uint32_t c = n.first_child_or_primitive;
        depth = std::max(depth, it.level);
        SiblingPair& rec = pairs[it.pair];
        std::memcpy(rec.lb, nodes[c].bounds, 24);
        std::memcpy(rec.rb, nodes[c + 1].bounds, 24);
        const RefNode* ch[2] = {&nodes[c], &nodes[c + 1]};
        uint32_t cnt[2], first[2];
        Item push[2]; int npush = 0;
        for (int k = 0; k < 2; ++k) {
            cnt[k] = ch[k]->primitive_count;
            if (cnt[k]) {
                if (!check_leaf(*ch[k])) return set_error(CERES_EINVAL, "leaf range out of bounds");
                first[k] = ch[k]->first_child_or_primitive;
            } else {
                const uint32_t gc = ch[k]->first_child_or_primitive;
                if (size_t(gc) + 1 >= n_nodes) return set_error(CERES_EINVAL, "child index out of range");
                first[k] = uint32_t(pairs.size());
                pairs.emplace_back();
                push[npush++] = {c + uint32_t(k), first[k], it.level + 1};
            }
        }
        SiblingPair& r2 = pairs[it.pair];                            // (emplace_back may have moved rec)
        r2.lcount = cnt[0]; r2.lfirst = first[0];
        r2.rcount = cnt[1]; r2.rfirst = first[1];
        for (int k = npush - 1; k >= 0; --k) st.push_back(push[k]);   // left subtree first
    }
    return CERES_OK;
}

int ensure_workspace(ceres_scene* s, size_t jobs, size_t px, bool want_px, bool want_rgb) {
    if (jobs > s->jobs_cap) {
        dfree(s->d_jobs);
        HIP_TRY(hipMalloc(&s->d_jobs, jobs * sizeof(ShadowJob)));
        s->jobs_cap = jobs;
    }
    if ((want_px || want_rgb) && px > s->px_cap) {
        dfree(s->d_pixels); dfree(s->d_rgb8);
        HIP_TRY(hipMalloc(&s->d_pixels, px * 3 * sizeof(float)));
        HIP_TRY(hipMalloc(&s->d_rgb8, px * 3));
        s->px_cap = px;
    }
    return CERES_OK;
}

int launch(ceres_scene* s, const float basis12[12], const float sun[3], int mode, size_t W, size_t H,
           const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, hipStream_t stream,
           int32_t* d_rec_prim = nullptr, float* d_rec_tuv = nullptr, int8_t* d_rec_shadow = nullptr) {
    if (!s || !basis12 || !sun) return set_error(CERES_EINVAL, "render: null argument");
    if (mode != CERES_MODE_FULL && mode != CERES_MODE_PRIMARY) return set_error(CERES_EINVAL, "render: bad mode %d", mode);
    if (W == 0 || H == 0 || W > 65535u * 16u || H > 0xffffffu) return set_error(CERES_EINVAL, "render: bad size %zux%zu", W, H);
    ceres_tiling t{uint32_t(H), 0, 1};
    if (tiling) t = *tiling;
    if (t.world == 0 || t.rank >= t.world || t.row_block == 0) return set_error(CERES_EINVAL, "render: bad tiling");
    const size_t rows = local_rows_of(H, t.row_block, t.rank, t.world);
    if (W * rows > 0xffffffffull) return set_error(CERES_EINVAL, "render: more than 2^32 pixels per rank");
    HIP_TRY(hipSetDevice(s->device));
    const bool twopass = s->variant != kVariantFrame;
    const uint32_t bx = uint32_t((W + 15) / 16), by = uint32_t((rows + 15) / 16);
    const size_t nblocks = size_t(bx) * by;
    const uint32_t cap = uint32_t(((nblocks + kShards - 1) / kShards) * dev::kBlock);
    if (twopass)
        if (int rc = ensure_workspace(s, size_t(cap) * kShards, 0, false, false)) return rc;

    KParams P{};
    std::memcpy(P.eye, basis12, 12); std::memcpy(P.dir, basis12 + 3, 12);
    std::memcpy(P.iu, basis12 + 6, 12); std::memcpy(P.iv, basis12 + 9, 12);
    std::memcpy(P.sun, sun, 12);
    P.W = uint32_t(W); P.H = uint32_t(H);
    P.row_block = t.row_block; P.rank = t.rank; P.world = t.world; P.local_rows = uint32_t(rows);
    P.stack_entries = s->stack_entries;
    P.root_leaf_count = s->root_leaf_count; P.root_leaf_first = s->root_leaf_first;
    P.shard_capacity = cap;
    P.tiles_x = uint32_t((W + 7) / 8); P.tiles_y = uint32_t((rows + 7) / 8);
    P.n_chunks = uint32_t((size_t(P.tiles_x) * P.tiles_y + dev::kChunkTiles - 1) / dev::kChunkTiles);
    P.pairs = s->d_pairs; P.tris = s->d_tris; P.orig = s->d_orig; P.norms = s->d_norms;
    P.pixels = d_pixels; P.rgb8 = d_rgb8; P.jobs = s->d_jobs; P.shards = s->d_shards;
    P.rec_prim = d_rec_prim; P.rec_tuv = d_rec_tuv; P.rec_shadow = d_rec_shadow;
    if ((d_rec_prim != nullptr) != (d_rec_tuv != nullptr) || (d_rec_prim != nullptr) != (d_rec_shadow != nullptr))
        return set_error(CERES_EINVAL, "render: hit records need all three arrays");

    const bool stats = (s->flags & CERES_SCENE_STATS) != 0;
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr;
    if (s->timing) {
        while (s->ev_pool.size() < 3) { hipEvent_t e; HIP_TRY(hipEventCreate(&e)); s->ev_pool.push_back(e); }
        e0 = s->ev_pool.back(); s->ev_pool.pop_back();
        e1 = s->ev_pool.back(); s->ev_pool.pop_back();
        e2 = s->ev_pool.back(); s->ev_pool.pop_back();
        s->ev_used.push_back(e0); s->ev_used.push_back(e1); s->ev_used.push_back(e2);
    }
    HIP_TRY(hipMemsetAsync(s->d_shards, 0, sizeof(Shard) * kShards, stream));
    if (e0) HIP_TRY(hipEventRecord(e0, stream));
    if (!twopass) {
        // persistent frame kernel: one resident grid of independent wavefronts
        const size_t lds = size_t(dev::kFrameBlock / 64) * (size_t(s->stack_entries) * 64 + dev::kQueueWords) * 4;
        const int mi = (mode == CERES_MODE_PRIMARY ? 1 : 0) * 2 + (stats ? 1 : 0);
        const void* fn[4] = {reinterpret_cast<const void*>(dev::ceres_frame<CERES_MODE_FULL, false>),
                             reinterpret_cast<const void*>(dev::ceres_frame<CERES_MODE_FULL, true>),
                             reinterpret_cast<const void*>(dev::ceres_frame<CERES_MODE_PRIMARY, false>),
                             reinterpret_cast<const void*>(dev::ceres_frame<CERES_MODE_PRIMARY, true>)};
        if (s->frame_blocks_per_cu[mi] <= 0) {
            int nb = 0;
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn[mi], dev::kFrameBlock, lds));
            s->frame_blocks_per_cu[mi] = std::max(1, nb);
        }
        const size_t want_waves = size_t(P.n_chunks);                 // never more waves than chunks
        size_t grid = size_t(s->num_cus) * size_t(s->frame_blocks_per_cu[mi]);
        grid = std::max<size_t>(1, std::min(grid, (want_waves + 1) / 2));
        if (stats && s->wave_log_waves < grid * 2) {
            dfree(s->d_wave_log);
            HIP_TRY(hipMalloc(&s->d_wave_log, grid * 2 * 64));
            s->wave_log_waves = grid * 2;
        }
        P.wave_log = stats ? s->d_wave_log : nullptr;
        s->last_grid_waves = grid * 2;
        switch (mi) {
            case 0: hipLaunchKernelGGL((dev::ceres_frame<CERES_MODE_FULL, false>), dim3(uint32_t(grid)), dim3(dev::kFrameBlock), lds, stream, P); break;
            case 1: hipLaunchKernelGGL((dev::ceres_frame<CERES_MODE_FULL, true>), dim3(uint32_t(grid)), dim3(dev::kFrameBlock), lds, stream, P); break;
            case 2: hipLaunchKernelGGL((dev::ceres_frame<CERES_MODE_PRIMARY, false>), dim3(uint32_t(grid)), dim3(dev::kFrameBlock), lds, stream, P); break;
            default: hipLaunchKernelGGL((dev::ceres_frame<CERES_MODE_PRIMARY, true>), dim3(uint32_t(grid)), dim3(dev::kFrameBlock), lds, stream, P); break;
        }
        HIP_TRY(hipGetLastError());
        if (e1) HIP_TRY(hipEventRecord(e1, stream));
        if (e2) { s->ev_used.back() = nullptr; s->ev_pool.push_back(e2); }   // single kernel: no shadow interval
    } else {
        const bool w64 = s->variant == kVariantWave;
        const int bs = w64 ? 64 : dev::kBlock;
        const size_t lds = size_t(s->stack_entries) * bs * 4;
        dim3 grid(uint32_t((W + 15) / 16), uint32_t((rows + 15) / 16)), block(bs);
        if (w64) grid = dim3(uint32_t((size_t(P.tiles_x) * P.tiles_y + s->tiles_per_wave - 1) / s->tiles_per_wave));
#define CERES_PRIMARY(MODE, ST, BS, PF) hipLaunchKernelGGL((dev::ceres_primary<MODE, ST, BS, PF>), grid, block, lds, stream, P)
#define CERES_PRIMARY_PF(MODE, ST, BS) do { if (s->pf_primary) CERES_PRIMARY(MODE, ST, BS, true); else CERES_PRIMARY(MODE, ST, BS, false); } while (0)
        if (w64) {
            if (mode == CERES_MODE_PRIMARY) { if (stats) CERES_PRIMARY_PF(CERES_MODE_PRIMARY, true, 64); else CERES_PRIMARY_PF(CERES_MODE_PRIMARY, false, 64); }
            else { if (stats) CERES_PRIMARY_PF(CERES_MODE_FULL, true, 64); else CERES_PRIMARY_PF(CERES_MODE_FULL, false, 64); }
        } else {
            if (mode == CERES_MODE_PRIMARY) { if (stats) CERES_PRIMARY_PF(CERES_MODE_PRIMARY, true, 256); else CERES_PRIMARY_PF(CERES_MODE_PRIMARY, false, 256); }
            else { if (stats) CERES_PRIMARY_PF(CERES_MODE_FULL, true, 256); else CERES_PRIMARY_PF(CERES_MODE_FULL, false, 256); }
        }
#undef CERES_PRIMARY_PF
#undef CERES_PRIMARY
        HIP_TRY(hipGetLastError());
        if (e1) HIP_TRY(hipEventRecord(e1, stream));
        if (mode == CERES_MODE_FULL) {
            const size_t max_jobs = W * rows;
            const size_t want = (max_jobs + bs - 1) / bs;
            const size_t cap_blocks = size_t(s->num_cus) * (w64 ? 32 : 8);
            const uint32_t sgrid = uint32_t(std::max<size_t>(1, std::min<size_t>(want, cap_blocks)));
            if (stats) {
                const size_t waves = size_t(sgrid) * (bs / 64);
                if (s->wave_log_waves < waves) {
                    dfree(s->d_wave_log);
                    HIP_TRY(hipMalloc(&s->d_wave_log, waves * 64));
                    s->wave_log_waves = waves;
                }
                HIP_TRY(hipMemsetAsync(s->d_wave_log, 0, waves * 64, stream));
                P.wave_log = s->d_wave_log;
                s->last_grid_waves = waves;
            }
#define CERES_SHADOW(ST, BS, PF) hipLaunchKernelGGL((dev::ceres_shadow<ST, BS, PF>), dim3(sgrid), block, lds, stream, P)
#define CERES_SHADOW_PF(ST, BS) do { if (s->pf_shadow) CERES_SHADOW(ST, BS, true); else CERES_SHADOW(ST, BS, false); } while (0)
            if (w64) { if (stats) CERES_SHADOW_PF(true, 64); else CERES_SHADOW_PF(false, 64); }
            else { if (stats) CERES_SHADOW_PF(true, 256); else CERES_SHADOW_PF(false, 256); }
#undef CERES_SHADOW_PF
#undef CERES_SHADOW
            HIP_TRY(hipGetLastError());
        }
        if (e2) HIP_TRY(hipEventRecord(e2, stream));
    }
    if (d_counters) {
        hipLaunchKernelGGL(dev::ceres_finalize, dim3(1), dim3(64), 0, stream, s->d_shards, uint64_t(W * rows), d_counters);
        HIP_TRY(hipGetLastError());
    }
    return CERES_OK;
}

}  // namespace

extern "C" {

const char* ceres_last_error(void) { return error_buffer(); }
const char* ceres_version(void) { return "ceres-mi355x 0.1 (gfx950)"; }
const char* ceres_kernel_names(void) { return "ceres_frame,ceres_primary,ceres_shadow,ceres_finalize"; }

size_t ceres_tiling_local_rows(size_t height, const ceres_tiling* t) {
    if (!t) return height;
    if (t->world == 0 || t->row_block == 0 || t->rank >= t->world) return 0;
    return local_rows_of(height, t->row_block, t->rank, t->world);
}

ceres_scene* ceres_scene_create(const float* tri48, size_t n_tri, const float* norm36, const void* nodes32,
                                size_t n_nodes, const uint64_t* prim64, int device, uint32_t flags) {
    if (!tri48 || !norm36 || !nodes32 || !prim64 || n_tri == 0 || n_nodes == 0) {
        set_error(CERES_EINVAL, "ceres_scene_create: empty scene or null argument");
        return nullptr;
    }
    if (n_tri > 0xffffffffull || n_nodes > 0xffffffffull) { set_error(CERES_EUNSUPPORTED, "scene too large"); return nullptr; }
    std::vector<SiblingPair> pairs;
    std::vector<Tri48> leaf_tris;
    std::vector<uint32_t> orig;
    uint32_t depth = 0, rlc = 0, rlf = 0;
    if (relayout(static_cast<const RefNode*>(nodes32), n_nodes, prim64, n_tri, reinterpret_cast<const Tri48*>(tri48),
                 pairs, leaf_tris, orig, depth, rlc, rlf))
        return nullptr;
    auto* s = new (std::nothrow) ceres_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    s->device = device; s->flags = flags; s->n_tri = n_tri; s->n_pairs = pairs.size();
    s->depth = depth; s->root_leaf_count = rlc; s->root_leaf_first = rlf;
    s->stack_entries = std::max<uint32_t>(1, depth);                 // stack <= depth - 1 entries
    if (const char* v = std::getenv("CERES_KERNEL"))
        s->variant = std::strcmp(v, "wave") == 0 ? kVariantWave : std::strcmp(v, "frame") == 0 ? kVariantFrame : kVariantTwoPass;
    if (const char* v = std::getenv("CERES_TPW")) s->tiles_per_wave = std::max(1, std::atoi(v));
    if (const char* v = std::getenv("CERES_PF")) {                   // "pf_primary pf_shadow" bits, e.g. "01"
        s->pf_primary = v[0] == '1';
        s->pf_shadow = v[0] && v[1] ? v[1] == '1' : s->pf_primary;
    }
    auto fail = [&](int rc) -> ceres_scene* { (void)rc; scene_release(s); delete s; return nullptr; };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { set_error(CERES_EHIP, "no HIP device available"); return fail(0); }
    if (device < 0 || device >= ndev) { set_error(CERES_EINVAL, "device %d out of range (%d devices)", device, ndev); return fail(0); }
    auto body = [&]() -> int {
        HIP_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_error(CERES_EHIP, "device %d is %s, this build targets gfx950 only", device, prop.gcnArchName);
        s->num_cus = prop.multiProcessorCount;
        HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        HIP_TRY(hipMalloc(&s->d_pairs, pairs.size() * sizeof(SiblingPair)));
        HIP_TRY(hipMalloc(&s->d_tris, n_tri * sizeof(Tri48)));
        HIP_TRY(hipMalloc(&s->d_orig, n_tri * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&s->d_norms, n_tri * 36));
        HIP_TRY(hipMalloc(&s->d_shards, sizeof(Shard) * kShards));
        HIP_TRY(hipMalloc(&s->d_counters, 8 * sizeof(uint64_t)));
        HIP_TRY(hipMemcpy(s->d_pairs, pairs.data(), pairs.size() * sizeof(SiblingPair), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->d_tris, leaf_tris.data(), n_tri * sizeof(Tri48), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->d_orig, orig.data(), n_tri * sizeof(uint32_t), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->d_norms, norm36, n_tri * 36, hipMemcpyHostToDevice));
        return CERES_OK;
    };
    if (body()) return fail(0);
    return s;
}

void ceres_scene_destroy(ceres_scene* s) {
    if (!s) return;
    scene_release(s);
    delete s;
}

int ceres_scene_info(const ceres_scene* s, uint32_t* depth, uint32_t* stack_entries, size_t* n_pairs, size_t* device_bytes) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    if (depth) *depth = s->depth;
    if (stack_entries) *stack_entries = s->stack_entries;
    if (n_pairs) *n_pairs = s->n_pairs;
    if (device_bytes) *device_bytes = s->n_pairs * sizeof(SiblingPair) + s->n_tri * (sizeof(Tri48) + 4 + 36);
    return CERES_OK;
}

int ceres_render_device(ceres_scene* s, const float basis12[12], const float sun[3], int mode, size_t W, size_t H,
                        const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    return launch(s, basis12, sun, mode, W, H, tiling, d_pixels, d_rgb8, d_counters, static_cast<hipStream_t>(stream));
}

int ceres_render_f32(ceres_scene* s, const float basis12[12], const float sun[3], int mode, float* pixels,
                     uint8_t* rgb8, size_t W, size_t H, ceres_stats* stats) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    if (int rc = ensure_workspace(s, 0, W * H, pixels != nullptr, rgb8 != nullptr)) return rc;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, s->stream));
    int rc = launch(s, basis12, sun, mode, W, H, nullptr, pixels ? s->d_pixels : nullptr, rgb8 ? s->d_rgb8 : nullptr,
                    s->d_counters, s->stream);
    if (rc) { (void)hipEventDestroy(a); (void)hipEventDestroy(b); return rc; }
    HIP_TRY(hipEventRecord(b, s->stream));
    uint64_t c[8] = {0};
    HIP_TRY(hipMemcpyAsync(c, s->d_counters, sizeof c, hipMemcpyDeviceToHost, s->stream));
    if (pixels) HIP_TRY(hipMemcpyAsync(pixels, s->d_pixels, W * H * 3 * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, s->d_rgb8, W * H * 3, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (stats) {
        stats->rays = c[0]; stats->hits = c[1]; stats->primary_rays = c[2]; stats->shadow_rays = c[3];
        stats->node_pairs = c[4]; stats->tri_tests = c[5]; stats->ms = ms;
    }
    if (c[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

int ceres_render_records(ceres_scene* s, const float basis12[12], const float sun[3], int mode, size_t W, size_t H,
                         int32_t* prim, float* tuv, int8_t* shadow, ceres_stats* stats) {
    if (!s || !prim || !tuv || !shadow) return set_error(CERES_EINVAL, "ceres_render_records: null argument");
    HIP_TRY(hipSetDevice(s->device));
    const size_t n = W * H;
    int32_t* dp = nullptr; float* dt = nullptr; int8_t* ds = nullptr;
    auto cleanup = [&] { dfree(dp); dfree(dt); dfree(ds); };
    if (hipMalloc(&dp, n * 4) != hipSuccess || hipMalloc(&dt, n * 12) != hipSuccess || hipMalloc(&ds, n) != hipSuccess) {
        cleanup();
        return set_error(CERES_ENOMEM, "ceres_render_records: device allocation failed");
    }
    int rc = launch(s, basis12, sun, mode, W, H, nullptr, nullptr, nullptr, s->d_counters, s->stream, dp, dt, ds);
    uint64_t c[8] = {0};
    if (!rc) {
        if (hipMemcpyAsync(c, s->d_counters, sizeof c, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipMemcpyAsync(prim, dp, n * 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipMemcpyAsync(tuv, dt, n * 12, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipMemcpyAsync(shadow, ds, n, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess)
            rc = set_error(CERES_EHIP, "ceres_render_records: copy back failed");
    }
    cleanup();
    if (rc) return rc;
    if (stats) {
        stats->rays = c[0]; stats->hits = c[1]; stats->primary_rays = c[2]; stats->shadow_rays = c[3];
        stats->node_pairs = c[4]; stats->tri_tests = c[5]; stats->ms = 0;
    }
    if (c[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

int ceres_scene_wave_log(ceres_scene* s, uint64_t* out, size_t max_waves, size_t* n_waves) {
    if (!s || !out || !n_waves) return set_error(CERES_EINVAL, "ceres_scene_wave_log: null argument");
    if (!s->d_wave_log) return set_error(CERES_EINVAL, "wave log needs a CERES_SCENE_STATS scene and a persistent-kernel render");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(nullptr));
    const size_t n = std::min(max_waves, s->last_grid_waves);
    HIP_TRY(hipMemcpy(out, s->d_wave_log, n * 64, hipMemcpyDeviceToHost));
    *n_waves = n;
    return CERES_OK;
}

// Per-kernel device timing for the roofline leg of bench.py: while enabled, every render
// records HIP events around ceres_primary and ceres_shadow on the caller's stream.
int ceres_scene_set_timing(ceres_scene* s, int enable) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    s->timing = enable != 0;
    return CERES_OK;
}

// Synchronises, sums the recorded kernel durations (ms) and recycles the events.
int ceres_scene_read_timing(ceres_scene* s, double* primary_ms, double* shadow_ms, uint64_t* renders) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    double p = 0, q = 0;
    const size_t n = s->ev_used.size() / 3;
    for (size_t k = 0; k < n; ++k) {
        hipEvent_t e0 = s->ev_used[3 * k], e1 = s->ev_used[3 * k + 1], e2 = s->ev_used[3 * k + 2];
        HIP_TRY(hipEventSynchronize(e2 ? e2 : e1));
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, e0, e1));
        if (e2) HIP_TRY(hipEventElapsedTime(&b, e1, e2));
        p += a; q += b;
    }
    for (auto e : s->ev_used) if (e) s->ev_pool.push_back(e);
    s->ev_used.clear();
    if (primary_ms) *primary_ms = p;
    if (shadow_ms) *shadow_ms = q;
    if (renders) *renders = n;
    return CERES_OK;
}

}  // extern "C"
