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
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"

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

template <bool kAnyHit, bool kStats>
__device__ __forceinline__ bool trace(const KParams& P, F3 o, F3 d, uint32_t* stk, Hit& best,
                                      uint32_t& n_pairs, uint32_t& n_tests, bool& overflow) {
    const float tmin = 0.0f;
    float tmax = FLT_MAX;                                           // ray.hpp:17-21
    bool have = false;
    auto leaf = [&](uint32_t first, uint32_t count) -> bool {        // intersect_leaf, :43-63
        if (kStats) n_tests += count;
        for (uint32_t k = first; k < first + count; ++k) {
            const TriV tr = load_tri(P.tris + k);
            const F3 c = tr.p0 - o;                                   // Triangle::intersect, triangle.hpp:95-115
            const F3 r = cross(d, c);
            const float inv_det = 1.0f / dot(tr.n, d);
            const float u = dot(r, tr.e2) * inv_det;
            const float v = dot(r, tr.e1) * inv_det;
            const float w = 1.0f - u - v;
            if (u >= 0 && v >= 0 && w >= 0) {
                const float t = dot(tr.n, c) * inv_det;
                if (t >= tmin && t <= tmax) {
                    best = {k, t, u, v};
                    have = true;
                    if (kAnyHit) return true;
                    tmax = t;
                }
            }
        }
        return false;
    };
    if (P.root_leaf_count) {                                          // :72-73
        leaf(P.root_leaf_first, P.root_leaf_count);
        return have;
    }
    // FastNodeIntersector (node_intersectors.hpp:83-103): octant, safe_inverse, -o * inv
    const bool ox = signbit(d.x), oy = signbit(d.y), oz = signbit(d.z);
    auto safe_inv = [](float x) { return 1.0f / (fabsf(x) < FLT_EPSILON ? copysignf(FLT_EPSILON, x) : x); };
    const float ix = safe_inv(d.x), iy = safe_inv(d.y), iz = safe_inv(d.z);
    const float sx = (-o.x) * ix, sy = (-o.y) * iy, sz = (-o.z) * iz;
    uint32_t cur = 0, sp = 0;                                         // pair of the root's children
    while (true) {                                                    // single_ray_traverser.hpp:82-123
        if (kStats) ++n_pairs;
        const float4* q = reinterpret_cast<const float4*>(P.pairs + cur);
        const float4 A = q[0], B = q[1], C = q[2];
        const uint4 L = reinterpret_cast<const uint4*>(q)[3];
        // left child bounds A.x A.y A.z A.w B.x B.y ; right child B.z B.w C.x C.y C.z C.w
        const float le = rmax(__builtin_fmaf(ox ? A.y : A.x, ix, sx),
                         rmax(__builtin_fmaf(oy ? A.w : A.z, iy, sy),
                         rmax(__builtin_fmaf(oz ? B.y : B.x, iz, sz), tmin)));
        const float lx = rmin(__builtin_fmaf(ox ? A.x : A.y, ix, sx),
                         rmin(__builtin_fmaf(oy ? A.z : A.w, iy, sy),
                         rmin(__builtin_fmaf(oz ? B.x : B.y, iz, sz), tmax)));
        const float re = rmax(__builtin_fmaf(ox ? B.w : B.z, ix, sx),
                         rmax(__builtin_fmaf(oy ? C.y : C.x, iy, sy),
                         rmax(__builtin_fmaf(oz ? C.w : C.z, iz, sz), tmin)));
        const float rx = rmin(__builtin_fmaf(ox ? B.z : B.w, ix, sx),
                         rmin(__builtin_fmaf(oy ? C.x : C.y, iy, sy),
                         rmin(__builtin_fmaf(oz ? C.z : C.w, iz, sz), tmax)));
        bool go_l = false, go_r = false;
        if (le <= lx) {
            if (L.x) { if (leaf(L.y, L.x) && kAnyHit) return true; }
            else go_l = true;
        }
        if (re <= rx) {
            if (L.z) { if (leaf(L.w, L.z) && kAnyHit) return true; }
            else go_r = true;
        }
        if (go_l) {
            if (go_r) {
                uint32_t near_c = L.y, far_c = L.w;
                if (le > re) { near_c = L.w; far_c = L.y; }
                if (sp >= P.stack_entries) { overflow = true; return have; }
                stk[sp * kBlock] = far_c;
                ++sp;
                cur = near_c;
            } else {
                cur = L.y;
            }
        } else if (go_r) {
            cur = L.w;
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * kBlock];
        }
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
        const float spec = 0.8f * float(pow(double(dot(N, normalize(sun_line + vneg))), 24.0));
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
template <int kMode, bool kStats>
__global__ __launch_bounds__(kBlock) void ceres_primary(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* stk = lds + tid;                                       // [entries][kBlock]
    uint32_t* red = lds + P.stack_entries * kBlock;                  // block-reduction scratch (16 words)
    // 16x16 pixel block = 2x2 wavefront tiles of 8x8 (coherent primary rays per wave)
    const uint32_t i = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const uint32_t lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
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
        hit = trace<false, kStats>(P, eye, view, stk, h, n_pairs, n_tests, overflow);
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
    // wave-level compaction of shadow rays + hit count; one queue atomic per workgroup
    const unsigned long long jm = __ballot(job);
    const unsigned long long hm = __ballot(hit);
    if (lane == 0) { red[wave] = __popcll(jm); red[kWaves + wave] = __popcll(hm); }
    __syncthreads();
    const uint32_t shard = (blockIdx.y * gridDim.x + blockIdx.x) % kShards;
    if (tid == 0) {
        uint32_t nj = 0, nh = 0;
        for (int w = 0; w < kWaves; ++w) { nj += red[w]; nh += red[kWaves + w]; }
        red[2 * kWaves] = nj ? atomicAdd(&P.shards[shard].queued, nj) : 0u;
        if (nh) atomicAdd(&P.shards[shard].hits, (unsigned long long)nh);
    }
    __syncthreads();
    if (job) {
        uint32_t off = red[2 * kWaves];
        for (uint32_t w = 0; w < wave; ++w) off += red[w];
        off += __popcll(jm & ((1ull << lane) - 1ull));
        ShadowJob* dst = P.jobs + size_t(shard) * P.shard_capacity + off;
        float4* q = reinterpret_cast<float4*>(dst);
        q[0] = make_float4(__uint_as_float(lr * P.W + i), __uint_as_float(h.slot), h.u, h.v);
        q[1] = make_float4(shadow_o.x, shadow_o.y, shadow_o.z, 0.f);
    }
    if (kStats) {
        const uint32_t wp = wave_sum(n_pairs), wt = wave_sum(n_tests);
        __syncthreads();
        if (lane == 0) { red[wave] = wp; red[kWaves + wave] = wt; }
        __syncthreads();
        if (tid == 0) {
            unsigned long long sp = 0, st = 0;
            for (int w = 0; w < kWaves; ++w) { sp += red[w]; st += red[kWaves + w]; }
            atomicAdd(&P.shards[shard].pairs, sp);
            atomicAdd(&P.shards[shard].tests, st);
        }
    }
    if (overflow) atomicOr(&P.shards[shard].error, 1u);
}

// ---------------------------------------------------------------- shadow kernel
template <bool kStats>
__global__ __launch_bounds__(kBlock) void ceres_shadow(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* stk = lds + tid;
    uint32_t* pre = lds + P.stack_entries * kBlock;                  // 33 prefix words + 8 reduction words
    uint32_t* red = pre + 36;
    if (tid < kShards) pre[tid + 1] = P.shards[tid].queued;
    __syncthreads();
    if (tid == 0) { pre[0] = 0; for (int s = 1; s <= kShards; ++s) pre[s] += pre[s - 1]; }
    __syncthreads();
    const uint32_t total = pre[kShards];
    const F3 sun{P.sun[0], P.sun[1], P.sun[2]};
    uint32_t occluded = 0, n_pairs = 0, n_tests = 0;
    bool overflow = false;
    for (uint32_t g = blockIdx.x * kBlock + tid; g < total; g += gridDim.x * kBlock) {
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
        const bool blocked = trace<true, kStats>(P, o, sun_line, stk, h2, n_pairs, n_tests, overflow);
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
    const uint32_t wp = kStats ? wave_sum(n_pairs) : 0u, wt = kStats ? wave_sum(n_tests) : 0u;
    if (lane == 0) { red[wave] = wo; red[kWaves + wave] = wp; red[2 * kWaves + wave] = wt; }
    __syncthreads();
    const uint32_t shard = blockIdx.x % kShards;
    if (tid == 0) {
        unsigned long long so = 0, sp = 0, st = 0;
        for (int w = 0; w < kWaves; ++w) { so += red[w]; sp += red[kWaves + w]; st += red[2 * kWaves + w]; }
        if (so) atomicAdd(&P.shards[shard].hits, so);
        if (kStats) { atomicAdd(&P.shards[shard].pairs, sp); atomicAdd(&P.shards[shard].tests, st); }
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
    // optional per-kernel device timing (bench.py roofline leg)
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<hipEvent_t> ev_used;   // triples: start, after primary, after shadow
};

namespace {

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
    dfree(s->d_shards); dfree(s->d_counters); dfree(s->d_jobs); dfree(s->d_pixels); dfree(s->d_rgb8);
    for (auto e : s->ev_pool) (void)hipEventDestroy(e);
    for (auto e : s->ev_used) (void)hipEventDestroy(e);
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
    const uint32_t bx = uint32_t((W + 15) / 16), by = uint32_t((rows + 15) / 16);
    const size_t nblocks = size_t(bx) * by;
    const uint32_t cap = uint32_t(((nblocks + kShards - 1) / kShards) * dev::kBlock);
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
    P.pairs = s->d_pairs; P.tris = s->d_tris; P.orig = s->d_orig; P.norms = s->d_norms;
    P.pixels = d_pixels; P.rgb8 = d_rgb8; P.jobs = s->d_jobs; P.shards = s->d_shards;
    P.rec_prim = d_rec_prim; P.rec_tuv = d_rec_tuv; P.rec_shadow = d_rec_shadow;
    if ((d_rec_prim != nullptr) != (d_rec_tuv != nullptr) || (d_rec_prim != nullptr) != (d_rec_shadow != nullptr))
        return set_error(CERES_EINVAL, "render: hit records need all three arrays");

    const bool stats = (s->flags & CERES_SCENE_STATS) != 0;
    const size_t lds_primary = (size_t(s->stack_entries) * dev::kBlock + 16) * 4;
    const size_t lds_shadow = (size_t(s->stack_entries) * dev::kBlock + 48) * 4;
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
    const dim3 grid(bx, by), block(dev::kBlock);
    if (mode == CERES_MODE_PRIMARY) {
        if (stats) hipLaunchKernelGGL((dev::ceres_primary<CERES_MODE_PRIMARY, true>), grid, block, lds_primary, stream, P);
        else hipLaunchKernelGGL((dev::ceres_primary<CERES_MODE_PRIMARY, false>), grid, block, lds_primary, stream, P);
    } else {
        if (stats) hipLaunchKernelGGL((dev::ceres_primary<CERES_MODE_FULL, true>), grid, block, lds_primary, stream, P);
        else hipLaunchKernelGGL((dev::ceres_primary<CERES_MODE_FULL, false>), grid, block, lds_primary, stream, P);
    }
    HIP_TRY(hipGetLastError());
    if (e1) HIP_TRY(hipEventRecord(e1, stream));
    if (mode == CERES_MODE_FULL) {
        const size_t max_jobs = W * rows;
        const size_t want = (max_jobs + dev::kBlock - 1) / dev::kBlock;
        const uint32_t sgrid = uint32_t(std::max<size_t>(1, std::min<size_t>(want, size_t(s->num_cus) * 8)));
        if (stats) hipLaunchKernelGGL((dev::ceres_shadow<true>), dim3(sgrid), block, lds_shadow, stream, P);
        else hipLaunchKernelGGL((dev::ceres_shadow<false>), dim3(sgrid), block, lds_shadow, stream, P);
        HIP_TRY(hipGetLastError());
    }
    if (e2) HIP_TRY(hipEventRecord(e2, stream));
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
const char* ceres_kernel_names(void) { return "ceres_primary,ceres_shadow,ceres_finalize"; }

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
        HIP_TRY(hipEventSynchronize(e2));
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, e0, e1));
        HIP_TRY(hipEventElapsedTime(&b, e1, e2));
        p += a; q += b;
    }
    for (auto e : s->ev_used) s->ev_pool.push_back(e);
    s->ev_used.clear();
    if (primary_ms) *primary_ms = p;
    if (shadow_ms) *shadow_ms = q;
    if (renders) *renders = n;
    return CERES_OK;
}

}  // extern "C"
