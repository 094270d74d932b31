// render_hip.hip -- the CERES hot path as hand-written HIP for gfx950 (MI355X) + its C ABI.
//
// Replaces render<float>() of include/render.hpp:86-156 (iracigt/ceres-raytracer): per-pixel
// primary rays (render.hpp:105-113), BVH2 traversal (single_ray_traverser.hpp:68-126) with the
// fast slab test (node_intersectors.hpp:35-47,83-103), Moller-Trumbore (triangle.hpp:95-115),
// the offset shadow ray (render.hpp:119-138) and smooth Blinn-Phong shading (render.hpp:46-84),
// plus the PPM quantiser of static.cpp:135-147.
//
// Full mode: ONE kernel per batch of frames, ceres_fused (DESIGN.md "Kernels"): one 64-thread
// workgroup per 8x8 pixel tile (coherent primary rays), tiles walked centre-first (views of
// >= 4 Mpixel: frame after frame, XCD-local Morton order for batches and DRAM-resident scenes);
// an exact root-box pre-test, then closest-hit BVH2 traversal per pixel (software-pipelined: the
// next record is loaded before the step's triangle tests), then the tile's shadow rays over an
// exact BVH4 collapse (any-hit: only the boolean matters, render.hpp:139; one-frame launches
// share the rays' work among the lanes), then shading of the lit pixels.  Primary-only mode
// (C2): ceres_primary.  CERES_MODE_QBVH4: shadow rays over a compressed BVH4 (not exact).
// A batch is 1..kMaxFrames frames (own camera + sun each, e.g. the anim.cpp:93-110 orbit),
// each restricted to this rank's rows (ceres_tiling).
// Traversal stacks live in LDS ([entries][lanes], lane-contiguous = bank-conflict free),
// sized from the BVH at scene creation, 16-bit entries when every node index fits.
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32 div/sqrt, explicit
// fmaf only where the reference calls fast_multiply_add, x^24 in double for std::pow (pow24.hpp,
// exhaustively equal to glibc for every float) -- every float matches the reference compiled
// without contraction bit for bit.  CERES_MODE_FMA instantiates every kernel a second time with
// an explicit fmaf at exactly the sites where the reference's own CMake build (g++ -O3 -mfma)
// contracts (kG, oracle/contraction_sites.txt): then every float matches THAT build bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "pow24.hpp"

#pragma clang fp contract(off)

#ifndef CERES_COUNTING
#define CERES_COUNTING 0                       // 1: the diagnostic build (make count): fetch tallies + stack guard
#endif
#ifndef CERES_TILES_PER_WAVE
#define CERES_TILES_PER_WAVE 4                // fused kernel, batches: consecutive tile-order entries (1, 2, 4 or 8) per
#endif                                        // wavefront (A/B, 16-frame batches x 8 streams: 4 beats 2 by 2 %; round 5
                                              // profiles/r05/s8-s9: 8 vs 4 within +-1 %, no consistent sign)
#ifndef CERES_TPW_BY_SIZE
#define CERES_TPW_BY_SIZE 1                    // batches of 16-bit-stack 1080p-class frames: 2 tiles per wave (batch_tiles_per_wave)
#endif
#ifndef CERES_FRAME_MAJOR_PIXELS
#define CERES_FRAME_MAJOR_PIXELS (1u << 20)    // batches of frames of >= this many pixels: frame after frame, XCD-local
                                               // Morton order (0: never; round 5: 1 Mpixel, was 4)
#endif
#ifndef CERES_SPLIT_UNIFORM
#define CERES_SPLIT_UNIFORM 1                  // wave-uniform triangle / BVH4 fetches get their own copy of the test
#endif
#ifndef CERES_ROOT_TEST
#define CERES_ROOT_TEST 1                      // primary rays test the root box before the first record (set_root_box)
#endif
#ifndef CERES_OCTANT_SLAB
#define CERES_OCTANT_SLAB 3                    // traversal loops specialised per wave-uniform ray octant:
                                               // 1 BVH2, 2 shadow BVH4 (multi-frame kernel), 4 also in the single-frame kernel
#endif
#ifndef CERES_SHADOW_PACKET
#define CERES_SHADOW_PACKET 1                  // batch kernel: a tile's shadow rays as one wave-wide masked packet (packet_any4)
#endif
#ifndef CERES_TRUST_STACK_BOUND
#define CERES_TRUST_STACK_BOUND 1              // BVH2 steps of non-stats kernels: no stack clamps / overflow flag
#endif
#ifndef CERES_PAIR_STORES
#define CERES_PAIR_STORES 1                    // batch kernels: a wavefront's tile pairs store back to back (PairStash)
#endif
#ifndef CERES_STACK_GUARD
#define CERES_STACK_GUARD CERES_COUNTING       // the BVH2 stack's guard slot (guarded_trace): the diagnostic (counting)
#endif                                         // build only -- in the product it cost 1.9 % (C3) / 6.5 % (C5) of a batch
#ifndef CERES_ASSEMBLE_NT
#define CERES_ASSEMBLE_NT 0                    // ceres_assemble: nontemporal loads / stores
#endif
#ifndef CERES_LOCAL_ORDER
#define CERES_LOCAL_ORDER 1                    // XCD-local Morton tile order (ensure_tile_order); 0: never
#endif
#ifndef CERES_LOCAL_CHUNK_BATCH
#define CERES_LOCAL_CHUNK_BATCH 128            // tiles per XCD block: frame-major batches (round 6 A/B, 16-frame
                                               // batches x 8 streams: 64 -> 128 C3 +1.4..1.8 %, dragon 4096^2
                                               // +1.0..1.6 %, bunny 1080p +0.7 %, C5 +-0; profiles/r06/chunk) ...
#endif
#ifndef CERES_XCD_GROUP_TILES
#define CERES_XCD_GROUP_TILES 16               // centre-first batch orders: runs of this many adjacent tiles of a row on
#endif                                        // one XCD (xcd_group_rows; 0: off)
#ifndef CERES_LOCAL_CHUNK_SOLO
#define CERES_LOCAL_CHUNK_SOLO 16              // ... and single large frames of a DRAM-resident scene
#endif
#ifndef CERES_RCP_UNIFORM
#define CERES_RCP_UNIFORM 2                    // rcp_exact's IEEE-division fallback behind a wave-uniform branch
#endif                                         // (ballot) instead of a divergent one: 0 nowhere, 1 in every
                                               // kernel, 2 in the single-frame kernel only
#ifndef CERES_RCP_IFTHEN
#define CERES_RCP_IFTHEN 1                     // rcp_exact (non-uniform form): fast quotient everywhere, division in an if-then
#endif
#ifndef CERES_PK_PACKET
#define CERES_PK_PACKET 1                      // packet_any4: slab fmas two children at a time (v_pk_fma_f32)
#endif
#ifndef CERES_LOAD_ALWAYS
#define CERES_LOAD_ALWAYS 1                    // trace(): finished lanes load a (cached) record too -- no branch
                                               // (batch kernel; A/B profiles/r04/s4 "ldall": batches -0.7..-1.5 %)
#endif
#ifndef CERES_CULL
#define CERES_CULL 1                           // tiles whose rays provably miss the root box: stored as misses (tile_misses_root)
#endif
#ifndef CERES_TRI_SELECT
#define CERES_TRI_SELECT 1                     // triangle test without control flow (t always computed, one
#endif                                         // predicate) and closest-hit updates as selects

namespace ceres {

char* error_buffer() {
    static thread_local char buf[kErrorBufferSize] = "";
    return buf;
}

namespace dev {

constexpr int kBlock = 256;            // 4 wavefronts of 64 lanes

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(F3 a, F3 b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
__device__ __forceinline__ F3 cross(F3 a, F3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// Correctly rounded 1/x (IEEE division: the reference's `1 / dot(n, d)`), fast path: one
// Newton step r1 = fma(fma(-x, r0, 1), r0, r0) on the hardware estimate r0 = v_rcp_f32(x) is
// bit-identical to the IEEE quotient for every normal |x| in [2^-126, 2^126) -- checked
// exhaustively over all 2^32 inputs on gfx950 (tools/probes/rcp_exhaustive.hip,
// tests/test_gpu_parity.py::test_fast_reciprocal_is_exact).  Zero, denormal, huge, inf and NaN
// inputs take the full v_div_scale/fmas/fixup division.
// kU: the division fallback behind a wave-uniform branch (the estimate and the Newton step run in
// every lane; only a wavefront with an out-of-range input pays the division) -- used where
// CERES_RCP_UNIFORM selects it (2: the single-frame kernel, where it measured -1..-2 %; in the
// multi-frame kernel it measured neutral alone and +12 % together with CERES_TRI_SELECT)
template <bool kU = false>
__device__ __forceinline__ float rcp_exact(float x) {
    const uint32_t m = __float_as_uint(x) & 0x7fffffffu;
    if (kU) {
        // only x is live at the wave-uniform branch: each side computes its own quotient
        const bool slow = m - 0x00800000u >= 0x7e000000u - 0x00800000u;
        if (__builtin_expect(__ballot(slow) != 0, 0)) {
            const float q = 1.0f / x;
            const float r0 = __builtin_amdgcn_rcpf(x);
            return slow ? q : __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
        }
        const float r0 = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    }
    if constexpr (CERES_RCP_IFTHEN) {
        // the fast quotient in every lane, the division only in the (rare) lanes that need it: a
        // one-sided branch (no else arm: two fewer exec-mask instructions per triangle test)
        const float r0 = __builtin_amdgcn_rcpf(x);
        float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
        if (__builtin_expect(m - 0x00800000u >= 0x7e000000u - 0x00800000u, 0)) r = 1.0f / x;
        return r;
    }
    if (__builtin_expect(m - 0x00800000u >= 0x7e000000u - 0x00800000u, 0)) return 1.0f / x;
    const float r0 = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
}

// rcp_exact's fast path alone, for an x known to be a normal float with |x| < 2^126 or NaN: then
// it IS the IEEE quotient (NaN in, NaN out -- its payload may differ from the division's, so only
// where a NaN can reach nothing but comparisons).  safe_inverse's argument: |d| <= 1 (d is
// normalized), clamped to >= FLT_EPSILON.
__device__ __forceinline__ float rcp_fast(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ F3 normalize(F3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
__device__ __forceinline__ F3 f3(const float* p) { return {p[0], p[1], p[2]}; }

// The reference as its own CMake build compiles it (CMakeLists.txt:11-13, g++ -O3 -mavx2 -mfma;
// CERES_MODE_FMA, kernels instantiated with kG = true): GCC contracts a*b+c into one FMA at the
// sites its widening_mul pass picks -- read from the compiler's dump of the reference, listed in
// oracle/contraction_sites.txt.  dot (vector.hpp:134-141) becomes fma(a2,b2, fma(a0,b0, a1 b1))
// ("A") everywhere but Triangle::intersect's v = dot(r, e1), fused as fma(a2,b2, fma(a1,b1, a0 b0))
// ("B"); cross (vector.hpp:159-167) a_j b_k - a_k b_j becomes fma(a_j, b_k, -(a_k b_j)).  With
// kG = false every helper is the plain contraction-free expression.
template <bool kG> __device__ __forceinline__ float dotA(F3 a, F3 b) {
    if constexpr (kG) return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.x, b.x, a.y * b.y));
    else return dot(a, b);
}
template <bool kG> __device__ __forceinline__ float dotB(F3 a, F3 b) {
    if constexpr (kG) return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
    else return dot(a, b);
}
template <bool kG> __device__ __forceinline__ F3 crossG(F3 a, F3 b) {
    if constexpr (kG)
        return {__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
                __builtin_fmaf(a.x, b.y, -(a.y * b.x))};
    else return cross(a, b);
}
template <bool kG> __device__ __forceinline__ F3 normalizeG(F3 v) { float inv = 1.0f / sqrtf(dotA<kG>(v, v)); return v * inv; }

// Wave-uniform fetches.  The fused kernel is bound by the vector-memory return path (PMC of an
// 8-frame C3 batch: TD busy 79 %, TA 70 % of cycles), which delivers every active lane's 16 B
// per dwordx4 even when all lanes read the same record -- and in half the primary BVH2 steps
// they do (coherent 8x8 tiles; tools/diag_uniform.py: C3 49 %, bunny 64 %, dragon 4096^2 65 %
// of wave-steps; shadow BVH4 steps 33-51 %, leaf triangles 48-77 %).  Such a record is read
// once through the scalar cache instead (s_load into SGPRs: no TA/TD traffic) and broadcast.
// uniform_id: true and r = the id when every active lane of the wavefront holds the same id.
__device__ __forceinline__ bool uniform_id(uint32_t id, uint32_t& r) {
    r = __builtin_amdgcn_readfirstlane(id);
    return __ballot(id != r) == 0;
}
// Counting build (CERES_COUNTING=1, `make count` -> libceres_hip_count.so; never the product): every
// fetch site adds the bytes it moves to a device-global tally (round 6, VERDICT r5 item 1: "the
// build's own counted bytes").  A vector fetch moves its bytes for EVERY active lane (the per-lane
// records of a divergent walk); a scalar (s_load) fetch moves them once per wavefront.  In the
// product the macros are empty, so the kernels are the ones bench.py times.
enum FetchKind : int {
    kFBvh2V = 0,   // 64-B sibling-pair records, vector loads (per lane)
    kFBvh4V,       // 112-B BVH4 records (64-B QBVH4), vector loads (per lane)
    kFBvh4S,       // BVH4 records through the scalar cache (per wavefront; 116 B with nleaf)
    kFTriV,        // 48-B triangles, vector loads (per lane)
    kFTriS,        // 48-B triangles through the scalar cache (per wavefront)
    kFShadeV,      // per hit: the 48-B hit triangle; per lit pixel: 4-B orig + 36-B normals
    kFStoreV,      // framebuffer stores: 12-B float + 3-B RGB8 per pixel
    kFOrderS,      // tile-order entries (scalar)
    kFKinds
};
#if CERES_COUNTING
constexpr int kFetchShards = 16;
__device__ unsigned long long g_fetch[kFetchShards][kFKinds];
__device__ __forceinline__ void count_fetch(int k, uint32_t bytes, bool per_lane) {
    const uint64_t m = __ballot(1);                                    // the active lanes
    if ((threadIdx.x & 63u) == uint32_t(__builtin_ctzll(m)))
        atomicAdd(&g_fetch[blockIdx.x % kFetchShards][k], (unsigned long long)(per_lane ? __popcll(m) : 1) * bytes);
}
#define CERES_COUNT_V(k, b) ::ceres::dev::count_fetch((k), (b), true)
#define CERES_COUNT_S(k, b) ::ceres::dev::count_fetch((k), (b), false)
#else
#define CERES_COUNT_V(k, b) ((void)0)
#define CERES_COUNT_S(k, b) ((void)0)
#endif

typedef float F4v __attribute__((ext_vector_type(4)));
typedef uint32_t U4v __attribute__((ext_vector_type(4)));
// 16-B piece i of a read-only record through the constant address space: s_load_dwordx*
// (the address must be wave-uniform; the scene is never written while a kernel runs)
__device__ __forceinline__ float4 sload_f4(const void* p, int i) {
    const F4v v = ((const __attribute__((address_space(4))) F4v*)(p))[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t sload_u32(const void* p) {
    return *((const __attribute__((address_space(4))) uint32_t*)(p));
}
__device__ __forceinline__ uint4 sload_u4(const void* p, int i) {
    const U4v v = ((const __attribute__((address_space(4))) U4v*)(p))[i];
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct TriV { F3 p0, e1, e2, n; };
__device__ __forceinline__ TriV load_tri(const Tri48* t) {
    const float4* q = reinterpret_cast<const float4*>(t);
    const float4 a = q[0], b = q[1], c = q[2];
    return {{a.x, a.y, a.z}, {a.w, b.x, b.y}, {b.z, b.w, c.x}, {c.y, c.z, c.w}};
}
// the same record through the scalar cache (t wave-uniform)
__device__ __forceinline__ TriV load_tri_s(const Tri48* t) {
    const float4 a = sload_f4(t, 0), b = sload_f4(t, 1), c = sload_f4(t, 2);
    return {{a.x, a.y, a.z}, {a.w, b.x, b.y}, {b.z, b.w, c.x}, {c.y, c.z, c.w}};
}
// triangle `idx` for the active lanes: one scalar fetch when they all test the same triangle
__device__ __forceinline__ TriV load_tri_u(const Tri48* tris, uint32_t idx) {
    uint32_t r;
    if (uniform_id(idx, r)) { CERES_COUNT_S(kFTriS, 48); return load_tri_s(tris + r); }
    CERES_COUNT_V(kFTriV, 48);
    return load_tri(tris + idx);
}

// 24-bit LDS stack entries for scenes whose node indices need more than 16 bits but fewer
// than 24 (C5: 5.3M pairs): a u16 plane + a u8 plane, [entry][lane] each.  3 B per entry
// instead of 4 keeps a 28-deep stack's LDS under the 6-waves/SIMD budget.
struct Stk24 {
    uint16_t* lo;
    uint8_t* hi;
    struct Ref {
        uint16_t* lo; uint8_t* hi;
        __device__ __forceinline__ operator uint32_t() const { return uint32_t(*lo) | (uint32_t(*hi) << 16); }
        __device__ __forceinline__ Ref& operator=(uint32_t v) { *lo = uint16_t(v); *hi = uint8_t(v >> 16); return *this; }
    };
    __device__ __forceinline__ Ref operator[](uint32_t i) const { return {lo + i, hi + i}; }
};

// The guard value of a stack type: all ones in its width (no node index reaches it: stack_width
// picks a width whose largest value exceeds every pair / BVH4 index of the scene).
template <typename StkT> __device__ __forceinline__ constexpr uint32_t stack_guard() {
    return std::is_same<StkT, uint16_t*>::value ? 0xffffu : std::is_same<StkT, Stk24>::value ? 0xffffffu : 0xffffffffu;
}

// Per-ray hit; closest hit keeps the LAST accepted hit with t <= tmax (intersect_leaf :54-60).
struct Hit { uint32_t slot; float t, u, v; };
constexpr uint32_t kNoSlot = 0xffffffffu;                            // no hit yet (slots are < 2^32 - 1)

// Triangle::intersect (triangle.hpp:95-115, left-handed normal).
template <bool kG = false, bool kU = false>
__device__ __forceinline__ bool tri_test(const TriV& tr, F3 o, F3 d, float tmin, float tmax, float& t_out,
                                         float& u_out, float& v_out) {
    const F3 c = tr.p0 - o;
    const F3 r = crossG<kG>(d, c);
    const float inv_det = rcp_exact<kU>(dotA<kG>(tr.n, d));
    const float u = dotA<kG>(r, tr.e2) * inv_det;
    const float v = dotB<kG>(r, tr.e1) * inv_det;
    const float w = 1.0f - u - v;
    if (CERES_TRI_SELECT) {
        // the same values and the same decision, without control flow: t is computed whether or not
        // (u, v, w) pass, and the comparisons (false on NaN) are combined with bitwise ands
        const float t = dotA<kG>(tr.n, c) * inv_det;
        t_out = t; u_out = u; v_out = v;
        // the conjunction as selects (VALU) instead of and-ed lane masks (SALU): each stage passes
        // its operand on only while the earlier comparisons held; -1 fails every later one (tmin > -1;
        // round 5 A/B: batches -0.2..-0.4 %)
        const float x1 = u >= 0 ? v : -1.0f;
        const float x2 = x1 >= 0 ? w : -1.0f;
        const float x3 = x2 >= 0 ? t : -1.0f;
        return (x3 >= tmin) & (x3 <= tmax);
    }
    if (u >= 0 && v >= 0 && w >= 0) {
        const float t = dotA<kG>(tr.n, c) * inv_det;
        if (t >= tmin && t <= tmax) { t_out = t; u_out = u; v_out = v; return true; }
    }
    return false;
}

// tri_test on triangle `idx`, the wave-uniform case with its own copy of the test: the test
// then reads the record from SGPRs instead of first copying the 12 scalar-loaded words into
// VGPRs to join the vector path (12 v_mov per uniform test; CERES_SPLIT_UNIFORM)
template <bool kG = false, bool kU = false>
__device__ __forceinline__ bool tri_test_u(const Tri48* tris, uint32_t idx, F3 o, F3 d, float tmin, float tmax,
                                           float& t_out, float& u_out, float& v_out) {
    if (!CERES_SPLIT_UNIFORM) return tri_test<kG, kU>(load_tri_u(tris, idx), o, d, tmin, tmax, t_out, u_out, v_out);
    uint32_t r;
    if (uniform_id(idx, r)) {
        CERES_COUNT_S(kFTriS, 48);
        return tri_test<kG, kU>(load_tri_s(tris + r), o, d, tmin, tmax, t_out, u_out, v_out);
    }
    CERES_COUNT_V(kFTriV, 48);
    return tri_test<kG, kU>(load_tri(tris + idx), o, d, tmin, tmax, t_out, u_out, v_out);
}

// tri_test's decision for every lane as a wave mask (the packet's any-hit): one ballot per
// comparison, and'ed as masks -- the same predicate without materialising a per-lane boolean
template <bool kG = false, bool kU = false>
__device__ __forceinline__ uint64_t tri_mask(const TriV& tr, F3 o, F3 d, float tmin, float tmax) {   // tmin > -1
    const F3 c = tr.p0 - o;
    const F3 r = crossG<kG>(d, c);
    const float inv_det = rcp_exact<kU>(dotA<kG>(tr.n, d));
    const float u = dotA<kG>(r, tr.e2) * inv_det;
    const float v = dotB<kG>(r, tr.e1) * inv_det;
    const float w = 1.0f - u - v;
    const float t = dotA<kG>(tr.n, c) * inv_det;
    // the conjunction as a chain of selects (VALU) rather than and-ed lane masks (SALU): each stage
    // passes its next operand only while every earlier comparison held (-1 fails all later ones,
    // t >= tmin included since tmin > -1; a NaN fails them as the comparison it replaces would)
    const float x1 = u >= 0 ? v : -1.0f;
    const float x2 = x1 >= 0 ? w : -1.0f;
    const float x3 = x2 >= 0 ? t : -1.0f;
    return __ballot((x3 >= tmin) & (x3 <= tmax));
}

// Per-ray constants of the ray-box (slab) test and the test of one box.
//   kRobust = false: FastNodeIntersector (node_intersectors.hpp:83-103): inv = safe_inverse(d)
//     (vector.hpp:69-74), s = -o * inv, slab = fma(bound, inv, s) -- restated octant-free below.
//   kRobust = true: RobustNodeIntersector (node_intersectors.hpp:54-79): inv = 1 / d, entry slab
//     (near - o) * inv, exit slab (far - o) * pinv with pinv = inv padded by 2 ulps of magnitude
//     (add_ulp_magnitude, utilities.hpp:102-106); near/far chosen by the ray octant as in
//     NodeIntersector::intersect (:35-47) -- inv may be +-inf here, so the octant-free min/max
//     form does not apply: (p - o) * inf is NaN when p == o, which robust_max/min (and
//     fmaxf/fminf) drop, but a min over both slabs would not.
template <bool kRobust>
struct Slab {
    float ix, iy, iz;          // inverse direction
    float sx, sy, sz;          // fast: -o * inv; robust: padded inverse
    F3 o;                      // robust only
};
__device__ __forceinline__ float pad_ulps2(float x) {
    return isfinite(x) ? __uint_as_float(__float_as_uint(x) + 2u) : x;
}
template <bool kRobust>
__device__ __forceinline__ Slab<kRobust> make_slab(F3 o, F3 d) {
    Slab<kRobust> s;
    if constexpr (kRobust) {
        s.ix = 1.0f / d.x; s.iy = 1.0f / d.y; s.iz = 1.0f / d.z;
        s.sx = pad_ulps2(s.ix); s.sy = pad_ulps2(s.iy); s.sz = pad_ulps2(s.iz);
    } else {
        // safe_inverse (vector.hpp:69-74): 1 / d, |d| clamped to >= FLT_EPSILON; d is normalized, so the
        // quotient's argument lies in [FLT_EPSILON, 1 + ulp] (or is NaN, which every slab comparison
        // rejects whatever its payload): rcp_fast is the IEEE quotient there
        auto safe_inv = [](float x) { return rcp_fast(fabsf(x) < FLT_EPSILON ? copysignf(FLT_EPSILON, x) : x); };
        s.ix = safe_inv(d.x); s.iy = safe_inv(d.y); s.iz = safe_inv(d.z);
        s.sx = (-o.x) * s.ix; s.sy = (-o.y) * s.iy; s.sz = (-o.z) * s.iz;
    }
    s.o = o;
    return s;
}
// entry / exit distances of one box (bounds lo, hi per axis); hit iff e <= x.
// kOct >= 0 (fast test only): the ray octant is known at compile time -- bit a set when axis a's
// inverse direction is negative -- and each axis's entry / exit bound is picked by it, as the
// reference's NodeIntersector does (node_intersectors.hpp:35-47): three fmas per side and no
// per-axis min / max (16 -> 10 VALU per box).
template <bool kRobust, int kOct = -1>
__device__ __forceinline__ void slab_box(const Slab<kRobust>& s, float lox, float hix, float loy, float hiy, float loz,
                                         float hiz, float tmin, float tmax, float& e, float& x) {
    if constexpr (!kRobust && kOct >= 0) {
        const float nx = (kOct & 1) ? hix : lox, fx = (kOct & 1) ? lox : hix;
        const float ny = (kOct & 2) ? hiy : loy, fy = (kOct & 2) ? loy : hiy;
        const float nz = (kOct & 4) ? hiz : loz, fz = (kOct & 4) ? loz : hiz;
        e = fmaxf(__builtin_fmaf(nx, s.ix, s.sx), fmaxf(__builtin_fmaf(ny, s.iy, s.sy), fmaxf(__builtin_fmaf(nz, s.iz, s.sz), tmin)));
        x = fminf(__builtin_fmaf(fx, s.ix, s.sx), fminf(__builtin_fmaf(fy, s.iy, s.sy), fminf(__builtin_fmaf(fz, s.iz, s.sz), tmax)));
    } else if constexpr (kRobust) {
        const bool nx = __float_as_uint(s.ix) >> 31, ny = __float_as_uint(s.iy) >> 31, nz = __float_as_uint(s.iz) >> 31;
        const float ex = ((nx ? hix : lox) - s.o.x) * s.ix, xx = ((nx ? lox : hix) - s.o.x) * s.sx;
        const float ey = ((ny ? hiy : loy) - s.o.y) * s.iy, xy = ((ny ? loy : hiy) - s.o.y) * s.sy;
        const float ez = ((nz ? hiz : loz) - s.o.z) * s.iz, xz = ((nz ? loz : hiz) - s.o.z) * s.sz;
        e = fmaxf(ex, fmaxf(ey, fmaxf(ez, tmin)));
        x = fminf(xx, fminf(xy, fminf(xz, tmax)));
    } else {
        const float a0 = __builtin_fmaf(lox, s.ix, s.sx), a1 = __builtin_fmaf(hix, s.ix, s.sx);
        const float b0 = __builtin_fmaf(loy, s.iy, s.sy), b1 = __builtin_fmaf(hiy, s.iy, s.sy);
        const float c0 = __builtin_fmaf(loz, s.iz, s.sz), c1 = __builtin_fmaf(hiz, s.iz, s.sz);
        e = fmaxf(fminf(a0, a1), fmaxf(fminf(b0, b1), fmaxf(fminf(c0, c1), tmin)));
        x = fminf(fmaxf(a0, a1), fminf(fmaxf(b0, b1), fminf(fmaxf(c0, c1), tmax)));
    }
}

// The octant of a fast slab (see slab_box) and, when every active lane of the wavefront shares it,
// fn(std::integral_constant<int, octant>) -- the traversal loop instantiated for that octant; else
// false.  Primary rays of an 8x8 tile and the shadow rays of its hits nearly always share one.
template <typename Fn>
__device__ __forceinline__ bool with_uniform_octant(const Slab<false>& s, Fn&& fn) {
    const uint32_t oct = (__float_as_uint(s.ix) >> 31) | (__float_as_uint(s.iy) >> 31) << 1 | (__float_as_uint(s.iz) >> 31) << 2;
    uint32_t r;
    if (!uniform_id(oct, r)) return false;
    switch (r) {
        case 0: fn(std::integral_constant<int, 0>{}); break;
        case 1: fn(std::integral_constant<int, 1>{}); break;
        case 2: fn(std::integral_constant<int, 2>{}); break;
        case 3: fn(std::integral_constant<int, 3>{}); break;
        case 4: fn(std::integral_constant<int, 4>{}); break;
        case 5: fn(std::integral_constant<int, 5>{}); break;
        case 6: fn(std::integral_constant<int, 6>{}); break;
        default: fn(std::integral_constant<int, 7>{}); break;
    }
    return true;
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
template <bool kAnyHit, bool kStats, int kS = kBlock, typename StkT = uint32_t*, bool kRobust = false, int kOct = -1,
          bool kG = false>
__device__ __forceinline__ bool trace(const KParams& P, F3 o, F3 d, StkT stk, Hit& best,
                                      uint32_t& n_pairs, uint32_t& n_tests, bool& overflow) {
    const float tmin = 0.0f;
    float tmax = FLT_MAX;                                           // ray.hpp:17-21
    bool have = false;
    // kOct -2 = the single-frame kernel's generic loop
    constexpr bool kU = CERES_RCP_UNIFORM == 1 || (CERES_RCP_UNIFORM == 2 && kOct == -2);
    if (P.root_leaf_count) {                                          // root is a leaf, :72-73
        if (kStats) n_tests += P.root_leaf_count;
        for (uint32_t k = P.root_leaf_first; k < P.root_leaf_first + P.root_leaf_count; ++k) {
            float t, u, v;
            CERES_COUNT_V(kFTriV, 48);
            if (tri_test<kG, kU>(load_tri(P.tris + k), o, d, tmin, tmax, t, u, v)) {
                best = {k, t, u, v}; have = true;
                if (kAnyHit) return true;
                tmax = t;
            }
        }
        return have;
    }
    const Slab<kRobust> sl = make_slab<kRobust>(o, d);
    if constexpr (!kRobust && kOct == -1 && (CERES_OCTANT_SLAB & 1)) {
        bool r = false;
        if (with_uniform_octant(sl, [&](auto k) {
                r = trace<kAnyHit, kStats, kS, StkT, kRobust, decltype(k)::value, kG>(P, o, d, stk, best, n_pairs, n_tests, overflow);
            }))
            return r;
    }
    if (P.root_box_ok) {                                              // exact early miss (set_root_box)
        float e, x;
        slab_box<kRobust, kOct>(sl, P.root_box[0], P.root_box[1], P.root_box[2], P.root_box[3], P.root_box[4],
                          P.root_box[5], tmin, tmax, e, x);
        if (!(e <= x)) {
            if (kStats) ++n_pairs;                                    // the reference's first step, both children missed
            return false;
        }
    }
    uint32_t sp = 0;
    if (CERES_TRI_SELECT && !kAnyHit) best.slot = kNoSlot;
    // Software-pipelined steps: the next record (near child or stack top) follows from this
    // step's box tests alone (the leaf hits only lower tmax for LATER steps, :89-121), so its
    // load is issued before this step's triangle tests and overlaps them.
    const float4* q = reinterpret_cast<const float4*>(P.pairs);       // pair of the root's children (:81)
    float4 A = q[0], B = q[1], C = q[2];
    uint4 L = reinterpret_cast<const uint4*>(q)[3];
    CERES_COUNT_V(kFBvh2V, 64);
    while (true) {                                                    // :82-123
        if (kStats) ++n_pairs;
        const uint32_t top = stk[(sp ? sp - 1 : 0) * kS];             // popped if this step descends nowhere
        // left bounds A.x A.y | A.z A.w | B.x B.y ; right bounds B.z B.w | C.x C.y | C.z C.w
        float le, lx, re, rx;
        slab_box<kRobust, kOct>(sl, A.x, A.y, A.z, A.w, B.x, B.y, tmin, tmax, le, lx);
        slab_box<kRobust, kOct>(sl, B.z, B.w, C.x, C.y, C.z, C.w, tmin, tmax, re, rx);
        const bool hit_l = le <= lx, hit_r = re <= rx;
        const bool go_l = hit_l && !L.x, go_r = hit_r && !L.z;
        // the three cases as selects: the far child is written to slot sp every step (a free slot
        // unless this step pushes; the LDS stack has stack_entries + 1 slots), the stack top was
        // read at the start of the step, only the exit branches
        const bool both = go_l && go_r, none = !go_l && !go_r;
        const bool swap = le > re;                                    // near first, ties left (:109-115)
        const bool done = none && sp == 0;                            // :118-121
        const uint32_t near = both ? (swap ? L.w : L.y) : (go_l ? L.y : L.w);   // :115-117
        const uint32_t nxt = none ? top : near;
        if (kStats || !CERES_TRUST_STACK_BOUND) {
            overflow |= both && sp >= P.stack_entries;
            stk[(sp < P.stack_entries ? sp : P.stack_entries) * kS] = swap ? L.y : L.w;
            sp = both ? (sp < P.stack_entries ? sp + 1 : sp) : (none ? (sp ? sp - 1 : 0) : sp);
        } else {
            // the scene's stack bound is exact (a push per level descended: at most depth - 1
            // entries, stack_entries = depth), so the production kernels skip the clamps; the
            // stats kernels (records, statistics: every parity test config) keep the check.  The
            // production kernels still REPORT a broken bound (round 6) through
            // a guard slot around the call (guarded_trace).
            stk[sp * kS] = swap ? L.y : L.w;
            sp = sp + (both ? 1u : 0u) - (none ? 1u : 0u);            // none && sp == 0 exits (done)
        }
        // leaves of this step, left then right (intersect_leaf on each, :89-107), one loop so a
        // wavefront runs max(left + right) trips rather than max(left) + max(right)
        // (one counter over the left leaf's then the right leaf's triangles: a single loop bound)
        const uint32_t nl = hit_l ? L.x : 0u, nr = hit_r ? L.z : 0u;
        const uint32_t n_leaf = nl + nr, k2 = L.w - nl;
        if (kStats) n_tests += n_leaf;
        float4 nA, nB, nC;                                            // undefined for done lanes
        uint4 nL;
        if (CERES_LOAD_ALWAYS && kOct != -2) {                        // (not the single-frame kernel: measured +1.4 % there)
            // every lane loads (a done lane the root's pair, cached), so no exec-mask branch
            const float4* nq = reinterpret_cast<const float4*>(P.pairs + (done ? 0u : nxt));
            nA = nq[0]; nB = nq[1]; nC = nq[2]; nL = reinterpret_cast<const uint4*>(nq)[3];
            CERES_COUNT_V(kFBvh2V, 64);
        } else if (!done) {
            const float4* nq = reinterpret_cast<const float4*>(P.pairs + nxt);
            nA = nq[0]; nB = nq[1]; nC = nq[2]; nL = reinterpret_cast<const uint4*>(nq)[3];
            CERES_COUNT_V(kFBvh2V, 64);
        }
        for (uint32_t j = 0; j < n_leaf; ++j) {
            const uint32_t idx = (j < nl ? L.y : k2) + j;
            float t, u, v;
            if (CERES_TRI_SELECT && !kAnyHit) {                          // closest hit: selects, no branch
                // (no separate "have" flag: a boolean carried through the loop costs exec-mask
                // merges at every join; best.slot starts at kNoSlot instead)
                const bool h = tri_test_u<kG, kU>(P.tris, idx, o, d, tmin, tmax, t, u, v);
                best.slot = h ? idx : best.slot; best.t = h ? t : best.t;
                best.u = h ? u : best.u; best.v = h ? v : best.v;
                tmax = h ? t : tmax;
                continue;
            }
            if (tri_test_u<kG, kU>(P.tris, idx, o, d, tmin, tmax, t, u, v)) {
                best = {idx, t, u, v}; have = true;
                if (kAnyHit) return true;
                tmax = t;
            }
        }
        if (done) break;
        A = nA; B = nB; C = nC; L = nL;
    }
    if (CERES_TRI_SELECT && !kAnyHit) return best.slot != kNoSlot;
    return have;
}

// trace() with a stack guard (round 6; CERES_STACK_GUARD: compiled into the
// diagnostic build, libceres_hip_count.so).  Without the stats kernels' clamps
// (CERES_TRUST_STACK_BOUND), a step writes the far child to slot sp, and with the exact bound
// sp <= depth - 1 = stack_entries - 1, so slot stack_entries is never written unless the bound is
// broken -- and a walk that overruns it must pass through it (sp moves by one per step).  The slot
// holds a value no node index takes (stack_guard); a changed guard sets the overflow flag, hence
// the error word.  One LDS write and one read per ray -- measured in the product: 16-frame batches
// x 8 streams C3 +1.9 %, C5 +6.5 % (one more VGPR spill; the 24-bit-stack batch kernel 80 -> 84
// VGPRs, a wave per SIMD less; profiles/r06/ab_guard), so the product relies on the exact bound,
// and bench.py checks every timed view with the stats kernels (clamps + flag) and with this
// build's guard before it times them.
template <bool kStats, int kS, typename StkT, bool kRobust, int kOct, bool kG>
__device__ __forceinline__ bool guarded_trace(const KParams& P, F3 o, F3 d, StkT stk, Hit& best, uint32_t& n_pairs,
                                              uint32_t& n_tests, bool& overflow) {
    constexpr bool kGuard = !kStats && CERES_TRUST_STACK_BOUND && CERES_STACK_GUARD;
    const uint32_t slot = P.stack_entries * kS;
    if (kGuard) stk[slot] = stack_guard<StkT>();
    const bool hit = trace<false, kStats, kS, StkT, kRobust, kOct, kG>(P, o, d, stk, best, n_pairs, n_tests, overflow);
    if (kGuard) overflow |= uint32_t(stk[slot]) != stack_guard<StkT>();
    return hit;
}

// Any-hit traversal of the shadow BVH4 (build_shadow_bvh4): result-identical to trace<true>
// (see the equivalence argument there).  Per step: one 128-B record, four slab tests with the
// same fma/min/max restatement as trace(), the triangles of every passing leaf, then descend
// into one passing inner child (the first) and push the others.  The
// order only changes how soon an occluder is found, never whether one is.
struct N4 { float4 lx, hx, ly, hy, lz, hz; uint4 ch; };   // ch: packed child words (Node4::child)
__device__ __forceinline__ N4 load_n4(const Node4* n) {
    const float4* q = reinterpret_cast<const float4*>(n);
    const uint4* u = reinterpret_cast<const uint4*>(n);
    return {q[0], q[1], q[2], q[3], q[4], q[5], u[6]};
}
__device__ __forceinline__ uint32_t n4_count(uint32_t w) { return w & kNode4MaxCount; }
__device__ __forceinline__ uint32_t n4_first(uint32_t w) { return w >> kNode4CountBits; }
// node `cur` for the active lanes: one scalar fetch when they all visit the same node
__device__ __forceinline__ N4 load_n4_u(const Node4* nodes, uint32_t cur) {
    uint32_t r;
    if (uniform_id(cur, r)) {
        CERES_COUNT_S(kFBvh4S, 112);
        const Node4* q = nodes + r;
        return {sload_f4(q, 0), sload_f4(q, 1), sload_f4(q, 2), sload_f4(q, 3), sload_f4(q, 4), sload_f4(q, 5),
                sload_u4(q, 6)};
    }
    CERES_COUNT_V(kFBvh4V, 112);
    return load_n4(nodes + cur);
}
// compressed node (CERES_MODE_QBVH4, ceres_types.hpp QNode4): bound = fma(byte, scale, origin), the
// formula quantize_nodes4 checks on the host (the decoded box contains the exact one)
__device__ __forceinline__ float4 qdecode(uint32_t w, float scale, float origin) {
    return make_float4(__builtin_fmaf(float(w & 0xffu), scale, origin), __builtin_fmaf(float((w >> 8) & 0xffu), scale, origin),
                       __builtin_fmaf(float((w >> 16) & 0xffu), scale, origin), __builtin_fmaf(float(w >> 24), scale, origin));
}
__device__ __forceinline__ N4 load_q4_u(const QNode4* nodes, uint32_t cur) {
    float4 a, b;
    uint4 c, d;
    uint32_t r;
    if (uniform_id(cur, r)) {
        CERES_COUNT_S(kFBvh4S, 64);
        const QNode4* q = nodes + r;
        a = sload_f4(q, 0); b = sload_f4(q, 1); c = sload_u4(q, 2); d = sload_u4(q, 3);
    } else {
        CERES_COUNT_V(kFBvh4V, 64);
        const float4* q = reinterpret_cast<const float4*>(nodes + cur);
        a = q[0]; b = q[1];
        c = reinterpret_cast<const uint4*>(q)[2]; d = reinterpret_cast<const uint4*>(q)[3];
    }
    // a = {ox, oy, oz, sx}, b = {sy, sz, qlx, qhx}, c = {qly, qhy, qlz, qhz}, d = child words
    return {qdecode(__float_as_uint(b.z), a.w, a.x), qdecode(__float_as_uint(b.w), a.w, a.x),
            qdecode(c.x, b.x, a.y), qdecode(c.y, b.x, a.y), qdecode(c.z, b.y, a.z), qdecode(c.w, b.y, a.z), d};
}
template <bool kQ>
__device__ __forceinline__ N4 load_shadow_node(const KParams& P, uint32_t cur) {
    if constexpr (kQ) return load_q4_u(P.qnodes4, cur);
    else return load_n4_u(P.nodes4, cur);
}
__device__ __forceinline__ float pick(float4 v, uint32_t c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }
__device__ __forceinline__ uint32_t pick(uint4 v, uint32_t c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }

template <bool kStats, int kS = kBlock, typename StkT = uint32_t*, bool kRobust = false, bool kQ = false, int kOct = -1,
          bool kG = false>
__device__ __forceinline__ bool trace_any4(const KParams& P, F3 o, F3 d, StkT stk, uint32_t& n_pairs,
                                           uint32_t& n_tests, bool& overflow) {
    const float tmin = 0.0f, tmax = FLT_MAX;
    if (P.root_leaf_count) {
        Hit h;
        return trace<true, kStats, kS, StkT, kRobust, -1, kG>(P, o, d, stk, h, n_pairs, n_tests, overflow);
    }
    const Slab<kRobust> sl = make_slab<kRobust>(o, d);
    if constexpr (!kRobust && kOct == -1 && (CERES_OCTANT_SLAB & 2)) {
        bool r = false;
        if (with_uniform_octant(sl, [&](auto k) {
                r = trace_any4<kStats, kS, StkT, kRobust, kQ, decltype(k)::value, kG>(P, o, d, stk, n_pairs, n_tests, overflow);
            }))
            return r;
    }
    uint32_t sp = 0, cur = 0;
    while (true) {
        if (kStats) ++n_pairs;
        float e[4];
        uint32_t leaf_mask = 0, inner_mask = 0;
        // the four slab tests of a record; the wave-uniform record gets its own copy that reads
        // the scalar-loaded bounds from SGPRs (CERES_SPLIT_UNIFORM: no 28 v_mov to join the
        // vector path)
        auto classify = [&](const float4& LX, const float4& HX, const float4& LY, const float4& HY, const float4& LZ,
                            const float4& HZ, const uint4& CH) {
            const float lx[4] = {LX.x, LX.y, LX.z, LX.w}, hx[4] = {HX.x, HX.y, HX.z, HX.w};
            const float ly[4] = {LY.x, LY.y, LY.z, LY.w}, hy[4] = {HY.x, HY.y, HY.z, HY.w};
            const float lz[4] = {LZ.x, LZ.y, LZ.z, LZ.w}, hz[4] = {HZ.x, HZ.y, HZ.z, HZ.w};
            const uint32_t chw[4] = {CH.x, CH.y, CH.z, CH.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float x;
                slab_box<kRobust, kOct>(sl, lx[c], hx[c], ly[c], hy[c], lz[c], hz[c], tmin, tmax, e[c], x);
                const bool hit = e[c] <= x && chw[c] != kNode4Empty;
                const bool leaf = n4_count(chw[c]) != 0;
                leaf_mask |= (hit && leaf) ? (1u << c) : 0u;
                inner_mask |= (hit && !leaf) ? (1u << c) : 0u;
            }
        };
        uint4 CH;
        uint32_t rc;
        if (!kQ && CERES_SPLIT_UNIFORM && uniform_id(cur, rc)) {
            CERES_COUNT_S(kFBvh4S, 112);
            const Node4* q = P.nodes4 + rc;
            CH = sload_u4(q, 6);
            classify(sload_f4(q, 0), sload_f4(q, 1), sload_f4(q, 2), sload_f4(q, 3), sload_f4(q, 4), sload_f4(q, 5), CH);
            __asm__ volatile("; uniform BVH4 record" ::);               // keeps this copy from being merged with the other
        } else {
            if (!kQ && CERES_SPLIT_UNIFORM) CERES_COUNT_V(kFBvh4V, 112);
            const N4 nd = (!kQ && CERES_SPLIT_UNIFORM) ? load_n4(P.nodes4 + cur) : load_shadow_node<kQ>(P, cur);
            CH = nd.ch;
            classify(nd.lx, nd.hx, nd.ly, nd.hy, nd.lz, nd.hz, CH);
        }
        const uint32_t cnt[4] = {n4_count(CH.x), n4_count(CH.y), n4_count(CH.z), n4_count(CH.w)};
        const uint32_t fst[4] = {n4_first(CH.x), n4_first(CH.y), n4_first(CH.z), n4_first(CH.w)};
        // triangles of every passing leaf child, as one flattened loop (wave-coherent trip count)
        uint32_t k = 0, k_end = 0;
        while (true) {
            if (k >= k_end) {
                if (!leaf_mask) break;
                const uint32_t c = __builtin_ctz(leaf_mask);
                leaf_mask &= leaf_mask - 1;
                k = c == 0 ? fst[0] : c == 1 ? fst[1] : c == 2 ? fst[2] : fst[3];
                k_end = k + (c == 0 ? cnt[0] : c == 1 ? cnt[1] : c == 2 ? cnt[2] : cnt[3]);
                if (kStats) n_tests += k_end - k;
            }
            float t, u, v;
            if (tri_test_u<kG, CERES_RCP_UNIFORM == 1>(P.tris, k, o, d, tmin, tmax, t, u, v)) return true;
            ++k;
        }
        if (inner_mask) {
            // one passing inner child next; the others go on the stack
            // (any order gives the same answer; the nearest-first choice costs its selects in every
            // step and the batch regime is issue-bound, so batches take the first passing child)
            const uint32_t best = __builtin_ctz(inner_mask);
            uint32_t rest = inner_mask & ~(1u << best);
            if (sp + __builtin_popcount(rest) > P.shadow_stack_entries) { overflow = true; return false; }
            while (rest) {
                const uint32_t c = __builtin_ctz(rest);
                rest &= rest - 1;
                stk[sp * kS] = c == 0 ? fst[0] : c == 1 ? fst[1] : c == 2 ? fst[2] : fst[3];
                ++sp;
            }
            cur = best == 0 ? fst[0] : best == 1 ? fst[1] : best == 2 ? fst[2] : fst[3];
        } else {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * kS];
        }
    }
    return false;
}

// Any-hit of a whole wavefront's shadow rays as ONE masked packet over the shadow BVH4 (batch
// kernel).  The 8x8 tile's shadow rays start at neighbouring hit points and run to the same sun,
// so they reach nearly the same nodes: the wavefront walks the union of their paths once, every
// record and triangle read through the scalar cache (one wave-uniform s_load, no vector-memory
// traffic), each lane testing its own ray, and the lane masks (a v_cmp result IS the mask)
// decide where to go.  A ray's answer is "some leaf triangle it reaches is hit" -- every leaf
// whose box chain its ray passes is still tested for it (its lane is in the mask of every node
// on that chain, the slab test being the same per-lane arithmetic as trace_any4's) and the order
// of the tests never changes an any-hit result (render.hpp:137-139 uses only the boolean), so the
// occluded set equals trace_any4's bit for bit.  A lane leaves the masks once it is occluded.
// The stack of (node, mask) entries is wave-uniform: entry k lives in lane k of three VGPRs
// (a select on lane == sp / v_readlane, no memory); it holds at most shadow_stack_entries (the most pushes
// along any root-leaf path, build_shadow_bvh4) -- the host only takes this path when <= 64.
// `act`: lanes with a shadow ray; their o / slab in every lane (others: copies of an active one).
template <int kOct, bool kG>
__device__ __forceinline__ uint64_t packet_any4(const KParams& P, const Slab<false>& sl, F3 o, F3 d, uint64_t act,
                                                uint32_t lane) {
    constexpr float tmin = 0.0f, tmax = FLT_MAX;
    typedef float F2s __attribute__((ext_vector_type(2)));
    const F2s IX2{sl.ix, sl.ix}, IY2{sl.iy, sl.iy}, IZ2{sl.iz, sl.iz};   // CERES_PK_PACKET splats
    const F2s SX2{sl.sx, sl.sx}, SY2{sl.sy, sl.sy}, SZ2{sl.sz, sl.sz};
    uint64_t occ = 0, m = act;
    uint32_t cur = 0, sp = 0;
    int s_node = 0, s_lo = 0, s_hi = 0;                               // stack entry k in lane k
    while (true) {
        const Node4* q = P.nodes4 + cur;
        CERES_COUNT_S(kFBvh4S, 116);
        const float4 LX = sload_f4(q, 0), HX = sload_f4(q, 1), LY = sload_f4(q, 2), HY = sload_f4(q, 3);
        const float4 LZ = sload_f4(q, 4), HZ = sload_f4(q, 5);
        const uint4 CH = sload_u4(q, 6);
        const float lx[4] = {LX.x, LX.y, LX.z, LX.w}, hx[4] = {HX.x, HX.y, HX.z, HX.w};
        const float ly[4] = {LY.x, LY.y, LY.z, LY.w}, hy[4] = {HY.x, HY.y, HY.z, HY.w};
        const float lz[4] = {LZ.x, LZ.y, LZ.z, LZ.w}, hz[4] = {HZ.x, HZ.y, HZ.z, HZ.w};
        const uint32_t chw[4] = {CH.x, CH.y, CH.z, CH.w};
        const uint32_t nleaf = sload_u32(&q->nleaf);
        // per child the lanes whose ray passes its box; children 0..nleaf-1 are leaves, the rest
        // inner or empty (node4_leaves_first).  An empty slot holds the inverted infinite box, which
        // the octant-selected slab test always fails (entry +inf, exit -inf), so no empty-slot test.
        uint64_t hm[4];
        if constexpr (CERES_PK_PACKET) {
            // the same fmas two children at a time (v_pk_fma_f32: children 0-1 and 2-3 of one bound row
            // with the lane's splatted inverse direction / offset; each half is the scalar fma bit for bit)
            typedef float F2v __attribute__((ext_vector_type(2)));
            auto pk = [&](float a, float b, const F2v& i2, const F2v& s2) { return __builtin_elementwise_fma(F2v{a, b}, i2, s2); };
            const F2v lx01 = pk(LX.x, LX.y, IX2, SX2), lx23 = pk(LX.z, LX.w, IX2, SX2);
            const F2v hx01 = pk(HX.x, HX.y, IX2, SX2), hx23 = pk(HX.z, HX.w, IX2, SX2);
            const F2v ly01 = pk(LY.x, LY.y, IY2, SY2), ly23 = pk(LY.z, LY.w, IY2, SY2);
            const F2v hy01 = pk(HY.x, HY.y, IY2, SY2), hy23 = pk(HY.z, HY.w, IY2, SY2);
            const F2v lz01 = pk(LZ.x, LZ.y, IZ2, SZ2), lz23 = pk(LZ.z, LZ.w, IZ2, SZ2);
            const F2v hz01 = pk(HZ.x, HZ.y, IZ2, SZ2), hz23 = pk(HZ.z, HZ.w, IZ2, SZ2);
            const float ax[4] = {lx01.x, lx01.y, lx23.x, lx23.y}, bx[4] = {hx01.x, hx01.y, hx23.x, hx23.y};
            const float ay[4] = {ly01.x, ly01.y, ly23.x, ly23.y}, by[4] = {hy01.x, hy01.y, hy23.x, hy23.y};
            const float az[4] = {lz01.x, lz01.y, lz23.x, lz23.y}, bz[4] = {hz01.x, hz01.y, hz23.x, hz23.y};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                // the octant picks each axis's entry / exit slab (slab_box<false, kOct>)
                const float nx = (kOct & 1) ? bx[c] : ax[c], fx = (kOct & 1) ? ax[c] : bx[c];
                const float ny = (kOct & 2) ? by[c] : ay[c], fy = (kOct & 2) ? ay[c] : by[c];
                const float nz = (kOct & 4) ? bz[c] : az[c], fz = (kOct & 4) ? az[c] : bz[c];
                const float e = fmaxf(nx, fmaxf(ny, fmaxf(nz, tmin)));
                const float x = fminf(fx, fminf(fy, fminf(fz, tmax)));
                hm[c] = __ballot(e <= x) & m;
            }
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float e, x;
                slab_box<false, kOct>(sl, lx[c], hx[c], ly[c], hy[c], lz[c], hz[c], tmin, tmax, e, x);
                hm[c] = __ballot(e <= x) & m;
            }
        }
        // triangles of every passing leaf child, for the lanes that reach it and are not yet occluded
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (uint32_t(c) >= nleaf) break;
            uint64_t lm = hm[c] & ~occ;
            if (!lm) continue;
            const uint32_t n = n4_count(chw[c]);
            // do-while (n > 0 and lm != 0 on entry), the hit mask straight from the compares: two plain
            // exits, no combined predicate (round 5 A/B: batches -0.3..-1.2 %)
            const Tri48* tp = P.tris + n4_first(chw[c]);
            uint32_t left = n;
            while (true) {
                CERES_COUNT_S(kFTriS, 48);
                const float4 a = sload_f4(tp, 0), b = sload_f4(tp, 1), g = sload_f4(tp, 2);
                // all 48 B in flight before the first use (one scalar-load wait per triangle, not two)
                __asm__ volatile("" ::"s"(a.x), "s"(b.x), "s"(g.x));
                const TriV tr{{a.x, a.y, a.z}, {a.w, b.x, b.y}, {b.z, b.w, g.x}, {g.y, g.z, g.w}};
                occ |= tri_mask<kG, CERES_RCP_UNIFORM == 1>(tr, o, d, tmin, tmax) & lm;
                lm &= ~occ;
                if (!lm) break;
                if (--left == 0) break;
                ++tp;
            }
        }
        // one passing inner child next (the first), the others onto the stack with their masks
        // (the child with the most lanes first measured +4.5 % in batches)
        int nxt = -1;
        uint64_t nm = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (uint32_t(c) < nleaf) continue;
            const uint64_t mm = hm[c] & ~occ;
            if (!mm) continue;
            if (nxt < 0) { nxt = c; nm = mm; continue; }
            const bool mine = lane == sp;                              // a write into lane sp
            s_node = mine ? int(n4_first(chw[c])) : s_node;
            s_lo = mine ? int(uint32_t(mm)) : s_lo;
            s_hi = mine ? int(uint32_t(mm >> 32)) : s_hi;
            ++sp;
        }
        if (nxt >= 0) {
            cur = n4_first(chw[nxt]);
            m = nm;
            continue;
        }
        m = 0;
        while (sp) {                                                    // pop until a mask has live lanes
            --sp;
            m = (uint64_t(uint32_t(__builtin_amdgcn_readlane(s_hi, int(sp)))) << 32 |
                 uint32_t(__builtin_amdgcn_readlane(s_lo, int(sp)))) & ~occ;
            if (m) { cur = uint32_t(__builtin_amdgcn_readlane(s_node, int(sp))); break; }
        }
        if (!m) return occ;
    }
}

__device__ __forceinline__ uint8_t quantize(float x) {               // static.cpp:141-143
    const float a = x * 255;
    const float m = (255.0f < a) ? 255.0f : a;                       // std::min(a, 255)
    const float q = (m < 0.0f) ? 0.0f : m;                           // std::max(m, 0)
    return static_cast<uint8_t>(static_cast<int>(q));
}

// Pixel (frame f, local row lr, column i): float RGB at batch pixel (f*rows + lr)*W + i with
// row 0 at the bottom (render.hpp:107); RGB8 PPM body with local row lr stored at row
// rows-1-lr of its frame (static.cpp:137, rows written top-down).
__device__ __forceinline__ void store_pixel(const KParams& P, uint32_t f, uint32_t lr, uint32_t i, float c0, float c1,
                                            float c2) {
    const size_t frame_base = size_t(f) * P.local_rows;
    CERES_COUNT_V(kFStoreV, (P.pixels ? 12u : 0u) + (P.rgb8 ? 3u : 0u));
    if (P.pixels) {
        float* q = P.pixels + 3 * ((frame_base + lr) * P.W + i);
        q[0] = c0; q[1] = c1; q[2] = c2;
    }
    if (P.rgb8) {
        uint8_t* q = P.rgb8 + 3 * ((frame_base + (P.local_rows - 1 - lr)) * P.W + i);
        q[0] = quantize(c0); q[1] = quantize(c1); q[2] = quantize(c2);
    }
}

// kBands: the ceres_tiling.bands instantiations (frame f renders band (rank + f) mod world); a
// separate instantiation, so the row-block kernels carry none of its registers (a runtime flag cost
// 1 VGPR and 4-6 % of a C3 / C4 / C5 batch, profiles/r06/bands/ab_runtime_flag)
template <bool kBands = false>
__device__ __forceinline__ uint32_t global_row(const KParams& P, uint32_t f, uint32_t lr) {
    if (P.world == 1) return lr;                                      // one rank: local rows are the frame's rows
    if constexpr (kBands) {                                           // the frame's band: (rank + f) mod world
        // f is wave-uniform: a scalar multiply-high by the host's magic number instead of an
        // integer division per call (the division cost C4's band launches ~12 % at N = 8, where
        // most tiles are culled and cheap)
        const uint32_t x = P.rank + f, q = __umulhi(x, P.band_magic);
        return (x - q * P.world) * P.row_block + lr;
    }
    return ((lr / P.row_block) * P.world + P.rank) * P.row_block + lr % P.row_block;
}

// Primary ray direction of pixel (i, j) of frame f, render.hpp:109-111 (GCC: dir + fma(iv, v, iu u)).
template <bool kG = false>
__device__ __forceinline__ F3 primary_dir(const KParams& P, uint32_t f, uint32_t i, uint32_t j) {
    const float u = 2 * (float(i) + 0.5f) / float(P.W) - 1.0f;       // render.hpp:109-110 (IEEE division)
    const float v = 2 * (float(j) + 0.5f) / float(P.H) - 1.0f;
    const FrameCam& c = P.cam[f];
    F3 a;
    if constexpr (kG)
        a = F3{c.dir[0] + __builtin_fmaf(c.iv[0], v, c.iu[0] * u), c.dir[1] + __builtin_fmaf(c.iv[1], v, c.iu[1] * u),
               c.dir[2] + __builtin_fmaf(c.iv[2], v, c.iu[2] * u)};
    else a = f3(c.iu) * u + f3(c.iv) * v + f3(c.dir);
    return kG ? normalizeG<kG>(a) : normalize(a);
}

// Exact background cull (round 5).  A tile whose every pixel's primary ray provably misses the
// root box is stored as misses (render.hpp:116-117: RGB 0) without tracing: the root-box pre-test
// (set_root_box) already shows that such a ray fails both of the root's children in the
// reference's first step (single_ray_traverser.hpp:81-123), so the pixel, the ray count and the
// hit count are the reference's.  The host proves per frame which pixels' rays cannot reach the
// box (cull_rect: the image of the root box, expanded, is inside a pixel rectangle) and passes
// that rectangle in the kernel arguments; a tile is culled when none of its pixels lies inside.
// Stats / records kernels never cull (their per-ray counters count the root step).
__device__ __forceinline__ bool tile_misses_root(const KParams& P, uint32_t f, bool active, uint32_t i, uint32_t j) {
    const CullRect& r = P.cull_rect[f];
    const bool out = i < r.i0 || i > r.i1 || j < r.j0 || j > r.j1;
    return __ballot(active && !out) == 0;
}

// Hit point + self-intersection offset, render.hpp:127-133 (p1() = p0 - e1, p2() = p0 + e2).
// GCC: fma(n, scale, fma(w, p2, fma(v, p1, u p0))) per component.
template <bool kG>
__device__ __forceinline__ F3 hit_point(const TriV& tr, F3 normal, float hu, float hv) {
    const F3 p1 = tr.p0 - tr.e1, p2 = tr.p0 + tr.e2;
    const float scale = -0.00001;
    const float w = 1 - hu - hv;
    if constexpr (kG) {
        auto c = [&](float p0, float q1, float q2, float n) {
            return __builtin_fmaf(n, scale, __builtin_fmaf(w, q2, __builtin_fmaf(hv, q1, hu * p0)));
        };
        return {c(tr.p0.x, p1.x, p2.x, normal.x), c(tr.p0.y, p1.y, p2.y, normal.y), c(tr.p0.z, p1.z, p2.z, normal.z)};
    } else {
        F3 p = tr.p0 * hu + p1 * hv + p2 * w;
        return p + normal * scale;
    }
}

// smooth_shading, render.hpp:46-84 (pow in double: std::pow(float, int) promotes).  GCC fuses
// lambertian's sum like dot "A", amb + 0.5 lam into fma(lam, 0.5, amb) and each channel's
// (amb + diffuse) * k + specular into fma(amb + diffuse, k, specular); c[] += w * clamp stays unfused.
template <bool kG = false>
__device__ __forceinline__ void shade(F3 sun_line, const float* nrm, F3 view, float u, float v, float c[3]) {
    c[0] = c[1] = c[2] = 0.0f;
    const float amb = 0.2;
    const F3 vneg = view * -1.0f;
    const float w[3] = {u, v, 1 - u - v};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const F3 N{nrm[3 * k], nrm[3 * k + 1], nrm[3 * k + 2]};
        const float lam = kG ? fabsf(dotA<true>(sun_line, N)) : fabsf(sun_line.x * N.x + sun_line.y * N.y + sun_line.z * N.z);
        const float spec = 0.8f * pow24f(dotA<kG>(N, normalizeG<kG>(sun_line + vneg)));   // == (float)std::pow(double, 24)
        const float base = kG ? __builtin_fmaf(lam, 0.5f, amb) : amb + 0.5f * lam;
        auto clamp01 = [](float x) { return (x < 0.f) ? 0.f : (1.f < x) ? 1.f : x; };   // std::clamp
        auto ch = [&](float k) { return kG ? __builtin_fmaf(base, k, spec) : base * k + spec; };
        c[0] += w[k] * clamp01(ch(0.5f));
        c[1] += w[k] * clamp01(ch(0.0f));
        c[2] += w[k] * clamp01(ch(0.8f));
    }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// ---------------------------------------------------------------- primary-only kernel
// The "primary rays only" mode (C2; pixel = |normalize(tri.n)|, render.hpp:123-125).
// grid.x: 16-pixel column blocks; grid.y: frames x 16-row blocks of this rank's rows.  The
// four wavefronts of a workgroup take the 2x2 8x8 tiles of its 16x16 pixels (row-major lanes:
// C2's rays are coherent already, the Morton lane order measured +2.5 % on solo frames here).
template <bool kStats, bool kRobust, bool kG>
__global__ __launch_bounds__(kBlock) void ceres_primary(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* stk = lds + tid;                                       // [entries][kBlock]
    const uint32_t f = blockIdx.y / P.row_blocks_per_frame;          // workgroup-uniform frame
    const uint32_t by = blockIdx.y - f * P.row_blocks_per_frame;
    const uint32_t lx = lane & 7, ly = lane >> 3;
    const uint32_t i = blockIdx.x * 16 + (wave & 1) * 8 + lx;
    const uint32_t lr = by * 16 + (wave >> 1) * 8 + ly;
    const bool active = i < P.W && lr < P.local_rows;
    const uint32_t px = (f * P.local_rows + lr) * P.W + i;          // batch pixel (< 2^32, host-checked)
    bool hit = false;
    Hit h{0, 0.f, 0.f, 0.f};
    uint32_t n_pairs = 0, n_tests = 0;
    bool overflow = false;
    const bool culled = !kStats && P.cull && tile_misses_root(P, f, active, i, global_row(P, f, lr));
    if (culled) {
        if (active) store_pixel(P, f, lr, i, 0.f, 0.f, 0.f);        // render.hpp:116-117, every pixel a miss
    } else if (active) {
        const F3 view = primary_dir<kG>(P, f, i, global_row(P, f, lr));
        hit = guarded_trace<kStats, kBlock, uint32_t*, kRobust, -1, kG>(P, f3(P.cam[f].eye), view, stk, h, n_pairs, n_tests,
                                                                      overflow);
        if (P.rec_prim) {
            P.rec_prim[px] = hit ? int32_t(P.orig[h.slot]) : -1;
            P.rec_tuv[3 * size_t(px)] = hit ? h.t : 0.f;
            P.rec_tuv[3 * size_t(px) + 1] = hit ? h.u : 0.f;
            P.rec_tuv[3 * size_t(px) + 2] = hit ? h.v : 0.f;
            P.rec_shadow[px] = -1;
        }
        if (!hit) {
            store_pixel(P, f, lr, i, 0.f, 0.f, 0.f);                 // render.hpp:116-117
        } else {                                                     // render.hpp:123-125
            CERES_COUNT_V(kFShadeV, 48);
            const F3 normal = normalizeG<kG>(load_tri(P.tris + h.slot).n);
            store_pixel(P, f, lr, i, fabsf(normal.x), fabsf(normal.y), fabsf(normal.z));
        }
    }
    const uint32_t wave_id = (blockIdx.y * gridDim.x + blockIdx.x) * (kBlock / 64) + wave;
    const uint32_t shard = wave_id % kShards;
    const uint32_t nh = __popcll(__ballot(hit));
    if (lane == 0 && nh) atomicAdd(&P.shards[shard].hits, (unsigned long long)nh);
    if (kStats) {
        const uint32_t wp = wave_sum(n_pairs), wt = wave_sum(n_tests);
        if (lane == 0) {
            atomicAdd(&P.shards[shard].pairs, (unsigned long long)wp);
            atomicAdd(&P.shards[shard].tests, (unsigned long long)wt);
        }
    }
    if (overflow) atomicOr(&P.shards[shard].error, 1u);
}

#ifndef CERES_LEAN_WRITES
// 1: the 7-wave batch kernel keeps no per-wavefront scratch spill (a lane's pixel decoded again after
// the traversals, the culled tiles' zeros made at the store).  Its spill, written once per wavefront
// and evicted to DRAM, is the C3 launch's write excess over the framebuffers: WRITE_SIZE 619 -> 524 MB
// per 16-frame launch, but C3 -1.9 %, bunny 1080p -1.9 % (profiles/r06/spill), so off by default
#define CERES_LEAN_WRITES 0
#endif
#ifndef CERES_FUSED_MINW16
#define CERES_FUSED_MINW16 7     // waves per SIMD the compiler budgets VGPRs for, 16-bit-stack scenes, batch kernel (with shadow packets, A/A/B/B: 7 waves / 72 VGPRs beat 6 / 80 by 2.6 % on C3, bunny -0.5 %, dragon 4096^2 +-0)
#endif
#ifndef CERES_FUSED_MINW16_TPW4
#define CERES_FUSED_MINW16_TPW4 6   // ... and the 4-tiles-per-wave batch kernel (frames outside 1-4 Mpixel: C1, C4): 6 waves /
                                    // 80 VGPRs, no spills (round 6 A/B, 16-frame batches x 8 streams: dragon 4096^2 -3.1 %,
                                    // bunny 640 +-0; profiles/r06/minw_tpw4)
#endif
#ifndef CERES_FUSED_MINW16_SOLO
#define CERES_FUSED_MINW16_SOLO 7  // ... and the work-stealing single-frame kernel (72 VGPRs, no VGPR spill: dragon 4096^2 -4 %, bunny -1.5 %, C3 +-1 %)
#endif
#ifndef CERES_FUSED_MINW32
#define CERES_FUSED_MINW32 1     // ... and 32-bit-stack scenes (1 = no constraint)
#endif
#ifndef CERES_STACK16
#define CERES_STACK16 1          // 16-bit LDS stack entries for scenes with < 65536 pairs and BVH4 nodes
#endif
#ifndef CERES_STACK24
#define CERES_STACK24 1          // 24-bit LDS stack entries for scenes with < 2^24 pairs and BVH4 nodes
#endif
constexpr size_t kTileShuffleWindow = 64;   // tiles per shuffled window of the centre-first order (XCD balance)

// ---------------------------------------------------------------- work-stealing shadow phase
// One-frame launches (latency-bound: a frame ends when its slowest tiles end) trace a
// wavefront's shadow rays with the work shared among its lanes:
// a shadow ray is any-hit, so the subtrees left on a ray's stack may be traversed in any
// order and by any lane, and the ray is occluded iff ANY of those pieces finds a triangle hit
// (the same set of leaf tests as trace_any4, see build_shadow_bvh4).  After every step, lanes
// that have finished their own piece take the BOTTOM entry (the largest pending subtree) of a
// lane that still has stacked subtrees, together with that ray's origin / inverse direction
// (cross-lane shuffles); a hit marks the owning lane's pixel occluded in LDS and cancels the
// ray's other pieces.  A single long ray -- 60+ BVH4 steps on C3, which set the duration of a
// one-ray-per-lane frame -- is thus traversed by up to 64 lanes at once.  Pixels are shaded
// together once the wavefront has no work left.  Stacks are per-lane ring buffers in LDS.
struct RayWork {
    F3 o, d;
    float ix, iy, iz, sx, sy, sz;    // Slab<kRobust> constants of the ray
};
template <bool kRobust>
__device__ __forceinline__ Slab<kRobust> slab_of(const RayWork& w) { return {w.ix, w.iy, w.iz, w.sx, w.sy, w.sz, w.o}; }

// LDS scratch of the work-stealing loop, per workgroup
template <int kS>
struct StealLdsT {
    uint32_t blocked[kS];            // pixel of lane tid occluded (set by any piece of its ray)
    uint32_t mail[kS];               // stolen node, by thief rank within the wavefront
    uint32_t from[kS];               // donor lane, by thief rank
};

// Paired framebuffer stores of the batch kernel (round 6; CERES_PAIR_STORES).  A
// wavefront of a batch takes consecutive tiles of the tile order, and consecutive tiles of the
// Morton / row-run orders are horizontal neighbours (tiles 2k and 2k + 1 differ in the lowest x
// bit), so each 8-pixel row of an even tile shares a 64-B sector with the next tile's row: floats
// at 96 B per tile row (a pair of rows = 192 B = three whole sectors when the pair starts at an
// even tile), RGB8 at 24 B.  Stored tile by tile, the shared sector arrives at the L2 as two
// partial writes tens of microseconds apart and leaves it twice when the line is evicted in
// between (DRAM writes 1.3x the framebuffers, round 5).  Here the even tile's pixels wait in LDS and
// both tiles' stores issue back to back, so the two halves of a sector meet in the L2.
struct PairStash {
    float c[3][64];                  // colour of lane k's pixel of the even tile (its position is
};                                   // decoded again from the wavefront's tile-order entry)
struct NoStash {};

// Any-hit traversal of the wavefront's shadow rays (lane `tid` owns one ray when has_job) with
// intra-wavefront work stealing; on return L.blocked[tid] holds the lane's answer.  Must be
// reached by all 64 lanes of the wavefront (it loops on wavefront ballots).
template <bool kStats, int kS = kBlock, typename StkT = uint32_t*, bool kRobust = false, bool kQ = false, bool kG = false>
__device__ __forceinline__ void steal_traverse(const KParams& P, bool has_job, RayWork w, StkT stk, StealLdsT<kS>& L,
                                               uint32_t tid, uint32_t lane, uint32_t& n_pairs, uint32_t& n_tests,
                                               bool& overflow, uint32_t* n_iters = nullptr) {
    const float tmin = 0.0f, tmax = FLT_MAX;
    const uint32_t cap = P.shadow_stack_entries;
    const uint32_t wbase = tid & ~63u;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    L.blocked[tid] = 0;
    bool active = has_job;
    uint32_t owner = tid, cur = 0, top = 0, bot = 0, cnt = 0;
    if (P.root_leaf_count) {                                           // single-leaf scene
        if (has_job) {
            Hit h;
            L.blocked[tid] = trace<true, kStats, kS, StkT, kRobust, -1, kG>(P, w.o, w.d, stk, h, n_pairs, n_tests, overflow) ? 1u : 0u;
        }
        active = false;
    }
    __builtin_amdgcn_wave_barrier();
    while (__ballot(active)) {
        if (kStats && n_iters) ++*n_iters;

        if (active && L.blocked[owner]) active = false;                 // another piece found an occluder
        if (active) {
            if (kStats) ++n_pairs;
            float e[4];
            uint32_t leaf_mask = 0, inner_mask = 0;
            auto classify = [&](const N4& n) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    float x;
                    slab_box<kRobust>(slab_of<kRobust>(w), pick(n.lx, c), pick(n.hx, c), pick(n.ly, c), pick(n.hy, c),
                                      pick(n.lz, c), pick(n.hz, c), tmin, tmax, e[c], x);
                    const uint32_t cw = pick(n.ch, c), cn = n4_count(cw);
                    const bool hit = e[c] <= x && cw != kNode4Empty;
                    leaf_mask |= (hit && cn != 0) ? (1u << c) : 0u;
                    inner_mask |= (hit && cn == 0) ? (1u << c) : 0u;
                }
            };
            N4 n;
            uint32_t rc;
            if (!kQ && CERES_SPLIT_UNIFORM && uniform_id(cur, rc)) {   // own copy: bounds read from SGPRs
                CERES_COUNT_S(kFBvh4S, 112);
                const Node4* q = P.nodes4 + rc;
                n = {sload_f4(q, 0), sload_f4(q, 1), sload_f4(q, 2), sload_f4(q, 3), sload_f4(q, 4), sload_f4(q, 5),
                     sload_u4(q, 6)};
                classify(n);
                __asm__ volatile("; uniform BVH4 record" ::);
            } else {
                if (!kQ && CERES_SPLIT_UNIFORM) CERES_COUNT_V(kFBvh4V, 112);
                n = (!kQ && CERES_SPLIT_UNIFORM) ? load_n4(P.nodes4 + cur) : load_shadow_node<kQ>(P, cur);
                classify(n);
            }
            bool found = false;
            uint32_t k = 0, k_end = 0;
            while (true) {
                if (k >= k_end) {
                    if (!leaf_mask) break;
                    const uint32_t c = __builtin_ctz(leaf_mask);
                    leaf_mask &= leaf_mask - 1;
                    k = n4_first(pick(n.ch, c));
                    k_end = k + n4_count(pick(n.ch, c));
                    if (kStats) n_tests += k_end - k;
                }
                float t, u, v;
                if (tri_test_u<kG, CERES_RCP_UNIFORM != 0>(P.tris, k, w.o, w.d, tmin, tmax, t, u, v)) { found = true; break; }
                ++k;
            }
            if (found) {
                L.blocked[owner] = 1u;
                active = false;
            } else if (inner_mask) {
                // nearest first here: with work stealing it pays (first-child order: bunny solo +20 %);
                // the first passing child when the scene's LDS budget asks for the smaller stack
                // bound of that order (P.steal_first, order_shadow_bvh4)
                uint32_t best = __builtin_ctz(inner_mask);
                if (!P.steal_first) {
                    float be = best == 0 ? e[0] : best == 1 ? e[1] : best == 2 ? e[2] : e[3];
#pragma unroll
                    for (int c = 1; c < 4; ++c)
                        if ((inner_mask >> c & 1u) && e[c] < be) { be = e[c]; best = c; }
                }
                uint32_t rest = inner_mask & ~(1u << best);
                if (cnt + __builtin_popcount(rest) > cap) { overflow = true; rest = 0; }
                while (rest) {
                    const uint32_t c = __builtin_ctz(rest);
                    rest &= rest - 1;
                    stk[top * kS] = n4_first(pick(n.ch, c));
                    top = top + 1 == cap ? 0 : top + 1;
                    ++cnt;
                }
                cur = n4_first(pick(n.ch, best));
            } else if (cnt) {
                top = (top == 0 ? cap : top) - 1;
                cur = stk[top * kS];
                --cnt;
            } else {
                active = false;                                       // this piece is done, no hit
            }
        }
        // idle lanes take the bottom stack entry of lanes with pending subtrees
        const unsigned long long idle = __ballot(!active);
        const unsigned long long donors = __ballot(active && cnt > 0);
        if (idle && donors) {
            const uint32_t n_idle = __popcll(idle), n_don = __popcll(donors);
            if (active && cnt > 0) {
                const uint32_t r = __popcll(donors & lt_mask);
                if (r < n_idle) {
                    L.mail[wbase + r] = stk[bot * kS];
                    L.from[wbase + r] = lane;
                    bot = bot + 1 == cap ? 0 : bot + 1;
                    --cnt;
                }
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t mail = 0, donor = 0;
            const uint32_t r = __popcll(idle & lt_mask);
            const bool thief = !active && r < n_don;
            if (thief) { mail = L.mail[wbase + r]; donor = L.from[wbase + r]; }
            // every lane runs the shuffles; only thieves keep the values
            const float ox = __shfl(w.o.x, donor, 64), oy = __shfl(w.o.y, donor, 64), oz = __shfl(w.o.z, donor, 64);
            const float dx = __shfl(w.d.x, donor, 64), dy = __shfl(w.d.y, donor, 64), dz = __shfl(w.d.z, donor, 64);
            const float jx = __shfl(w.ix, donor, 64), jy = __shfl(w.iy, donor, 64), jz = __shfl(w.iz, donor, 64);
            const float tx = __shfl(w.sx, donor, 64), ty = __shfl(w.sy, donor, 64), tz = __shfl(w.sz, donor, 64);
            const uint32_t down = __shfl(owner, donor, 64);
            if (thief) {
                w.o = F3{ox, oy, oz}; w.d = F3{dx, dy, dz};
                w.ix = jx; w.iy = jy; w.iz = jz; w.sx = tx; w.sy = ty; w.sz = tz;
                owner = down;
                cur = mail;
                top = bot = cnt = 0;
                active = true;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
}

template <bool kRobust = false, bool kG = false>
__device__ __forceinline__ RayWork make_shadow_ray(F3 o, F3 sun) {
    RayWork w;
    w.o = o;
    w.d = normalizeG<kG>(sun - o);                                     // render.hpp:135
    const Slab<kRobust> sl = make_slab<kRobust>(o, w.d);
    w.ix = sl.ix; w.iy = sl.iy; w.iz = sl.iz; w.sx = sl.sx; w.sy = sl.sy; w.sz = sl.sz;
    return w;
}

// A tile's shadow rays as one packet_any4 when every lane with a shadow ray shares one ray octant
// (nearly every tile), the scene is L2-resident (P.packets) and the packet stack fits the 64
// lanes: returns true and this lane's answer in `blocked`; false (nothing traced) otherwise.
template <typename StkT, bool kRobust, bool kQ, bool kG>
__device__ __forceinline__ bool shadow_packet(const KParams& P, bool hit, const RayWork& w, uint32_t lane, bool& blocked) {
    if constexpr (!kRobust && !kQ && CERES_SHADOW_PACKET && std::is_same<StkT, uint16_t*>::value) {
        const uint64_t act = __ballot(hit);
        if (!act) { blocked = false; return true; }
        const uint32_t oct = (__float_as_uint(w.ix) >> 31) | (__float_as_uint(w.iy) >> 31) << 1 |
                             (__float_as_uint(w.iz) >> 31) << 2;
        const int first = __builtin_ctzll(act);
        const uint32_t oct0 = uint32_t(__builtin_amdgcn_readlane(int(oct), first));
        // packet_any4 relies on every slab value being finite: an empty BVH4 slot (inverted infinite
        // box) then fails the slab test by itself, so its child word is never looked at.  A NaN or
        // infinite slab constant (a non-finite sun, a hit point exactly at the sun: normalize(0))
        // would let the empty slot pass and send the walk to n4_first(kNode4Empty); such a tile
        // takes the per-lane loop, which tests the child word.
        const bool finite = isfinite(w.ix) && isfinite(w.iy) && isfinite(w.iz) && isfinite(w.sx) && isfinite(w.sy) &&
                            isfinite(w.sz);
        if (!P.packets || P.shadow_stack_entries > 64 || P.root_leaf_count || __ballot(hit && (oct != oct0 || !finite)))
            return false;
        // lanes without a shadow ray take a copy of the first one's (masked out, but finite)
        auto bc = [&](float x) { return hit ? x : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), first)); };
        const F3 o{bc(w.o.x), bc(w.o.y), bc(w.o.z)}, d{bc(w.d.x), bc(w.d.y), bc(w.d.z)};
        const Slab<false> sl{bc(w.ix), bc(w.iy), bc(w.iz), bc(w.sx), bc(w.sy), bc(w.sz), o};
        uint64_t occ = 0;
        switch (oct0) {
            case 0: occ = packet_any4<0, kG>(P, sl, o, d, act, lane); break;
            case 1: occ = packet_any4<1, kG>(P, sl, o, d, act, lane); break;
            case 2: occ = packet_any4<2, kG>(P, sl, o, d, act, lane); break;
            case 3: occ = packet_any4<3, kG>(P, sl, o, d, act, lane); break;
            case 4: occ = packet_any4<4, kG>(P, sl, o, d, act, lane); break;
            case 5: occ = packet_any4<5, kG>(P, sl, o, d, act, lane); break;
            case 6: occ = packet_any4<6, kG>(P, sl, o, d, act, lane); break;
            default: occ = packet_any4<7, kG>(P, sl, o, d, act, lane); break;
        }
        blocked = (occ >> lane) & 1u;
        return true;
    }
    return false;
}

// Colour of a pixel with a primary hit, lit or occluded (render.hpp:139-150).
template <bool kG, bool kBands = false>
__device__ __forceinline__ void shade_pixel(const KParams& P, uint32_t f, uint32_t lr, uint32_t i, uint32_t pix,
                                            bool blocked, F3 sun_line, uint32_t slot, float hu, float hv,
                                            uint32_t& occluded, float c[3]) {
    if (P.rec_shadow) P.rec_shadow[pix] = blocked ? 1 : 0;
    c[0] = c[1] = c[2] = 0.f;
    if (blocked) {
        ++occluded;
    } else {
        const F3 view = primary_dir<kG>(P, f, i, global_row<kBands>(P, f, lr));
        CERES_COUNT_V(kFShadeV, 40);
        shade<kG>(sun_line, P.norms + 9 * size_t(P.orig[slot]), view, hu, hv, c);
    }
}

// ---------------------------------------------------------------- fused frame kernel
// Primary + shadow + shading of an 8x8 pixel tile per wavefront in ONE kernel: each wavefront
// traces its tile's primary rays (BVH2, exact reference order), then the shadow rays of its
// own hits over the BVH4 (any-hit; one-frame launches with intra-wavefront work stealing, lanes
// whose pixel missed help the others), then shades.  No shadow-ray queue in HBM, no second
// launch: the shadow work of early tiles overlaps the primary work of later ones.
constexpr int kFusedB = 64;      // single-wavefront workgroups (LDS is released per workgroup)
constexpr size_t kLdsPerCu = 160 * 1024;   // LDS per CU (MI355X_MICROARCH.md)
// 0.f materialised at its use: the compiler otherwise keeps one zero register triple live from the
// prologue across every loop and, short of VGPRs, spills it to scratch once per wavefront
__device__ __forceinline__ float fresh_zero() {
    float z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

template <bool kStats, typename StkT, int kMinW, bool kRobust, bool kSteal, bool kQ, bool kG, int kTPWo = 0, bool kBands = false>
__global__ __launch_bounds__(kFusedB) __attribute__((amdgpu_waves_per_eu(kMinW))) void ceres_fused(const KParams P) {
    constexpr int kB = kFusedB;
    // kernels that trace shadow packets keep only the generic per-lane any-hit loop as fallback
    constexpr bool kPacketsCompiled = !kStats && !kSteal && !kRobust && !kQ && CERES_SHADOW_PACKET && std::is_same<StkT, uint16_t*>::value;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ StealLdsT<kB> L;
    const uint32_t lane = threadIdx.x, tid = lane;
    // paired stores (PairStash): batch kernels of 16-bit-stack scenes, whose LDS has room (2.8 KB of
    // stacks per wavefront; the 24-bit-stack kernels are LDS-bound)
    constexpr uint32_t kTPWp = (kStats || kSteal) ? 1 : kTPWo ? uint32_t(kTPWo) : uint32_t(CERES_TILES_PER_WAVE);
    constexpr bool kPair = CERES_PAIR_STORES && !kStats && !kSteal && kTPWp >= 2 && std::is_same<StkT, uint16_t*>::value;
    __shared__ typename std::conditional<kPair, PairStash, NoStash>::type S;
    // this lane's pixel of tile-order entry t: frame, local row, column, and whether it exists
    auto tile_pixel = [&](uint32_t t, uint32_t& f_, uint32_t& lr_, uint32_t& i_) {
        uint32_t by_, bx_;
        if (P.tile_packed) {                        // bit fields (pack_tile), wave-uniform
            bx_ = t & ((1u << kTileXBits) - 1u);
            by_ = (t >> kTileXBits) & ((1u << kTileYBits) - 1u);
            f_ = t >> (kTileXBits + kTileYBits);
        } else {
            const uint32_t per_frame_ = P.tiles_x * P.row_blocks_per_frame;
            f_ = t / per_frame_;
            const uint32_t rem = t - f_ * per_frame_;
            by_ = rem / P.tiles_x; bx_ = rem - by_ * P.tiles_x;
        }
        // lanes in Morton order over the tile: every quad of lanes (4k..4k+3) is a 2x2 pixel block,
        // so the quads the texture addresser processes together hold neighbouring rays (A/B: solo
        // C3 -2.4 %, C5 batches -1.5 %)
        const uint32_t lx = (lane & 1) | ((lane >> 1) & 2) | ((lane >> 2) & 4), ly = ((lane >> 1) & 1) | ((lane >> 2) & 2) | ((lane >> 3) & 4);
        i_ = bx_ * 8u + lx;
        lr_ = by_ * 8u + ly;
        return i_ < P.W && lr_ < P.local_rows && (!kBands || global_row<true>(P, f_, lr_) < P.H);
    };
    // a pixel's colour: stored now, or (the even tile of a pair) stashed for the odd tile's stores;
    // t_prev: the even tile's order entry (its pixel positions are decoded again, not stashed)
    auto emit = [&](uint32_t q, bool last, uint32_t t_prev, bool act, uint32_t f_, uint32_t lr_, uint32_t i_, float c0, float c1,
                    float c2) {
        if constexpr (kPair) {
            if (!(q & 1u) && !last) {
                S.c[0][lane] = c0; S.c[1][lane] = c1; S.c[2][lane] = c2;
                return;
            }
            if (q & 1u) {                                              // the even tile's pixels first
                uint32_t pf, plr, pi;
                if (tile_pixel(t_prev, pf, plr, pi)) store_pixel(P, pf, plr, pi, S.c[0][lane], S.c[1][lane], S.c[2][lane]);
            }
        }
        if (act) store_pixel(P, f_, lr_, i_, c0, c1, c2);
    };
    // traversal stacks [entry][lane]: 16-, 24- or 32-bit entries, the narrowest every node index
    // of the scene fits (host choice)
    StkT stk;
    if constexpr (std::is_same<StkT, Stk24>::value)
        stk = Stk24{reinterpret_cast<uint16_t*>(lds) + tid,
                    reinterpret_cast<uint8_t*>(lds) + size_t(P.lds_entries) * kB * 2 + tid};
    else
        stk = reinterpret_cast<StkT>(lds) + tid;
    // 1-D grid over the batch's 8x8 tiles in tile_order (centre of the image first, so the
    // expensive tiles start early and cheap background tiles fill the end of the launch); one
    // tile per single-wavefront workgroup, so a long tile holds only its own LDS and wave slot.
    constexpr uint32_t kTile = 8;
    // kTPW consecutive entries of the order per wavefront in batches (throughput: fewer, longer
    // wavefronts -- the background tiles' short waves are mostly launch and first-fetch latency);
    // one per wavefront for single frames (latency: their longest tiles set the frame time) and
    // in stats builds (the wave log is per tile)
    constexpr uint32_t kTPW = (kStats || kSteal) ? 1 : kTPWo ? uint32_t(kTPWo) : uint32_t(CERES_TILES_PER_WAVE);
    const uint32_t per_frame = P.tiles_x * P.row_blocks_per_frame;
    const uint32_t n_tiles = per_frame * P.frames;
    uint32_t n_shadow = 0, occluded = 0, n_pairs = 0, n_tests = 0;
    bool overflow = false;
    // this wavefront's tile-order entries, read once through the scalar cache (a vector load of a
    // uniform address would put a full vector-memory round trip in front of every tile; the order
    // buffer is padded to a multiple of 8 entries)
    static_assert(kTPW == 1 || kTPW == 2 || kTPW == 4 || kTPW == 8, "CERES_TILES_PER_WAVE must be 1, 2, 4 or 8");
    uint4 tiles4 = make_uint4(0, 0, 0, 0), tiles4b = make_uint4(0, 0, 0, 0);
    if constexpr (kTPW == 8) {
        tiles4 = sload_u4(P.tile_order + 8 * size_t(blockIdx.x), 0);
        tiles4b = sload_u4(P.tile_order + 8 * size_t(blockIdx.x), 1);
    } else if constexpr (kTPW == 4) {
        tiles4 = sload_u4(P.tile_order + 4 * size_t(blockIdx.x), 0);
    } else if constexpr (kTPW == 2) {
        tiles4.x = sload_u32(P.tile_order + 2 * size_t(blockIdx.x));
        tiles4.y = sload_u32(P.tile_order + 2 * size_t(blockIdx.x) + 1);
    } else {
        tiles4.x = sload_u32(P.tile_order + blockIdx.x);
    }
    CERES_COUNT_S(kFOrderS, 4 * kTPW);
    for (uint32_t q = 0; q < kTPW; ++q) {
    const uint32_t slot_q = blockIdx.x * kTPW + q;
    if (kTPW > 1 && slot_q >= n_tiles) break;
    const uint4 tq = q < 4 ? tiles4 : tiles4b;
    const uint32_t qq = q & 3;
    const uint32_t t = kTPW == 1 ? tiles4.x : qq == 0 ? tq.x : qq == 1 ? tq.y : qq == 2 ? tq.z : tq.w;
    // the previous entry (paired stores: the even tile of this odd one)
    const uint32_t qp = (q - 1) & 3;
    const uint4 tp = q - 1 < 4 ? tiles4 : tiles4b;
    const uint32_t t_prev = qp == 0 ? tp.x : qp == 1 ? tp.y : qp == 2 ? tp.z : tp.w;
    uint32_t f, lr, i;
    bool active = tile_pixel(t, f, lr, i);
    uint32_t px = (f * P.local_rows + lr) * P.W + i;
    // the lane's pixel decoded again from the wave-uniform entry, for uses after a traversal: kept
    // live across the traversals, lr / i / px were spilled to scratch by the 7-wave batch kernel
    // (CERES_LEAN_WRITES; the empty asm keeps the compiler from reusing the first decode)
    auto redecode = [&]() {
        if constexpr (CERES_LEAN_WRITES) {
            uint32_t tr = t;
            asm volatile("" : "+s"(tr));
            active = tile_pixel(tr, f, lr, i);
            px = (f * P.local_rows + lr) * P.W + i;
        }
    };
    bool hit = false;
    Hit h{0, 0.f, 0.f, 0.f};
    RayWork w{};
    uint64_t t_start = 0;
    if (kStats && P.wave_log) t_start = __builtin_amdgcn_s_memrealtime();   // diagnostic wave timeline (100 MHz)
    // the last tile of this wavefront (a stashed even tile with no odd partner is stored at once)
    const bool last_q = q + 1 == kTPW || (kTPW > 1 && slot_q + 1 >= n_tiles);
    if (!kStats && P.cull && tile_misses_root(P, f, active, i, global_row<kBands>(P, f, lr))) {
        // render.hpp:116-117, every pixel a miss (zeros made here: a zero triple kept from the
        // prologue was the 7-wave batch kernel's scratch spill)
        const float z = CERES_LEAN_WRITES ? fresh_zero() : 0.f;
        emit(q, last_q, t_prev, active, f, lr, i, z, z, z);
        continue;
    }
    if (active) {
        const F3 view = primary_dir<kG>(P, f, i, global_row<kBands>(P, f, lr));
        // kOct -1: the traversal dispatches on a wave-uniform octant; -2: generic loop only
        constexpr int kOctMode = (!kSteal || (CERES_OCTANT_SLAB & 4)) ? -1 : -2;
        hit = guarded_trace<kStats, kB, StkT, kRobust, kOctMode, kG>(P, f3(P.cam[f].eye), view, stk, h, n_pairs,
                                                                   n_tests, overflow);
        if (P.rec_prim) {
            redecode();
            P.rec_prim[px] = hit ? int32_t(P.orig[h.slot]) : -1;
            P.rec_tuv[3 * size_t(px)] = hit ? h.t : 0.f;
            P.rec_tuv[3 * size_t(px) + 1] = hit ? h.u : 0.f;
            P.rec_tuv[3 * size_t(px) + 2] = hit ? h.v : 0.f;
            P.rec_shadow[px] = -1;
        }
        // a missed pixel (render.hpp:116-117) is stored with the tile's lit ones, at the end: a
        // store here would sit in the in-order vector-memory counter ahead of the hit lanes'
        // triangle fetch below, which would then wait for the store's write acknowledgement
        if (hit) {                                                   // render.hpp:127-135
            CERES_COUNT_V(kFShadeV, 48);
            const TriV tr = load_tri(P.tris + h.slot);
            const F3 normal = normalizeG<kG>(tr.n);
            w = make_shadow_ray<kRobust, kG>(hit_point<kG>(tr, normal, h.u, h.v), f3(P.cam[f].sun));
        }
    }
    const uint32_t n_shadow_t = __popcll(__ballot(hit));
    n_shadow += n_shadow_t;
    uint64_t t_primary = 0;
    uint32_t prim_pairs = n_pairs, shadow_iters = 0;
    if (kStats && P.wave_log) t_primary = __builtin_amdgcn_s_memrealtime();
    // shadow phase: intra-wavefront work stealing shortens a frame's longest tiles (a one-frame
    // launch is tail-bound); a multi-frame batch is throughput-bound, and there one ray per lane
    // spends fewer instructions per node (the steal bookkeeping runs every iteration)
    // (the stats kernels keep one ray per lane: their counters are the per-ray traversal's; the
    // single-frame kernel keeps work stealing: with packets compiled in, its spills cost solo C3
    // +3 % whether or not a tile takes them -- docs/EXPERIMENTS.md)
    bool pk_blocked = false;
    const bool pk = !kStats && !kSteal && shadow_packet<StkT, kRobust, kQ, kG>(P, hit, w, lane, pk_blocked);
    if (pk)
        L.blocked[tid] = pk_blocked ? 1u : 0u;
    else if constexpr (kSteal)
        steal_traverse<kStats, kB, StkT, kRobust, kQ, kG>(P, hit, w, stk, L, tid, lane, n_pairs, n_tests, overflow, &shadow_iters);
    else
        L.blocked[tid] = hit && trace_any4<kStats, kB, StkT, kRobust, kQ, kPacketsCompiled ? -2 : -1, kG>(
                                    P, w.o, w.d, stk, n_pairs, n_tests, overflow) ? 1u : 0u;
    redecode();
    float col[3] = {0.f, 0.f, 0.f};                                    // a miss: render.hpp:116-117
    if (hit) shade_pixel<kG, kBands>(P, f, lr, i, px, L.blocked[tid] != 0, w.d, h.slot, h.u, h.v, occluded, col);
    emit(q, last_q, t_prev, active, f, lr, i, col[0], col[1], col[2]);
    if (kStats && P.wave_log) {
        // [start, after primary, end] (100-MHz ticks), longest primary chain, shadow loop trips,
        // primary hits, wave primary pairs, wave shadow pairs
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint32_t mx = prim_pairs;
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, uint32_t(__shfl_xor(int(mx), off, 64)));
        const uint32_t sp = wave_sum(prim_pairs), ss = wave_sum(n_pairs - prim_pairs);
        if (lane == 0) {
            unsigned long long* wl = P.wave_log + 8 * size_t(blockIdx.x);
            wl[0] = t_start; wl[1] = t_primary; wl[2] = t_end; wl[3] = mx; wl[4] = shadow_iters;
            wl[5] = n_shadow_t; wl[6] = sp; wl[7] = ss;
        }
    }
    }
    const uint32_t wo = wave_sum(occluded);
    const uint32_t shard = blockIdx.x % kShards;
    if (lane == 0 && n_shadow) {
        atomicAdd(&P.shards[shard].queued, n_shadow);                  // shadow rays traced
        atomicAdd(&P.shards[shard].hits, (unsigned long long)(n_shadow + wo));
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

// ---------------------------------------------------------------- compacted float readback
// The lit pixels of a float framebuffer (any bit of r, g, b set) as {pixel, r, g, b} records, in
// no particular order (one atomic per wavefront); *n counts them.  ceres_render_f32 copies only
// these and the host writes the zeros (render.hpp:116-117,147-150: misses and shadowed hits).
// At most `cap` records are written (the buffer holds kCompactMaxLitFrac of the frame); *n still
// counts every lit pixel, and a count above cap sends the host to the full copy.
__global__ __launch_bounds__(256) void ceres_compact_lit(const float* __restrict__ px, uint32_t n_pix,
                                                         uint4* __restrict__ out, uint32_t* __restrict__ n,
                                                         uint32_t cap) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
    uint32_t r = 0, g = 0, b = 0;
    if (p < n_pix) {
        const float* q = px + 3 * size_t(p);
        r = __float_as_uint(q[0]); g = __float_as_uint(q[1]); b = __float_as_uint(q[2]);
    }
    const bool lit = (r | g | b) != 0;
    const uint64_t m = __ballot(lit);
    if (!m) return;                                                   // wave-uniform
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(n, uint32_t(__popcll(m)));
    base = uint32_t(__shfl(int(base), 0, 64));
    const uint32_t k = base + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
    if (lit && k < cap) out[k] = make_uint4(p, r, g, b);
}

// ---------------------------------------------------------------- counters
// Sums the counter shards and zeroes them for the next render (so a render that follows a
// counted one needs no memset).
__global__ void ceres_finalize(Shard* shards, uint64_t primary_rays, uint64_t* out) {
    if (threadIdx.x != 0) return;
    unsigned long long q = 0, h = 0, p = 0, t = 0;
    uint32_t err = 0;
    for (int s = 0; s < kShards; ++s) { q += shards[s].queued; h += shards[s].hits; p += shards[s].pairs; t += shards[s].tests; err |= shards[s].error; }
    for (int s = 0; s < kShards; ++s) { shards[s].queued = 0; shards[s].hits = 0; shards[s].pairs = 0; shards[s].tests = 0; shards[s].error = 0; }
    out[0] = primary_rays + q; out[1] = h; out[2] = primary_rays; out[3] = q;
    out[4] = p; out[5] = t; out[6] = err; out[7] = 0;
}

// ---------------------------------------------------------------- multi-GPU frame assembly
// Un-interleaves the rank-major gathered RGB8 rows of a batch into F PPM
// bodies: rank r's buffer (at r * rank_stride) holds its F frames back to back, n_r local rows
// each, local row k at position n_r - 1 - k (as ceres_primary / ceres_shadow store them).
// Output row y of frame f is global row j = H - 1 - y.  Pure copy: HBM-bound, 16-B vectors.
__device__ __forceinline__ uint32_t rank_rows(uint32_t H, uint32_t rb, uint32_t r, uint32_t world) {
    const uint32_t nb = (H + rb - 1) / rb;
    if (r >= nb) return 0;
    const uint32_t mine = (nb - 1 - r) / world + 1;                  // blocks r, r + world, ...
    const bool has_last = (nb - 1) % world == r;                     // the possibly partial last block
    return mine * rb - (has_last ? nb * rb - H : 0);
}

// kPacked: the rank buffers are back to back without padding (an all-to-all's receive
// buffer): rank r starts at row sum_{p<r} n_p instead of at r * rank_stride bytes.
template <bool kVec, bool kPacked = false>
__global__ __launch_bounds__(256) void ceres_assemble(const uint8_t* __restrict__ src, size_t rank_stride,
                                                      uint8_t* __restrict__ dst, uint32_t frames, uint32_t H,
                                                      uint32_t row_bytes, uint32_t rb, uint32_t world) {
    const uint32_t units = kVec ? row_bytes / 16 : row_bytes;
    for (uint32_t oy = blockIdx.y; oy < frames * H; oy += gridDim.y) {
        const uint32_t f = oy / H, y = oy - f * H;
        const uint32_t j = H - 1 - y;
        const uint32_t b = j / rb, r = b % world;
        const uint32_t k = (b / world) * rb + j % rb;
        const uint32_t n = rank_rows(H, rb, r, world);
        size_t base = size_t(r) * rank_stride;
        if (kPacked) {
            base = 0;
            for (uint32_t p = 0; p < r; ++p) base += size_t(frames) * rank_rows(H, rb, p, world) * row_bytes;
        }
        const uint8_t* s = src + base + (size_t(f) * n + (n - 1 - k)) * row_bytes;
        uint8_t* d = dst + size_t(oy) * row_bytes;
        for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
            if (kVec) {
#if CERES_ASSEMBLE_NT
                // streamed through the caches (nontemporal): the un-interleave runs beside later
                // steps' renders, whose BVH / triangle lines it would otherwise evict
                const U4v x = __builtin_nontemporal_load(reinterpret_cast<const U4v*>(s) + u);
                __builtin_nontemporal_store(x, reinterpret_cast<U4v*>(d) + u);
#else
                reinterpret_cast<uint4*>(d)[u] = reinterpret_cast<const uint4*>(s)[u];
#endif
            }
            else d[u] = s[u];
        }
    }
}

}  // namespace dev
}  // namespace ceres

// =====================================================================================
// host side: scene upload + launch glue (C ABI)
// =====================================================================================
using namespace ceres;

#include "scene_internal.hpp"

namespace {

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return set_error(CERES_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <typename T>
void dfree(T*& p) { if (p) { (void)hipFree(p); p = nullptr; } }

}  // namespace

void ceres::scene_release(ceres_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    dfree(s->d_pairs64); dfree(s->d_tris64); dfree(s->d_norms64);
    for (auto& o : s->orders) dfree(o.d);
    for (auto& d : s->retired) dfree(d);
    s->orders.clear(); s->retired.clear(); s->retired_bytes = 0;
    dfree(s->d_pairs); dfree(s->d_nodes4); dfree(s->d_qnodes4); dfree(s->d_tris); dfree(s->d_orig); dfree(s->d_norms);
    dfree(s->d_shards); dfree(s->d_counters); dfree(s->d_wave_log); dfree(s->d_pixels); dfree(s->d_rgb8);
    for (auto e : s->ev_pool) (void)hipEventDestroy(e);
    for (auto e : s->ev_used) (void)hipEventDestroy(e);
    s->ev_pool.clear(); s->ev_used.clear();
    for (auto e : s->band_events) (void)hipEventDestroy(e);
    s->band_events.clear();
    dfree(s->d_band_counters);
    dfree(s->d_lit); dfree(s->d_lit_count);
    if (s->h_lit_pinned) (void)hipHostFree(s->h_lit_pinned);
    s->h_lit_pinned = nullptr;
    if (s->h_small) (void)hipHostFree(s->h_small);
    s->h_small = nullptr;
    if (s->ev_count) (void)hipEventDestroy(s->ev_count);
    s->ev_count = nullptr;
    if (s->copy_stream) (void)hipStreamDestroy(s->copy_stream);
    s->copy_stream = nullptr;
    if (s->stream) (void)hipStreamDestroy(s->stream);
    s->stream = nullptr;
}

namespace {

size_t local_rows_of(size_t H, uint32_t rb, uint32_t rank, uint32_t world);
size_t local_rows_of(size_t H, const ceres_tiling& t) {
    if (t.bands && t.world > 1) return t.row_block;                 // every frame: one band of row_block rows
    return local_rows_of(H, t.row_block, t.rank, t.world);
}
size_t local_rows_of(size_t H, uint32_t rb, uint32_t rank, uint32_t world) {
    const size_t nblocks = (H + rb - 1) / rb;
    size_t rows = 0;
    for (size_t b = rank; b < nblocks; b += world) rows += std::min<size_t>(rb, H - b * rb);
    return rows;
}

int ensure_workspace(ceres_scene* s, size_t px, bool want_px, bool want_rgb) {
    if ((want_px || want_rgb) && px > s->px_cap) {
        dfree(s->d_pixels); dfree(s->d_rgb8);
        HIP_TRY(hipMalloc(&s->d_pixels, px * 3 * sizeof(float)));
        HIP_TRY(hipMalloc(&s->d_rgb8, px * 3));
        s->px_cap = px;
    }
    return CERES_OK;
}

// Caches `order` on the scene under its key (see ensure_tile_order) and uploads it.
int upload_tile_order(ceres_scene* s, size_t W, size_t H, const ceres_tiling& t, uint32_t frames, uint32_t tile,
                      std::vector<uint32_t>& order, hipStream_t stream, const uint32_t** out, bool packed,
                      uint32_t bx, uint32_t by) {
    const size_t n = order.size();
    if (packed) {                                                    // linear ids -> pack_tile words
        const uint32_t per_frame = bx * by;
        for (auto& id : order) {
            const uint32_t f = id / per_frame, rem = id - f * per_frame, y = rem / bx;
            id = pack_tile(f, y, rem - y * bx);
        }
    }
    ceres_scene::TileOrder o;
    if (s->orders.size() >= ceres::kMaxTileOrders) {
        auto lru = std::min_element(s->orders.begin(), s->orders.end(),
                                    [](const auto& a, const auto& b) { return a.used < b.used; });
        s->retired.push_back(lru->d);                                // a launch may still read it
        s->retired_bytes += (lru->cap * sizeof(uint32_t) + kAllocGranule - 1) / kAllocGranule * kAllocGranule;
        s->orders.erase(lru);
        if (s->retired_bytes > ceres::kRetiredBytes || s->retired.size() >= ceres::kMaxRetired) {
            HIP_TRY(hipDeviceSynchronize());
            for (auto& d : s->retired) dfree(d);
            s->retired.clear();
            s->retired_bytes = 0;
        }
    }
    o.W = W; o.H = H; o.row_block = t.row_block; o.rank = t.rank; o.world = t.world; o.frames = frames; o.tile = tile;
    o.bands = t.bands;
    o.packed = packed;
    // padded to a multiple of 8 entries (zeros): the fused kernel reads its tile-order entries
    // up to eight at a time through the scalar cache
    const size_t padded = (n + 7) / 8 * 8;
    if (!o.d) {
        HIP_TRY(hipMalloc(&o.d, padded * sizeof(uint32_t)));
        o.cap = padded;
    }
    if ((padded > n && hipMemsetAsync(o.d + n, 0, (padded - n) * sizeof(uint32_t), stream) != hipSuccess) ||
        hipMemcpyAsync(o.d, order.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess) {
        dfree(o.d);
        return set_error(CERES_EHIP, "tile order upload failed");
    }
    o.used = ++s->order_clock;
    s->orders.push_back(o);
    *out = o.d;
    return CERES_OK;
}

// XCD row runs for batches: every run of CERES_XCD_GROUP_TILES horizontally adjacent tiles of a
// tile row (128 pixels) goes to one XCD, chosen by a hash of (frame, tile row, run) for balance;
// workgroup w runs on XCD w mod 8 and takes tpw consecutive order entries, so each XCD's tiles are
// queued in the centre-first order and dealt to that XCD's workgroups (when a queue runs dry --
// the hash is not exact -- the tail takes from the longest one).  Neighbouring tiles' rays share
// BVH records and triangles, which then stay in one L2.  Built to merge the framebuffer's partial
// 128-B lines in one L2; it does not (WRITE_SIZE +9 %: each store's 64-B sectors leave the L2 as
// they are), but the L2 reuse pays: 16-frame batches x 8 streams C3 -2.3 %, bunny 1080p -1.0 %,
// bunny 640 -1.3 %; single frames lose (C3 +3.6 %, bunny 640 +6.7 %: a one-frame launch needs the
// shuffled order's XCD balance), so only batches use it.  profiles/r05/s13.
static void xcd_group_rows(std::vector<uint32_t>& order, uint32_t bx, uint32_t per_frame, uint32_t tpw) {
    std::vector<uint32_t> q[8];
    for (auto& v : q) v.reserve(order.size() / 8 + 1);
    for (const uint32_t id : order) {
        const uint32_t f = id / per_frame, rem = id - f * per_frame, y = rem / bx, x = rem - y * bx;
        uint64_t h = (uint64_t(f) << 42) ^ (uint64_t(y) << 21) ^ uint64_t(x / CERES_XCD_GROUP_TILES);
        h *= 0x9e3779b97f4a7c15ull;
        h ^= h >> 29;
        h *= 0xbf58476d1ce4e5b9ull;
        q[(h >> 32) & 7].push_back(id);
    }
    size_t head[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (size_t p = 0; p < order.size(); ++p) {
        uint32_t x = uint32_t((p / tpw) % 8);
        if (head[x] == q[x].size()) {
            size_t best = 0;
            for (uint32_t k = 0; k < 8; ++k)
                if (q[k].size() - head[k] > best) { best = q[k].size() - head[k]; x = k; }
        }
        order[p] = q[x][head[x]++];
    }
}

// Centre-first order of a batch's tile x tile tiles for the fused kernel: ascending distance of the
// tile centre (global pixel coordinates) from the image centre, frames interleaved (views of
// CERES_FRAME_MAJOR_PIXELS and more: frame after frame), then shuffled in windows of 64 for the
// XCD balance.  Cached on the scene per (W, H, tiling, frames, tile) -- up to kMaxTileOrders
// orders; the least recently used one is retired (freed later, see ceres_scene::retired), so
// eviction neither rewrites an order a launch in flight reads nor stalls the streams.
int ensure_tile_order(ceres_scene* s, size_t W, size_t H, const ceres_tiling& t, size_t rows, uint32_t frames,
                      uint32_t bx, uint32_t by, uint32_t tile, hipStream_t stream, const uint32_t** out, bool packed,
                      uint32_t tpw) {
    const uint32_t tile_key = tile | tpw << 16;                    // the order depends on the tiles per wave
    for (auto& o : s->orders)
        if (o.W == W && o.H == H && o.row_block == t.row_block && o.rank == t.rank && o.world == t.world && o.bands == t.bands &&
            o.frames == frames && o.tile == tile_key && o.packed == packed) {
            o.used = ++s->order_clock;
            *out = o.d;
            return CERES_OK;
        }
    const size_t n = size_t(bx) * by * frames;
    const double cx = 0.5 * double(W), cy = 0.5 * double(H);
    std::vector<std::pair<double, uint32_t>> k(n);
    // Large views go one frame after another (each centre-first): the waves in flight then share
    // one view's BVH nodes and triangles in L2 instead of F views' (8 x 16-frame batches: dragon
    // 4096^2 -18 %, C5 -4 %; also for a rank's interleaved rows of such a view).  Smaller views
    // stay interleaved so every frame's expensive centre starts early (round 3, C3: frame-major
    // +0..6 %).  Round 5 moved the threshold from 4 to 1 Mpixel: with the current kernel the
    // frame-major batches' XCD-local Morton order below wins for 1080p views (16-frame batches x 8
    // streams: C3 orbit -8.3 %, C3 copies -5.8 %, bunny 1080p copies -3.5 %; 256 Kpixel: bunny 640
    // +5 %, so 1 Mpixel; profiles/r05/s27-s28).
    const uint64_t fm_pixels = CERES_FRAME_MAJOR_PIXELS;
    // (the pixels of a frame this launch renders: a rank's rows of a row-split frame count alone)
    const bool frame_major = fm_pixels != 0 && uint64_t(W) * rows >= fm_pixels;
    for (uint32_t f = 0; f < frames; ++f)
        for (uint32_t y = 0; y < by; ++y) {
            const size_t lr = std::min<size_t>(size_t(y) * tile + tile / 2, rows - 1);
            const size_t j = (t.bands && t.world > 1) ? ((t.rank + f) % t.world) * t.row_block + lr
                                                      : ((lr / t.row_block) * t.world + t.rank) * t.row_block + lr % t.row_block;
            for (uint32_t x = 0; x < bx; ++x) {
                const double dx = double(x) * tile + tile / 2 - cx, dy = double(j) - cy;
                const uint32_t id = (f * by + y) * bx + x;
                k[id] = {dx * dx + dy * dy, id};
            }
        }
    const uint32_t per_frame = bx * by;
    std::stable_sort(k.begin(), k.end(), [frame_major, per_frame](const auto& a, const auto& b) {
        if (frame_major && a.second / per_frame != b.second / per_frame) return a.second < b.second;
        return a.first < b.first;
    });
    std::vector<uint32_t> order(n);
    for (size_t q = 0; q < n; ++q) order[q] = k[q].second;
    // Workgroups b and b + 8 share an XCD (MI355X_MICROARCH.md: blocks are dealt round-robin over
    // the 8 XCDs), and the XCD with the most work sets a launch's length.  The centre-first order
    // is regular -- equal-distance tiles of the F frames and mirror-image tiles sit side by side --
    // so a fixed stride of 8 hands an XCD a systematic part of the frames or of the image (one view
    // of four; the left half of a mesh).  Shuffling each window of 64 (fixed seed) keeps the order
    // centre-first at that granularity and gives every XCD an unbiased sample: solo bunny 1080p
    // -9.5 %, dragon 4096^2 -5.5 %; one rank of a 2-GPU split 40 % -> 0 % apart.
    // XCD-local order for large views: each frame's tiles along a Morton curve, every run of 8 x c
    // tiles dealt so that XCD x (workgroups w = x mod 8) takes the x-th block of c consecutive
    // curve tiles -- the waves of one XCD render one compact image region at a time, so the BVH
    // nodes and triangles that region's rays share stay in that XCD's L2.  Used for frame-major
    // batches (A/B, 16-frame batches x 8 streams: dragon 4096^2 -3.2 %, C5 -1.7..-1.9 %) and for
    // single frames of a scene that does not fit the L2s (C5 solo frame 3.11 -> 2.66 ms, -14 %); a
    // single frame of an L2-resident scene keeps the centre-first order (dragon 4096^2: local
    // +9 %: its expensive centre tiles must start first).  profiles/r03/local_order/.
    const size_t scene_bytes = s->n_pairs * sizeof(SiblingPair) + s->n_nodes4 * sizeof(Node4) +
                               s->n_tri * (sizeof(Tri48) + 4 + 36);
    const size_t lchunk = !CERES_LOCAL_ORDER || !frame_major ? 0
                          : frames > 1 ? size_t(CERES_LOCAL_CHUNK_BATCH)
                          : scene_bytes >= kDramSceneBytes ? size_t(CERES_LOCAL_CHUNK_SOLO) : 0;
    if (lchunk) {
        auto morton = [](uint32_t x, uint32_t y) {
            uint64_t m = 0;
            for (int b = 0; b < 16; ++b) m |= (uint64_t((x >> b) & 1) << (2 * b)) | (uint64_t((y >> b) & 1) << (2 * b + 1));
            return m;
        };
        std::vector<std::pair<uint64_t, uint32_t>> mk(n);
        for (uint32_t id = 0; id < n; ++id) {
            const uint32_t f = id / per_frame, rem = id - f * per_frame, y = rem / bx, x = rem - y * bx;
            mk[id] = {(uint64_t(f) << 40) | morton(x, y), id};
        }
        std::sort(mk.begin(), mk.end());
        const size_t c = std::max<size_t>(tpw, lchunk / tpw * tpw), cw = c / tpw, grp = 8 * c;
        const size_t full = n / grp * grp;
        for (size_t p = 0; p < n; ++p) {
            size_t src = p;
            if (p < full) {
                const size_t w = p / tpw, i = p % tpw, g = w / (8 * cw), wl = w % (8 * cw);
                src = g * grp + (wl % 8) * c + (wl / 8) * tpw + i;
            }
            order[p] = mk[src].second;
        }
        return upload_tile_order(s, W, H, t, frames, tile_key, order, stream, out, packed, bx, by);
    }
    uint64_t st = 0x9e3779b97f4a7c15ull;
    for (size_t b0 = 0; b0 < n; b0 += dev::kTileShuffleWindow) {
        const size_t len = std::min<size_t>(dev::kTileShuffleWindow, n - b0);
        for (size_t q = len - 1; q > 0; --q) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            std::swap(order[b0 + q], order[b0 + size_t((st >> 33) % (q + 1))]);
        }
    }
    if (CERES_XCD_GROUP_TILES && frames > 1) xcd_group_rows(order, bx, per_frame, tpw);
    return upload_tile_order(s, W, H, t, frames, tile_key, order, stream, out, packed, bx, by);
}

// CERES_MODE_QBVH4: the exact shadow BVH4 (Node4) -> compressed QNode4 records.  Per node and
// axis: origin = the smallest child lo, scale = the power of two that puts the children's extent
// in 250 steps; every child bound becomes a byte q with fma(q, scale, origin) <= lo (resp. >= hi),
// checked with the kernel's own formula, so each decoded box contains the exact box (and the
// fast slab test is monotone in the bounds: every box the exact test passes, the decoded one
// passes too).  Empty slots keep their kNode4Empty child word.
int quantize_nodes4(const std::vector<Node4>& in, std::vector<QNode4>& out) {
    out.assign(in.size(), QNode4{});
    for (size_t k = 0; k < in.size(); ++k) {
        const Node4& n = in[k];
        QNode4& q = out[k];
        const float* lo[3] = {n.lo_x, n.lo_y, n.lo_z};
        const float* hi[3] = {n.hi_x, n.hi_y, n.hi_z};
        float org[3], scl[3];
        uint32_t ql[3] = {0, 0, 0}, qh[3] = {0, 0, 0};
        for (int a = 0; a < 3; ++a) {
            float mn = INFINITY, mx = -INFINITY;
            for (int c = 0; c < 4; ++c)
                if (n.child[c] != kNode4Empty) { mn = std::min(mn, lo[a][c]); mx = std::max(mx, hi[a][c]); }
            if (mn > mx) { mn = 0.f; mx = 0.f; }                     // no children (cannot happen) or empty
            if (!std::isfinite(mn) || !std::isfinite(mx))
                return set_error(CERES_EUNSUPPORTED, "CERES_MODE_QBVH4: non-finite BVH bounds");
            const double ext = double(mx) - double(mn);
            int e = ext > 0 ? int(std::ceil(std::log2(ext / 250.0))) : -126;
            e = std::max(e, -126);
            float sc = std::ldexp(1.0f, e);
            org[a] = mn;
            for (int c = 0; c < 4; ++c) {
                uint32_t bl = 255, bh = 0;                           // empty slot: never read (child word)
                if (n.child[c] != kNode4Empty) {
                    double fl = std::floor((double(lo[a][c]) - double(mn)) / double(sc));
                    double fh = std::ceil((double(hi[a][c]) - double(mn)) / double(sc));
                    int il = int(std::max(0.0, std::min(255.0, fl))), ih = int(std::max(0.0, std::min(255.0, fh)));
                    while (il > 0 && std::fma(float(il), sc, mn) > lo[a][c]) --il;
                    while (ih < 255 && std::fma(float(ih), sc, mn) < hi[a][c]) ++ih;
                    if (std::fma(float(il), sc, mn) > lo[a][c] || std::fma(float(ih), sc, mn) < hi[a][c])
                        return set_error(CERES_EUNSUPPORTED, "CERES_MODE_QBVH4: bound not representable");
                    bl = uint32_t(il); bh = uint32_t(ih);
                }
                ql[a] |= bl << (8 * c);
                qh[a] |= bh << (8 * c);
            }
            scl[a] = sc;
        }
        q.ox = org[0]; q.oy = org[1]; q.oz = org[2];
        q.sx = scl[0]; q.sy = scl[1]; q.sz = scl[2];
        q.qlx = ql[0]; q.qhx = qh[0]; q.qly = ql[1]; q.qhy = qh[1]; q.qlz = ql[2]; q.qhz = qh[2];
        for (int c = 0; c < 4; ++c) q.child[c] = n.child[c];
    }
    return CERES_OK;
}

// First QBVH4 render of a scene: read its exact BVH4 back, compress it, upload the copy.
int build_qnodes4(ceres_scene* s) {
    if (!s->n_nodes4 || !s->d_nodes4) return CERES_OK;              // root is a leaf: shadow rays use the BVH2 path
    std::vector<Node4> n4(s->n_nodes4);
    HIP_TRY(hipMemcpy(n4.data(), s->d_nodes4, n4.size() * sizeof(Node4), hipMemcpyDeviceToHost));
    std::vector<QNode4> q;
    if (int rc = quantize_nodes4(n4, q)) return rc;
    HIP_TRY(hipMalloc(&s->d_qnodes4, q.size() * sizeof(QNode4)));
    HIP_TRY(hipMemcpy(s->d_qnodes4, q.data(), q.size() * sizeof(QNode4), hipMemcpyHostToDevice));
    return CERES_OK;
}

// The root box pre-test of primary rays (trace()): the reference never tests the root's own box
// (single_ray_traverser.hpp:81 starts at its children), but when both children's boxes lie inside
// it (exact float compare) a child box can pass the slab test only if the root box does -- the
// test is monotone in the bounds (see build_shadow_bvh4) -- so a ray failing the root box would
// fail both children in the reference's first step: same result, no record fetch.
void set_root_box(ceres_scene* s, const float root[6], const SiblingPair& p0) {
    for (int k = 0; k < 6; ++k) s->root_box[k] = root[k];
    auto inside = [&](const float* c) {
        return c[0] >= root[0] && c[1] <= root[1] && c[2] >= root[2] && c[3] <= root[3] && c[4] >= root[4] && c[5] <= root[5];
    };
    s->root_box_ok = (!s->root_leaf_count && inside(p0.lb) && inside(p0.rb)) ? 1u : 0u;
}

// The background cull's proof for one frame (tile_misses_root).  The primary ray of image
// coordinates (u, v) is eye + s (iu u + iv v + dir) (render.hpp:109-111), so a point X projects to
// (p / w, q / w) with (p, q, w) = [iu iv dir]^-1 (X - eye).  Every corner of the root box, EXPANDED
// by 1e-4 of the scene / eye coordinate scale, must lie in front of the eye (w > 0.01 |X - eye|);
// then the expanded box's image lies inside the bounding rectangle of the corner images (a convex
// set in front of the eye projects into the hull of its corners' images), and a pixel whose (u, v)
// = (2 (i + 0.5) / W - 1, 2 (j + 0.5) / H - 1) lies outside that rectangle widened by m = 2e-3 (1 +
// max |corner coordinate|) -- two pixels at 1080p -- has a ray that misses the expanded box.  The
// kernel's float ray (render.hpp:109-113: rounding of ~1e-6 in (u, v) and in the unit direction)
// and float slab test (~1e-6 relative in the slab distances, node_intersectors.hpp:83-103) stay far
// inside those margins, so its root-box test fails too.  Computed in double; anything degenerate
// (a corner behind the eye, NaN, a frame wider than 65,535 pixels) keeps every pixel.
static CullRect cull_rect(const FrameCam& c, const float root[6], uint32_t W, uint32_t H) {
    const CullRect keep{0u, 0xffffu, 0u, 0xffffu};
    if (W > 0xffffu || H > 0xffffu) return keep;
    double e[3], iu[3], iv[3], d[3];
    for (int k = 0; k < 3; ++k) { e[k] = c.eye[k]; iu[k] = c.iu[k]; iv[k] = c.iv[k]; d[k] = c.dir[k]; }
    double sc = 0;
    for (int k = 0; k < 3; ++k) sc = std::max(sc, std::fabs(e[k]));
    for (int k = 0; k < 6; ++k) sc = std::max(sc, std::fabs(double(root[k])));
    const double pad = 1e-4 * sc;
    auto cr = [](const double* a, const double* b, double* o) {
        o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0]; };
    double c0[3], c1[3], c2[3];
    cr(iv, d, c0); cr(d, iu, c1); cr(iu, iv, c2);
    const double det = iu[0] * c0[0] + iu[1] * c0[1] + iu[2] * c0[2];
    double u0 = HUGE_VAL, u1 = -HUGE_VAL, v0 = HUGE_VAL, v1 = -HUGE_VAL;
    for (int k = 0; k < 8; ++k) {
        const double X[3] = {(k & 1) ? root[1] + pad : root[0] - pad, (k & 2) ? root[3] + pad : root[2] - pad,
                             (k & 4) ? root[5] + pad : root[4] - pad};
        const double r[3] = {X[0] - e[0], X[1] - e[1], X[2] - e[2]};
        const double pw = r[0] * c0[0] + r[1] * c0[1] + r[2] * c0[2], qw = r[0] * c1[0] + r[1] * c1[1] + r[2] * c1[2];
        const double ww = r[0] * c2[0] + r[1] * c2[1] + r[2] * c2[2];
        if (!(ww / det > 0.01 * std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]))) return keep;
        u0 = std::min(u0, pw / ww); u1 = std::max(u1, pw / ww); v0 = std::min(v0, qw / ww); v1 = std::max(v1, qw / ww);
    }
    const double m = 2e-3 * (1 + std::max(std::max(std::fabs(u0), std::fabs(u1)), std::max(std::fabs(v0), std::fabs(v1))));
    // pixels whose u lies in [u0 - m, u1 + m]: i in [(u0 - m + 1) W / 2 - 0.5, (u1 + m + 1) W / 2 - 0.5], one more each side
    auto lo = [](double x, uint32_t n) { return x <= 0 ? 0u : x >= n ? n : uint32_t(std::floor(x)); };
    const double a0 = (u0 - m + 1) * W / 2 - 0.5 - 1, a1 = (u1 + m + 1) * W / 2 - 0.5 + 1;
    const double b0 = (v0 - m + 1) * H / 2 - 0.5 - 1, b1 = (v1 + m + 1) * H / 2 - 0.5 + 1;
    if (!(a0 == a0 && a1 == a1 && b0 == b0 && b1 == b1)) return keep;
    if (a1 < 0 || b1 < 0) return CullRect{1u, 0u, 1u, 0u};            // empty: the whole frame misses
    return CullRect{uint16_t(lo(a0, W)), uint16_t(std::min<double>(std::ceil(a1), 0xffff)),
                    uint16_t(lo(b0, H)), uint16_t(std::min<double>(std::ceil(b1), 0xffff))};
}

// One launch of a batch: `frames` (<= kFramesPerLaunch) cameras (basis12 = frames x {eye, dir, iu,
// iv}) and suns (frames x 3).  first / last: the first and last launch of a batch call (the counter
// shards are cleaned before the first and summed after the last, over `batch_frames` frames).
// LDS stack entry width of a scene's fused kernels: the narrowest every pair / BVH4 index fits
static int stack_width(size_t n_pairs, size_t n_nodes4) {
    const size_t nmax = std::max(n_pairs, n_nodes4);
    return CERES_STACK16 && nmax < (1u << 16) ? 2 : CERES_STACK24 && nmax < (1u << 24) ? 3 : 4;
}
// Tiles per wavefront of the batch kernel: consecutive tile-order entries a wave takes.  16-bit-stack
// scenes (dragon, bunny) with frames of 1-4 Mpixel (1080p) take 2, everything else
// CERES_TILES_PER_WAVE (A/B, 16-frame batches x 8 streams: C3 -2.1 %, bunny +-1 %, a C3 batch
// launch alone -11 %; 8 for 4096^2 measured +-0.6 %; profiles/r05/s38, s39).  The kernel
// instantiation for 2 exists for these scenes only.
static uint32_t batch_tiles_per_wave(size_t frame_pixels, int stw, bool qbvh) {
    if (!CERES_TPW_BY_SIZE || stw != 2 || qbvh) return CERES_TILES_PER_WAVE;
    return frame_pixels >= (size_t(1) << 20) && frame_pixels < (size_t(1) << 22) ? 2u : uint32_t(CERES_TILES_PER_WAVE);
}

// LDS of one fused-kernel wavefront for `entries` stack slots, and whether that costs waves: above
// kLdsPerCu / 28 a CU holds fewer than 7 waves per SIMD (the kernels' VGPR budget)
static size_t fused_lds_bytes(uint32_t entries, int stw) {
    return size_t(entries) * dev::kFusedB * stw + sizeof(dev::StealLdsT<dev::kFusedB>);
}
static bool lds_limits_waves(uint32_t entries, int stw) { return fused_lds_bytes(entries, stw) > dev::kLdsPerCu / 28; }

// Launch-time check of a fused kernel's LDS carve-up (round 6).  The dynamic
// block holds the traversal stacks -- lds_entries slots x 64 lanes x stw bytes, [entry][lane]
// (a 24-bit stack: the u16 plane, then the u8 plane at lds_entries x 64 x 2) -- and the static
// block the work-stealing mailboxes (StealLdsT: blocked / mail / from, 3 x 64 words).  Every
// index the kernel forms must fall in its own region:
//   BVH2 walk        slots 0 .. stack_entries (the far child is written to slot sp, sp <= depth - 1)
//   BVH4 walks       slots 0 .. shadow_stack_entries - 1 (pushes are bounded before they happen;
//                    the stealing loop's ring has exactly that many slots)
// and the whole allocation must fit what a workgroup may hold on this device.  A carve-up that
// breaks any of these is refused here with CERES_EINVAL instead of letting a stack entry land in
// another lane's slot or plane and come back as a node index (the failure mode of round 5's
// fault, DESIGN.md "Round 6: the round-5 fault").
static int check_fused_lds(const ceres_scene* s, const KParams& P, int stw, size_t dyn_bytes) {
    const size_t need = size_t(P.lds_entries) * dev::kFusedB * size_t(stw);
    const size_t total = dyn_bytes + sizeof(dev::StealLdsT<dev::kFusedB>);
    if (stw != 2 && stw != 3 && stw != 4)
        return set_error(CERES_EINVAL, "render: bad LDS stack entry width %d", stw);
    if (P.lds_entries < P.stack_entries + 1 || P.lds_entries < P.shadow_stack_entries || dyn_bytes < need)
        return set_error(CERES_EINVAL, "render: LDS stack of %u slots (%zu B) cannot hold the BVH2 stack (%u + 1) and the BVH4 "
                         "stack (%u)", P.lds_entries, dyn_bytes, P.stack_entries, P.shadow_stack_entries);
    if (total > s->max_lds_per_block)
        return set_error(CERES_EINVAL, "render: fused kernel needs %zu B of LDS per workgroup (%zu available)", total,
                         s->max_lds_per_block);
    return CERES_OK;
}

int launch_chunk(ceres_scene* s, uint32_t frames, const float* basis12, const float* sun, int mode, size_t W, size_t H,
                 const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, hipStream_t stream,
                 int32_t* d_rec_prim, float* d_rec_tuv, int8_t* d_rec_shadow, bool first, bool last,
                 uint64_t batch_primary) {
    if (!s || !basis12 || !sun) return set_error(CERES_EINVAL, "render: null argument");
    if (s->f64) return set_error(CERES_EINVAL, "scene is double precision: use ceres_render_f64");
    if (frames == 0 || frames > uint32_t(kFramesPerLaunch))
        return set_error(CERES_EINVAL, "render: %u frames per launch (1..%d)", frames, kFramesPerLaunch);
    const bool robust = (mode & CERES_MODE_ROBUST) != 0;            // RobustNodeIntersector traversal
    const bool qbvh = (mode & CERES_MODE_QBVH4) != 0;              // compressed shadow BVH4 (not exact)
    const bool gfma = (mode & CERES_MODE_FMA) != 0;                 // the reference CMake build's FMA contraction
    mode &= ~(CERES_MODE_ROBUST | CERES_MODE_QBVH4 | CERES_MODE_FMA);
    if (mode != CERES_MODE_FULL && mode != CERES_MODE_PRIMARY) return set_error(CERES_EINVAL, "render: bad mode %d", mode);
    if (W == 0 || H == 0 || W > 65535u * 16u || H > 0xffffffu) return set_error(CERES_EINVAL, "render: bad size %zux%zu", W, H);
    ceres_tiling t{uint32_t(H), 0, 1};
    if (tiling) t = *tiling;
    if (t.world == 0 || t.rank >= t.world || t.row_block == 0) return set_error(CERES_EINVAL, "render: bad tiling");
    if (t.world == 1) t.bands = 0;
    if (t.bands && (t.bands != 1 || t.world > 65535u || size_t(t.row_block) * t.world < H))
        return set_error(CERES_EINVAL, "render: bands of %u rows x %u ranks do not cover %zu rows", t.row_block, t.world, H);
    const size_t rows = local_rows_of(H, t);
    if (size_t(frames) * W * rows > 0xffffffffull) return set_error(CERES_EINVAL, "render: more than 2^32 pixels per batch");
    const uint32_t bx = uint32_t((W + 15) / 16), by = uint32_t((rows + 15) / 16);
    if (size_t(by) * frames > 65535u) return set_error(CERES_EINVAL, "render: frames x row blocks exceeds the grid limit");
    if ((d_rec_prim != nullptr) != (d_rec_tuv != nullptr) || (d_rec_prim != nullptr) != (d_rec_shadow != nullptr))
        return set_error(CERES_EINVAL, "render: hit records need all three arrays");
    if (qbvh && (robust || (s->flags & CERES_SCENE_STATS)))
        return set_error(CERES_EUNSUPPORTED, "render: CERES_MODE_QBVH4 takes neither CERES_MODE_ROBUST nor a stats scene");
    if (t.bands && (mode != CERES_MODE_FULL || robust || qbvh || (s->flags & CERES_SCENE_STATS) || d_rec_prim))
        return set_error(CERES_EUNSUPPORTED, "render: ceres_tiling.bands takes the full mode of a non-stats scene "
                                             "(not ROBUST, QBVH4, PRIMARY or hit records)");
    HIP_TRY(hipSetDevice(s->device));
    if (qbvh && mode == CERES_MODE_FULL && !s->d_qnodes4)
        if (int rc = build_qnodes4(s)) return rc;

    KParams P{};
    for (uint32_t f = 0; f < frames; ++f) {
        FrameCam& c = P.cam[f];
        std::memcpy(c.eye, basis12 + 12 * f, 12); std::memcpy(c.dir, basis12 + 12 * f + 3, 12);
        std::memcpy(c.iu, basis12 + 12 * f + 6, 12); std::memcpy(c.iv, basis12 + 12 * f + 9, 12);
        std::memcpy(c.sun, sun + 3 * f, 12);
    }
    P.frames = frames;
    P.W = uint32_t(W); P.H = uint32_t(H);
    P.row_block = t.row_block; P.rank = t.rank; P.world = t.world; P.local_rows = uint32_t(rows);
    P.bands = t.bands;
    P.band_magic = t.bands ? uint32_t(((uint64_t(1) << 32) + t.world - 1) / t.world) : 0u;   // exact for rank + f < 2^16
    P.row_blocks_per_frame = by;
    P.stack_entries = s->stack_entries;
    P.shadow_stack_entries = s->shadow_stack_entries;
    // wave-wide packets read every record through the scalar cache, one dependent miss at a time:
    // for a scene that streams from DRAM (C5) that latency is exposed and the per-lane loops are
    // faster (A/B, 16-frame batches: C5 +10 % with packets, L2-resident scenes -3..-5 %)
    P.packets = (s->n_pairs * sizeof(SiblingPair) + s->n_nodes4 * sizeof(Node4) + s->n_tri * sizeof(Tri48)) <
                kDramSceneBytes ? 1u : 0u;
    P.root_leaf_count = s->root_leaf_count; P.root_leaf_first = s->root_leaf_first;
    for (int k = 0; k < 6; ++k) P.root_box[k] = s->root_box[k];
    P.root_box_ok = CERES_ROOT_TEST ? s->root_box_ok : 0u;
    // the background cull rests on the root-box pre-test's argument (tile_misses_root); stats scenes
    // and hit records keep every ray's own root step
    P.cull = (CERES_CULL && P.root_box_ok && !(s->flags & CERES_SCENE_STATS) && !d_rec_prim) ? 1u : 0u;
    if (P.cull)
        for (uint32_t f = 0; f < frames; ++f) P.cull_rect[f] = cull_rect(P.cam[f], P.root_box, P.W, P.H);
    P.pairs = s->d_pairs; P.nodes4 = s->d_nodes4; P.tris = s->d_tris; P.orig = s->d_orig; P.norms = s->d_norms;
    P.qnodes4 = s->d_qnodes4;
    P.pixels = d_pixels; P.rgb8 = d_rgb8; P.shards = s->d_shards;
    P.rec_prim = d_rec_prim; P.rec_tuv = d_rec_tuv; P.rec_shadow = d_rec_shadow;

    const bool stats = (s->flags & CERES_SCENE_STATS) != 0;
    const bool full = mode == CERES_MODE_FULL;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (s->timing && rows) {
        while (s->ev_pool.size() < 2) { hipEvent_t e; HIP_TRY(hipEventCreate(&e)); s->ev_pool.push_back(e); }
        e0 = s->ev_pool.back(); s->ev_pool.pop_back();
        e1 = s->ev_pool.back(); s->ev_pool.pop_back();
        s->ev_used.push_back(e0); s->ev_used.push_back(e1);
    }
    constexpr uint32_t ftile = 8;                                    // fused kernel: 8x8 tiles
    const uint32_t fbx = uint32_t((W + ftile - 1) / ftile), fby = uint32_t((rows + ftile - 1) / ftile);
    const uint32_t* tile_order = nullptr;
    const bool packed = frames <= (1u << (32 - kTileXBits - kTileYBits)) &&
                        fbx <= (1u << kTileXBits) && fby <= (1u << kTileYBits);
    // tiles per wavefront of the fused kernel: 1 for the stealing single-frame and the stats
    // kernels; batch_tiles_per_wave for batches (the kernel instantiation must match the order)
    const uint32_t tpw = (!stats && (frames > 1 || t.bands)) ? batch_tiles_per_wave(size_t(W) * rows, stack_width(s->n_pairs, s->n_nodes4), qbvh)
                                                : 1u;
    if (full && rows)
        if (int rc = ensure_tile_order(s, W, H, t, rows, frames, fbx, fby, ftile, stream, &tile_order, packed, tpw)) return rc;
    // The shards must start at zero when they are read back (counters) or count primary-only hits;
    // the fused kernel without counters only adds to them, so its steady-state frames skip the
    // memset (ceres_finalize re-zeroes them after every counted render).
    const bool need_clean = d_counters || !full;
    if (first && need_clean && s->shards_dirty) HIP_TRY(hipMemsetAsync(s->d_shards, 0, sizeof(Shard) * kShards, stream));
    s->shards_dirty = true;
    if (rows) {                                                      // a rank may own no rows
        if (e0) HIP_TRY(hipEventRecord(e0, stream));
        if (full) {
            // one kernel: primary + shadow + shading per 8x8 tile
            const int stw = stack_width(s->n_pairs, s->n_nodes4);
            const bool st16 = stw == 2;
            // work stealing for one-frame launches (latency), one ray per lane for batches (throughput)
            const bool steal = frames == 1 && !t.bands;            // band launches: the batch kernel
            // BVH4 stack: the batch kernels' walks descend into the first passing child and need
            // only shadow_stack_first entries (order_shadow_bvh4); the stealing loop descends into
            // the nearest child (bunny solo -20 % against first-child order) and needs the
            // nearest-first bound -- unless that bound's LDS costs waves (C5: 37 entries x 3 B x
            // 64 lanes + the stealing mailboxes = 7.9 KB, 5 waves per SIMD; the first-child bound,
            // 27, fits the primary stack's 28: 6.1 KB), and there the loop takes the first
            // passing child too (scene creation ordered those scenes' records for it)
            P.steal_first = steal && !stats && ((s->flags & CERES_SCENE_FIRST_ORDER) ||
                                                lds_limits_waves(std::max(s->stack_entries + 1, s->shadow_stack_entries), stw))
                                ? 1u : 0u;
            P.shadow_stack_entries = (!steal || P.steal_first) ? s->shadow_stack_first : s->shadow_stack_entries;
            P.lds_entries = uint32_t(std::max(s->stack_entries + 1, P.shadow_stack_entries));
            const size_t flds = size_t(P.lds_entries) * dev::kFusedB * stw;
            if (int rc = check_fused_lds(s, P, stw, flds)) return rc;
            // Test hook (tests/test_gpu_hardening.py): CERES_DEBUG_GUARD_SLOT=k moves the production
            // kernels' stack guard (guarded_trace) down to slot k < stack_entries -- a slot deep walks
            // legitimately write -- so the overflow report can be exercised without a broken bound.
            // Only the guard's position changes: the LDS carve-up above and every stack index stay.
            if (!stats)
                if (const char* g = std::getenv("CERES_DEBUG_GUARD_SLOT")) {
                    const long k = std::strtol(g, nullptr, 10);
                    if (k > 0 && uint32_t(k) < P.stack_entries) P.stack_entries = uint32_t(k);
                }
            P.tile_order = tile_order;
            P.tile_packed = packed ? 1u : 0u;
            P.tiles_x = fbx;
            P.row_blocks_per_frame = fby;
            const uint32_t n_tiles = fbx * fby * frames;
            const dim3 fgrid((n_tiles + tpw - 1) / tpw), fblock(dev::kFusedB);
            if (stats) {                                             // per-wave diagnostic timeline
                const size_t waves = size_t(fbx) * fby * frames;
                if (s->wave_log_waves < waves) {
                    dfree(s->d_wave_log);
                    HIP_TRY(hipMalloc(&s->d_wave_log, waves * 64));
                    s->wave_log_waves = waves;
                }
                HIP_TRY(hipMemsetAsync(s->d_wave_log, 0, waves * 64, stream));
                P.wave_log = s->d_wave_log;
                s->last_grid_waves = waves;
            }
            // VGPR budgets: 16-bit-stack scenes (LDS for 7+ waves/SIMD) are compiled for 7 waves,
            // C5-size scenes keep the unconstrained allocation
            constexpr int w32 = CERES_FUSED_MINW32;
            auto fused = [&](auto rt, auto st, auto gt) {
                constexpr bool R = decltype(rt)::value, T = decltype(st)::value, G = decltype(gt)::value;
                constexpr int w16 = T ? CERES_FUSED_MINW16_SOLO : CERES_FUSED_MINW16;
                if constexpr (!R) {
                    if (qbvh) {                                      // compressed shadow BVH4 (non-stats, fast slabs)
                        if (st16) hipLaunchKernelGGL((dev::ceres_fused<false, uint16_t*, w16, false, T, true, G>), fgrid, fblock, flds, stream, P);
                        else if (stw == 3) hipLaunchKernelGGL((dev::ceres_fused<false, dev::Stk24, w32, false, T, true, G>), fgrid, fblock, flds, stream, P);
                        else hipLaunchKernelGGL((dev::ceres_fused<false, uint32_t*, w32, false, T, true, G>), fgrid, fblock, flds, stream, P);
                        return;
                    }
                }
                if (stats && st16) hipLaunchKernelGGL((dev::ceres_fused<true, uint16_t*, 1, R, T, false, G>), fgrid, fblock, flds, stream, P);
                else if (stats && stw == 3) hipLaunchKernelGGL((dev::ceres_fused<true, dev::Stk24, w32, R, T, false, G>), fgrid, fblock, flds, stream, P);
                else if (stats) hipLaunchKernelGGL((dev::ceres_fused<true, uint32_t*, w32, R, T, false, G>), fgrid, fblock, flds, stream, P);
                else if (st16) {
                    if constexpr (!T) {                              // batches: tiles per wave by frame size
                        if (tpw == 2) { hipLaunchKernelGGL((dev::ceres_fused<false, uint16_t*, w16, R, T, false, G, 2>), fgrid, fblock, flds, stream, P); return; }
                    }
                    constexpr int w16b = T ? CERES_FUSED_MINW16_SOLO : CERES_FUSED_MINW16_TPW4;
                    hipLaunchKernelGGL((dev::ceres_fused<false, uint16_t*, w16b, R, T, false, G>), fgrid, fblock, flds, stream, P);
                }
                else if (stw == 3) hipLaunchKernelGGL((dev::ceres_fused<false, dev::Stk24, w32, R, T, false, G>), fgrid, fblock, flds, stream, P);
                else hipLaunchKernelGGL((dev::ceres_fused<false, uint32_t*, w32, R, T, false, G>), fgrid, fblock, flds, stream, P);
            };
            auto fused_g = [&](auto rt, auto st) {
                if (gfma) fused(rt, st, std::true_type{});
                else fused(rt, st, std::false_type{});
            };
            auto fused_s = [&](auto rt) {
                if (steal) fused_g(rt, std::true_type{});
                else fused_g(rt, std::false_type{});
            };
            // ceres_tiling.bands: their own instantiations of the batch kernel (kBands)
            auto fused_bands = [&](auto gt) {
                constexpr bool G = decltype(gt)::value;
                if (st16) {
                    if (tpw == 2) hipLaunchKernelGGL((dev::ceres_fused<false, uint16_t*, CERES_FUSED_MINW16, false, false, false, G, 2, true>), fgrid, fblock, flds, stream, P);
                    else hipLaunchKernelGGL((dev::ceres_fused<false, uint16_t*, CERES_FUSED_MINW16_TPW4, false, false, false, G, 0, true>), fgrid, fblock, flds, stream, P);
                } else if (stw == 3) hipLaunchKernelGGL((dev::ceres_fused<false, dev::Stk24, w32, false, false, false, G, 0, true>), fgrid, fblock, flds, stream, P);
                else hipLaunchKernelGGL((dev::ceres_fused<false, uint32_t*, w32, false, false, false, G, 0, true>), fgrid, fblock, flds, stream, P);
            };
            if (t.bands) {
                if (gfma) fused_bands(std::true_type{});
                else fused_bands(std::false_type{});
            } else if (robust) fused_s(std::true_type{});
            else fused_s(std::false_type{});
        } else {
            const size_t lds = size_t(s->stack_entries + 1) * dev::kBlock * 4;
            if (lds > s->max_lds_per_block)
                return set_error(CERES_EINVAL, "render: primary-only traversal stack needs %zu B of LDS per workgroup (%zu available)",
                                 lds, s->max_lds_per_block);
            const dim3 grid(bx, by * frames), block(dev::kBlock);
            auto primary = [&](auto rt, auto gt) {
                constexpr bool R = decltype(rt)::value, G = decltype(gt)::value;
                if (stats) hipLaunchKernelGGL((dev::ceres_primary<true, R, G>), grid, block, lds, stream, P);
                else hipLaunchKernelGGL((dev::ceres_primary<false, R, G>), grid, block, lds, stream, P);
            };
            auto primary_g = [&](auto rt) {
                if (gfma) primary(rt, std::true_type{});
                else primary(rt, std::false_type{});
            };
            if (robust) primary_g(std::true_type{});
            else primary_g(std::false_type{});
        }
        HIP_TRY(hipGetLastError());
        if (e1) HIP_TRY(hipEventRecord(e1, stream));
    }
    if (d_counters && last) {
        hipLaunchKernelGGL(dev::ceres_finalize, dim3(1), dim3(64), 0, stream, s->d_shards,
                           batch_primary, d_counters);
        HIP_TRY(hipGetLastError());
        s->shards_dirty = false;
    }
    return CERES_OK;
}

// One batch call of 1..kMaxFrames frames: launches of at most kFramesPerLaunch frames on `stream`,
// frame f's outputs at offset f x W x local rows (pixels x 3) as in one launch.
int launch(ceres_scene* s, uint32_t frames, const float* basis12, const float* sun, int mode, size_t W, size_t H,
           const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, hipStream_t stream,
           int32_t* d_rec_prim = nullptr, float* d_rec_tuv = nullptr, int8_t* d_rec_shadow = nullptr) {
    if (frames == 0 || frames > uint32_t(kMaxFrames))
        return set_error(CERES_EINVAL, "render: %u frames per batch (1..%d)", frames, kMaxFrames);
    if (!basis12 || !sun) return set_error(CERES_EINVAL, "render: null argument");
    ceres_tiling t{uint32_t(H), 0, 1};
    if (tiling) t = *tiling;
    if (t.world == 0 || t.rank >= t.world || t.row_block == 0) return set_error(CERES_EINVAL, "render: bad tiling");
    // the batch's primary rays (render.hpp:102: one per pixel this rank renders): with bands, a
    // frame's band may end below its row_block rows (the last band of the frame)
    uint64_t primary = uint64_t(frames) * W * local_rows_of(H, t);
    if (t.bands && t.world > 1) {
        primary = 0;
        for (uint32_t f = 0; f < frames; ++f) {
            const size_t b = (t.rank + f) % t.world, top = b * size_t(t.row_block);
            primary += uint64_t(W) * (top < H ? std::min<size_t>(t.row_block, H - top) : 0);
        }
    }
    if (frames <= uint32_t(kFramesPerLaunch))
        return launch_chunk(s, frames, basis12, sun, mode, W, H, tiling, d_pixels, d_rgb8, d_counters, stream, d_rec_prim,
                            d_rec_tuv, d_rec_shadow, true, true, primary);
    const size_t fp = W * local_rows_of(H, t);                      // pixels per frame on this rank
    // equal chunks (64 frames: 32 + 32, not 56 + 8 -- a small last launch is all tail)
    const uint32_t n_launch = (frames + kFramesPerLaunch - 1) / kFramesPerLaunch;
    for (uint32_t c = 0, f0 = 0; c < n_launch; ++c) {
        const uint32_t n = frames / n_launch + (c < frames % n_launch ? 1u : 0u);
        const size_t o = size_t(f0) * fp;
        // bands: the chunk's frame 0 is the call's frame f0, so its band rotation starts at rank + f0
        ceres_tiling tc = t;
        if (t.bands) tc.rank = (t.rank + f0) % t.world;
        if (int rc = launch_chunk(s, n, basis12 + 12 * size_t(f0), sun + 3 * size_t(f0), mode, W, H, &tc,
                                  d_pixels ? d_pixels + 3 * o : nullptr, d_rgb8 ? d_rgb8 + 3 * o : nullptr, d_counters,
                                  stream, d_rec_prim ? d_rec_prim + o : nullptr, d_rec_tuv ? d_rec_tuv + 3 * o : nullptr,
                                  d_rec_shadow ? d_rec_shadow + o : nullptr, f0 == 0, f0 + n >= frames, primary))
            return rc;
        f0 += n;
    }
    return CERES_OK;
}

void fill_stats(ceres_stats* st, const uint64_t c[8], double ms) {
    if (!st) return;
    st->rays = c[0]; st->hits = c[1]; st->primary_rays = c[2]; st->shadow_rays = c[3];
    st->node_pairs = c[4]; st->tri_tests = c[5]; st->ms = ms;
}

}  // namespace

namespace ceres {
int frame_tile_order(ceres_scene* s, size_t W, size_t H, uint32_t tile, hipStream_t stream, const uint32_t** out) {
    const ceres_tiling t{uint32_t(H), 0, 1};
    return ensure_tile_order(s, W, H, t, H, 1, uint32_t((W + tile - 1) / tile), uint32_t((H + tile - 1) / tile), tile,
                             stream, out, false, 1u);
}
}  // namespace ceres

extern "C" {

const char* ceres_last_error(void) { return error_buffer(); }
extern const char ceres_src_sha[];     // build_info.o (Makefile): sha256 of the sources, 16 hex digits
const char* ceres_version(void) {
    static const std::string v = std::string("ceres-mi355x 0.3 (gfx950) src ") + ceres_src_sha;
    return v.c_str();
}
int ceres_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return set_error(CERES_EHIP, "hipGetDeviceCount failed");
    return n;
}
const char* ceres_kernel_names(void) {
    return "ceres_fused,ceres_primary,ceres_finalize,ceres_assemble";
}

size_t ceres_tiling_local_rows(size_t height, const ceres_tiling* t) {
    if (!t) return height;
    if (t->world == 0 || t->row_block == 0 || t->rank >= t->world) return 0;
    return local_rows_of(height, *t);
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
    if (relayout_bvh(static_cast<const RefNode*>(nodes32), n_nodes, prim64, n_tri, reinterpret_cast<const Tri48*>(tri48),
                     pairs, leaf_tris, orig, depth, rlc, rlf))
        return nullptr;
    std::vector<Node4> nodes4;
    uint32_t stack4 = 0, not_collapsed = 0;
    if (!rlc && build_shadow_bvh4(pairs, nodes4, stack4, not_collapsed)) return nullptr;

    // scenes whose nearest-first BVH4 stack costs waves (lds_limits_waves) get their inner
    // children ordered for the first-passing-child bound (order_shadow_bvh4; their single-frame
    // launches then walk in that order); the others keep the build order, which the nearest-first
    // stealing loop prefers (reordered: C3 solo +4 %, bunny +2 %, profiles/r05/s19)
    uint32_t stack4_first = stack4;
    if (!rlc && ((flags & CERES_SCENE_FIRST_ORDER) ||
                 lds_limits_waves(std::max(depth + 1, stack4), stack_width(pairs.size(), nodes4.size()))) &&
        order_shadow_bvh4(nodes4, stack4_first))
        return nullptr;
    if (nodes4.empty()) nodes4.emplace_back();
    auto* s = new (std::nothrow) ceres_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    s->n_nodes4 = nodes4.size();
    s->shadow_stack_entries = std::max<uint32_t>(1, stack4);
    s->shadow_stack_first = std::max<uint32_t>(1, std::min(stack4, stack4_first));
    s->device = device; s->flags = flags; s->n_tri = n_tri; s->n_pairs = pairs.size();
    s->depth = depth; s->root_leaf_count = rlc; s->root_leaf_first = rlf;
    s->stack_entries = std::max<uint32_t>(1, depth);                 // stack <= depth - 1 entries
    set_root_box(s, static_cast<const RefNode*>(nodes32)[0].bounds, pairs[0]);
    auto fail = [&]() -> ceres_scene* { scene_release(s); delete s; return nullptr; };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { set_error(CERES_EHIP, "no HIP device available"); return fail(); }
    if (device < 0 || device >= ndev) { set_error(CERES_EINVAL, "device %d out of range (%d devices)", device, ndev); return fail(); }
    auto body = [&]() -> int {
        HIP_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_error(CERES_EHIP, "device %d is %s, this build targets gfx950 only", device, prop.gcnArchName);
        s->num_cus = prop.multiProcessorCount;
        s->max_lds_per_block = prop.sharedMemPerBlock;
        HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        HIP_TRY(hipMalloc(&s->d_pairs, pairs.size() * sizeof(SiblingPair)));
        HIP_TRY(hipMalloc(&s->d_nodes4, nodes4.size() * sizeof(Node4)));
        HIP_TRY(hipMemcpy(s->d_nodes4, nodes4.data(), nodes4.size() * sizeof(Node4), hipMemcpyHostToDevice));
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
    if (body()) return fail();
    return s;
}

// Scene from arrays already in HBM (device `device`): the reference's Triangle[] / tri_norms
// (e.g. from ceres_obj_parse_device + ceres_rotate_triangles_device) and a BVH with u32
// primitive_indices (e.g. from ceres_bvh_build_device); relayout on the GPU (scene_device.hip).
// The caller keeps its buffers.  Work is ordered on `stream` (NULL: the scene's own stream).
ceres_scene* ceres_scene_create_device(const float* d_tri48, size_t n_tri, const float* d_norm36, const uint32_t* d_nodes32,
                                       size_t n_nodes, const uint32_t* d_prim32, int device, uint32_t flags, void* stream) {
    if (!d_tri48 || !d_norm36 || !d_nodes32 || !d_prim32 || n_tri == 0 || n_nodes == 0) {
        set_error(CERES_EINVAL, "ceres_scene_create_device: empty scene or null argument");
        return nullptr;
    }
    if (n_tri > 0xffffffffull || n_nodes > 0xffffffffull) { set_error(CERES_EUNSUPPORTED, "scene too large"); return nullptr; }
    auto* s = new (std::nothrow) ceres_scene;
    if (!s) { set_error(CERES_ENOMEM, "out of host memory"); return nullptr; }
    DeviceLayout L;
    auto fail = [&]() -> ceres_scene* {
        if (L.pairs) (void)hipFree(L.pairs);
        if (L.nodes4) (void)hipFree(L.nodes4);
        if (L.tris) (void)hipFree(L.tris);
        if (L.orig) (void)hipFree(L.orig);
        scene_release(s); delete s; return nullptr;
    };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { set_error(CERES_EHIP, "no HIP device available"); return fail(); }
    if (device < 0 || device >= ndev) { set_error(CERES_EINVAL, "device %d out of range (%d devices)", device, ndev); return fail(); }
    s->device = device; s->flags = flags; s->n_tri = n_tri;
    auto body = [&]() -> int {
        HIP_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_error(CERES_EHIP, "device %d is %s, this build targets gfx950 only", device, prop.gcnArchName);
        s->num_cus = prop.multiProcessorCount;
        s->max_lds_per_block = prop.sharedMemPerBlock;
        HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
        if (int rc = relayout_device(reinterpret_cast<const Tri48*>(d_tri48), uint32_t(n_tri),
                                     reinterpret_cast<const RefNode*>(d_nodes32), uint32_t(n_nodes), d_prim32, st, L))
            return rc;
        s->d_pairs = L.pairs; s->d_nodes4 = L.nodes4; s->d_tris = L.tris; s->d_orig = L.orig;
        s->n_pairs = L.n_pairs; s->n_nodes4 = L.n_nodes4;
        s->depth = L.depth; s->root_leaf_count = L.root_leaf_count; s->root_leaf_first = L.root_leaf_first;
        s->stack_entries = std::max<uint32_t>(1, L.depth);           // stack <= depth - 1 entries
        s->shadow_stack_entries = std::max<uint32_t>(1, L.stack4);
        s->shadow_stack_first = s->shadow_stack_entries;              // device records keep build order
        if (!L.root_leaf_count) {
            SiblingPair p0;
            HIP_TRY(hipMemcpyAsync(&p0, L.pairs, sizeof p0, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            set_root_box(s, L.root_box, p0);
        }
        L = DeviceLayout{};                                          // owned by the scene now
        HIP_TRY(hipMalloc(&s->d_norms, n_tri * 36));
        HIP_TRY(hipMemcpyAsync(s->d_norms, d_norm36, n_tri * 36, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMalloc(&s->d_shards, sizeof(Shard) * kShards));
        HIP_TRY(hipMalloc(&s->d_counters, 8 * sizeof(uint64_t)));
        HIP_TRY(hipStreamSynchronize(st));
        return CERES_OK;
    };
    if (body()) return fail();
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
    if (device_bytes)
        *device_bytes = s->n_pairs * sizeof(SiblingPair) + s->n_nodes4 * sizeof(Node4) + s->n_tri * (sizeof(Tri48) + 4 + 36);
    return CERES_OK;
}

int ceres_scene_shadow_stacks(const ceres_scene* s, uint32_t* nearest_first, uint32_t* first_passing) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    if (nearest_first) *nearest_first = s->shadow_stack_entries;
    if (first_passing) *first_passing = s->shadow_stack_first;
    return CERES_OK;
}

int ceres_render_device(ceres_scene* s, const float basis12[12], const float sun[3], int mode, size_t W, size_t H,
                        const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, void* stream) {
    return launch(s, 1, basis12, sun, mode, W, H, tiling, d_pixels, d_rgb8, d_counters, static_cast<hipStream_t>(stream));
}

int ceres_render_batch_device(ceres_scene* s, uint32_t frames, const float* basis12, const float* sun3, int mode,
                              size_t W, size_t H, const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8,
                              uint64_t* d_counters, void* stream) {
    return launch(s, frames, basis12, sun3, mode, W, H, tiling, d_pixels, d_rgb8, d_counters,
                  static_cast<hipStream_t>(stream));
}

// Workgroup rows of the un-interleave grid (its y extent; each workgroup strides over the output
// rows).  A grid of one workgroup per output row (16 x 1080-row frames: 34,560 workgroups) floods
// the dispatcher and takes wave slots from the render launches it runs beside (the exchange's
// assembly overlaps the next steps' renders); a bounded grid copies in the background.
// CERES_ASSEMBLE_ROWS overrides (A/B; 0 = one workgroup per row).
constexpr size_t kAssembleGridRows = 65535;   // default cap (A/B pending)
static uint32_t assemble_grid_rows(size_t out_rows) {
    static const long env = [] { const char* e = std::getenv("CERES_ASSEMBLE_ROWS"); return e ? std::strtol(e, nullptr, 10) : -1L; }();
    const size_t cap = env < 0 ? size_t(kAssembleGridRows) : env == 0 ? size_t(65535) : size_t(env);
    return uint32_t(std::max<size_t>(1, std::min<size_t>({out_rows, cap, 65535})));
}

int ceres_assemble_rgb8(const uint8_t* d_gathered, size_t rank_stride_bytes, uint8_t* d_out, uint32_t frames,
                        size_t W, size_t H, uint32_t row_block, uint32_t world, void* stream) {
    if (!d_gathered || !d_out || frames == 0 || W == 0 || H == 0 || row_block == 0 || world == 0)
        return set_error(CERES_EINVAL, "ceres_assemble_rgb8: bad argument");
    if (3 * W > 0xffffffffull || size_t(frames) * H > 0xffffffffull)
        return set_error(CERES_EINVAL, "ceres_assemble_rgb8: frame too large");
    const size_t max_rows = local_rows_of(H, row_block, 0, world);     // rank 0 owns the most rows
    if (rank_stride_bytes < size_t(frames) * max_rows * 3 * W)
        return set_error(CERES_EINVAL, "ceres_assemble_rgb8: rank stride smaller than a rank's batch");
    const uint32_t row_bytes = uint32_t(3 * W);
    const bool vec = row_bytes % 16 == 0 && rank_stride_bytes % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(d_gathered) % 16 == 0 && reinterpret_cast<uintptr_t>(d_out) % 16 == 0;
    const uint32_t units = vec ? row_bytes / 16 : row_bytes;
    const dim3 grid(uint32_t(std::min<size_t>((units + 255) / 256, 64)), assemble_grid_rows(size_t(frames) * H));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (vec)
        hipLaunchKernelGGL(dev::ceres_assemble<true>, grid, dim3(256), 0, st, d_gathered, rank_stride_bytes, d_out,
                           frames, uint32_t(H), row_bytes, row_block, world);
    else
        hipLaunchKernelGGL(dev::ceres_assemble<false>, grid, dim3(256), 0, st, d_gathered, rank_stride_bytes, d_out,
                           frames, uint32_t(H), row_bytes, row_block, world);
    HIP_TRY(hipGetLastError());
    return CERES_OK;
}

int ceres_assemble_rgb8_packed(const uint8_t* d_gathered, uint8_t* d_out, uint32_t frames, size_t W, size_t H,
                               uint32_t row_block, uint32_t world, void* stream) {
    if (!d_gathered || !d_out || frames == 0 || W == 0 || H == 0 || row_block == 0 || world == 0)
        return set_error(CERES_EINVAL, "ceres_assemble_rgb8_packed: bad argument");
    if (3 * W > 0xffffffffull || size_t(frames) * H > 0xffffffffull)
        return set_error(CERES_EINVAL, "ceres_assemble_rgb8_packed: frame too large");
    const uint32_t row_bytes = uint32_t(3 * W);
    const bool vec = row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(d_gathered) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(d_out) % 16 == 0;
    const uint32_t units = vec ? row_bytes / 16 : row_bytes;
    const dim3 grid(uint32_t(std::min<size_t>((units + 255) / 256, 64)), assemble_grid_rows(size_t(frames) * H));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (vec)
        hipLaunchKernelGGL((dev::ceres_assemble<true, true>), grid, dim3(256), 0, st, d_gathered, size_t(0), d_out, frames,
                           uint32_t(H), row_bytes, row_block, world);
    else
        hipLaunchKernelGGL((dev::ceres_assemble<false, true>), grid, dim3(256), 0, st, d_gathered, size_t(0), d_out, frames,
                           uint32_t(H), row_bytes, row_block, world);
    HIP_TRY(hipGetLastError());
    return CERES_OK;
}

// Row bands of a host-buffer render (ceres_render_f32).  The call's length is set by the copy of
// the framebuffer over the host link (C3: 24.9 MB of floats, ~0.45 ms at ~55 GB/s, against a
// 0.17-ms kernel), so the frame is rendered as `bands` launches of contiguous row bands on the
// scene stream and each band's rows are copied out on a second stream as soon as its kernel
// ends: the copies start after the first band instead of after the whole frame.  Each pixel is
// computed alone (render.hpp:104-153), so the bytes are those of one launch.  Measured on one
// MI355X (profiles/r03/e2e): dragon 4096^2 float frame 4.04 -> 3.73 ms per call, RGB8 (./render)
// 1.32 -> 1.04 ms with 4 bands; at 1080p the bands' own tails cost what the overlap saves (floats
// +-2 %, RGB8 +60 %), so frames under kBandMinBytes stay one launch.  CERES_HOST_BANDS overrides
// the count (1 = one launch, then the copy).
// at most half the tile-order cache: each band caches its own order ({rb, k, bands} keys), and a
// band count near kMaxTileOrders would evict every cached order on each call (each eviction
// round ends in a bulk free behind a device synchronise)
constexpr uint32_t kMaxHostBands = 8;
static_assert(2 * kMaxHostBands <= ceres::kMaxTileOrders, "host bands must leave room in the tile-order cache");
constexpr size_t kBandMinBytes = size_t(32) << 20;     // below this a frame is one launch (measured: 1080p floats ±2 %, 1080p RGB8 +60 %)

// The compacted float readback (ceres_render_f32): one launch, ceres_compact_lit, a 4-B count
// copy, then only the lit pixels' 16-B records cross the host link; meanwhile the caller's cores
// zero the float framebuffer (host_fill_zero), and the records are scattered over it.  C3: ~7 %
// of the pixels are lit, so ~2 MB cross the link instead of 24.9 MB.  Frames with more than half
// their pixels lit take the full copy (16-B records would not pay).
constexpr double kCompactMaxLitFrac = 0.5;
static int render_f32_compact(ceres_scene* s, const float basis12[12], const float sun[3], int mode, float* pixels,
                              uint8_t* rgb8, size_t W, size_t H, ceres_stats* stats) {
    const size_t np = W * H;
    // records for at most kCompactMaxLitFrac of the pixels (a full-frame record buffer
    // was 1.33x the float framebuffer); a denser frame overflows it and takes the full copy.
    // Round 6: the records go straight into pinned host memory (the compaction kernel's stores
    // cross the host link as it runs: no separate copy, one synchronisation per call instead of
    // two); CERES_COMPACT_ZC=0 keeps the device buffer + copy.
    static const bool zc = [] { const char* e = std::getenv("CERES_COMPACT_ZC"); return !(e && e[0] == '0'); }();
    const size_t cap = size_t(double(np) * kCompactMaxLitFrac) + 1;
    if (s->lit_cap < cap || s->lit_zc != zc) {
        dfree(s->d_lit);
        if (s->h_lit_pinned) { (void)hipHostFree(s->h_lit_pinned); s->h_lit_pinned = nullptr; }
        if (zc) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->h_lit_pinned), cap * sizeof(uint4)));
        else HIP_TRY(hipMalloc(&s->d_lit, cap * sizeof(uint4)));
        s->lit_cap = cap;
        s->lit_zc = zc;
    }
    uint4* lit_out = zc ? s->h_lit_pinned : s->d_lit;
    if (!s->d_lit_count) HIP_TRY(hipMalloc(&s->d_lit_count, sizeof(uint32_t)));
    if (!s->h_small) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->h_small), 16 * sizeof(uint64_t)));
    if (!s->ev_count) HIP_TRY(hipEventCreateWithFlags(&s->ev_count, hipEventDisableTiming));
    if (!s->d_band_counters) HIP_TRY(hipMalloc(&s->d_band_counters, kMaxHostBands * 8 * sizeof(uint64_t)));
    while (s->band_events.size() < kMaxHostBands + 2) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        s->band_events.push_back(e);
    }
    hipEvent_t a = s->band_events[kMaxHostBands], b = s->band_events[kMaxHostBands + 1];
    HIP_TRY(hipMemsetAsync(s->d_lit_count, 0, sizeof(uint32_t), s->stream));
    HIP_TRY(hipEventRecord(a, s->stream));
    if (int rc = launch(s, 1, basis12, sun, mode, W, H, nullptr, s->d_pixels, rgb8 ? s->d_rgb8 : nullptr,
                        s->d_band_counters, s->stream))
        return rc;
    HIP_TRY(hipEventRecord(b, s->stream));
    hipLaunchKernelGGL(dev::ceres_compact_lit, dim3(uint32_t((np + 255) / 256)), dim3(256), 0, s->stream, s->d_pixels,
                       uint32_t(np), lit_out, s->d_lit_count, uint32_t(cap));
    HIP_TRY(hipGetLastError());
    uint64_t* hs = reinterpret_cast<uint64_t*>(s->h_small);
    HIP_TRY(hipMemcpyAsync(hs + 8, s->d_band_counters, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipMemcpyAsync(hs, s->d_lit_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipEventRecord(s->ev_count, s->stream));
    host_fill_zero(pixels, 3 * np);                                  // the caller's cores, while the GPU renders
    HIP_TRY(hipEventSynchronize(s->ev_count));
    const size_t n = *reinterpret_cast<const uint32_t*>(hs);
    if (n > np) return set_error(CERES_EHIP, "render: compacted pixel count %zu exceeds the frame", n);
    const bool dense = n > cap;                                      // records overflowed: the full copy
    if (dense)
        HIP_TRY(hipMemcpyAsync(pixels, s->d_pixels, 3 * np * sizeof(float), hipMemcpyDeviceToHost, s->stream));
    else if (n && !zc) {
        if (s->h_lit.size() < n) s->h_lit.resize(n);
        HIP_TRY(hipMemcpyAsync(s->h_lit.data(), s->d_lit, n * sizeof(uint4), hipMemcpyDeviceToHost, s->stream));
    }
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, s->d_rgb8, 3 * np, hipMemcpyDeviceToHost, s->stream));
    if (dense || (n && !zc) || rgb8) HIP_TRY(hipStreamSynchronize(s->stream));
    if (!dense)                                                       // (zero-copy: complete at ev_count)
        host_scatter_lit(pixels, reinterpret_cast<const uint32_t*>(zc ? s->h_lit_pinned : s->h_lit.data()), n);
    s->last_lit_frac = double(n) / double(np);
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    uint64_t c[8];
    std::memcpy(c, hs + 8, sizeof(c));
    fill_stats(stats, c, ms);
    if (c[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

static uint32_t host_bands(size_t W, size_t H, bool pixels, bool rgb8) {
    uint32_t b = 4;
    if (const char* e = std::getenv("CERES_HOST_BANDS")) b = uint32_t(std::max(1, std::atoi(e)));
    const size_t bytes = W * H * 3 * ((pixels ? sizeof(float) : 0) + (rgb8 ? 1 : 0));
    if (bytes < kBandMinBytes) b = 1;
    return uint32_t(std::min<size_t>({size_t(b), size_t(kMaxHostBands), H}));
}

int ceres_render_f32(ceres_scene* s, const float basis12[12], const float sun[3], int mode, float* pixels,
                     uint8_t* rgb8, size_t W, size_t H, ceres_stats* stats) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    if (int rc = ensure_workspace(s, W * H, pixels != nullptr, rgb8 != nullptr)) return rc;
    // float framebuffers: the compacted readback unless the last frames were dense (re-tried
    // every 32nd call); CERES_COMPACT=0 forces the full copy
    static const bool no_compact = [] { const char* e = std::getenv("CERES_COMPACT"); return e && e[0] == '0'; }();
    if (pixels && !no_compact && W * H <= 0xffffffffull &&
        (s->last_lit_frac < kCompactMaxLitFrac || (++s->dense_calls & 31u) == 0))
        return render_f32_compact(s, basis12, sun, mode, pixels, rgb8, W, H, stats);
    const uint32_t want = host_bands(W, H, pixels != nullptr, rgb8 != nullptr);
    const uint32_t rb = uint32_t((H + want - 1) / want);
    const uint32_t bands = uint32_t((H + rb - 1) / rb);
    if (!s->d_band_counters) HIP_TRY(hipMalloc(&s->d_band_counters, kMaxHostBands * 8 * sizeof(uint64_t)));
    if (bands > 1 && !s->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&s->copy_stream, hipStreamNonBlocking));
    while (s->band_events.size() < kMaxHostBands + 2) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        s->band_events.push_back(e);
    }
    hipEvent_t a = s->band_events[kMaxHostBands], b = s->band_events[kMaxHostBands + 1];
    HIP_TRY(hipEventRecord(a, s->stream));
    for (uint32_t k = 0; k < bands; ++k) {
        // band k = global rows [j0, j1): one block of the tiling {rb, k, bands}; its float rows sit
        // at row j0 of the framebuffer (row 0 at the bottom), its PPM rows (flipped) at H - j1
        const size_t j0 = size_t(k) * rb, j1 = std::min<size_t>(H, j0 + rb);
        const ceres_tiling t{rb, k, bands};
        if (int rc = launch(s, 1, basis12, sun, mode, W, H, &t, pixels ? s->d_pixels + 3 * W * j0 : nullptr,
                            rgb8 ? s->d_rgb8 + 3 * W * (H - j1) : nullptr, s->d_band_counters + 8 * k, s->stream))
            return rc;
        HIP_TRY(hipEventRecord(s->band_events[k], s->stream));
    }
    HIP_TRY(hipEventRecord(b, s->stream));
    hipStream_t cs = bands > 1 ? s->copy_stream : s->stream;
    for (uint32_t k = 0; k < bands; ++k) {
        const size_t j0 = size_t(k) * rb, j1 = std::min<size_t>(H, j0 + rb);
        if (bands > 1) HIP_TRY(hipStreamWaitEvent(cs, s->band_events[k], 0));
        if (pixels)
            HIP_TRY(hipMemcpyAsync(pixels + 3 * W * j0, s->d_pixels + 3 * W * j0, 3 * W * (j1 - j0) * sizeof(float),
                                   hipMemcpyDeviceToHost, cs));
        if (rgb8)
            HIP_TRY(hipMemcpyAsync(rgb8 + 3 * W * (H - j1), s->d_rgb8 + 3 * W * (H - j1), 3 * W * (j1 - j0),
                                   hipMemcpyDeviceToHost, cs));
    }
    uint64_t cb[kMaxHostBands * 8] = {0};
    HIP_TRY(hipMemcpyAsync(cb, s->d_band_counters, bands * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (bands > 1) HIP_TRY(hipStreamSynchronize(cs));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    uint64_t c[8] = {0};
    for (uint32_t k = 0; k < bands; ++k)
        for (int i = 0; i < 8; ++i) c[i] = i == 6 ? std::max(c[i], cb[8 * k + i]) : c[i] + cb[8 * k + i];
    fill_stats(stats, c, ms);
    if (c[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

// Single-process multi-GPU frame (the `./render --gpus N` path): rank r renders its rows
// (ceres_tiling {row_block, r, world}) on scenes[r]'s device and stream; the RGB8 rows travel
// to scenes[0]'s device peer-to-peer (hipMemcpyPeerAsync: xGMI between MI355X devices), where
// ceres_assemble_rgb8 un-interleaves them into the PPM body -- one copy to the host.  Float
// pixels (optional) come back per rank and are scattered by row on the host.
int ceres_render_multi_f32(ceres_scene* const* scenes, uint32_t world, uint32_t row_block, const float basis12[12],
                           const float sun[3], int mode, float* pixels, uint8_t* rgb8, size_t W, size_t H,
                           ceres_stats* stats) {
    if (!scenes || world == 0 || row_block == 0 || !basis12 || !sun || (!pixels && !rgb8))
        return set_error(CERES_EINVAL, "ceres_render_multi_f32: bad argument");
    for (uint32_t r = 0; r < world; ++r) {
        if (!scenes[r]) return set_error(CERES_EINVAL, "ceres_render_multi_f32: null scene %u", r);
        for (uint32_t q = 0; q < r; ++q)
            if (scenes[q] == scenes[r]) return set_error(CERES_EINVAL, "ceres_render_multi_f32: ranks %u and %u share a scene", q, r);
    }
    const auto t0 = std::chrono::steady_clock::now();
    ceres_scene* s0 = scenes[0];
    const size_t row_bytes = 3 * W;
    const size_t max_rows = local_rows_of(H, row_block, 0, world);       // rank 0 owns the most rows
    const size_t stride = (max_rows * row_bytes + 255) / 256 * 256;
    uint8_t* gbuf = nullptr;
    std::vector<hipEvent_t> done(world, nullptr);
    auto cleanup = [&] {
        for (auto e : done) if (e) (void)hipEventDestroy(e);
        if (gbuf) { (void)hipSetDevice(s0->device); (void)hipFree(gbuf); }
    };
    int rc = CERES_OK;
    if (rgb8) {
        HIP_TRY(hipSetDevice(s0->device));
        if (hipMalloc(&gbuf, stride * world) != hipSuccess) return set_error(CERES_ENOMEM, "ceres_render_multi_f32: gather buffer");
    }
    for (uint32_t r = 0; r < world && !rc; ++r) {
        ceres_scene* s = scenes[r];
        const ceres_tiling t{row_block, r, world};
        const size_t rows = local_rows_of(H, row_block, r, world);
        if (hipSetDevice(s->device) != hipSuccess) { rc = set_error(CERES_EHIP, "hipSetDevice(%d)", s->device); break; }
        // rank 0's buffers also hold the assembled frame: size them for the whole frame up front
        if ((rc = ensure_workspace(s, r == 0 ? W * H : std::max<size_t>(rows, 1) * W, true, true))) break;
        if ((rc = launch(s, 1, basis12, sun, mode, W, H, &t, pixels ? s->d_pixels : nullptr, s->d_rgb8, s->d_counters,
                         s->stream)))
            break;
        if (rgb8 && rows && s->device != s0->device) {
            // direct xGMI access for the copy engine of rank r's device (once per device pair)
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, s->device, s0->device) == hipSuccess && can &&
                hipDeviceEnablePeerAccess(s0->device, 0) != hipSuccess)
                (void)hipGetLastError();          // already enabled: clear the sticky error, copy as usual
        }
        if (rgb8 && rows &&
            hipMemcpyPeerAsync(gbuf + r * stride, s0->device, s->d_rgb8, s->device, rows * row_bytes, s->stream) != hipSuccess) {
            rc = set_error(CERES_EHIP, "ceres_render_multi_f32: peer copy from rank %u", r);
            break;
        }
        if (hipEventCreateWithFlags(&done[r], hipEventDisableTiming) != hipSuccess || hipEventRecord(done[r], s->stream) != hipSuccess)
            rc = set_error(CERES_EHIP, "ceres_render_multi_f32: event");
    }
    if (!rc && rgb8) {
        (void)hipSetDevice(s0->device);
        for (uint32_t r = 0; r < world && !rc; ++r)
            if (hipStreamWaitEvent(s0->stream, done[r], 0) != hipSuccess) rc = set_error(CERES_EHIP, "stream wait");
        // rank 0's rows were copied out of s0->d_rgb8 earlier on this stream: reuse it as the output
        if (!rc) rc = ceres_assemble_rgb8(gbuf, stride, s0->d_rgb8, 1, W, H, row_block, world, s0->stream);
        if (!rc && hipMemcpyAsync(rgb8, s0->d_rgb8, W * H * 3, hipMemcpyDeviceToHost, s0->stream) != hipSuccess)
            rc = set_error(CERES_EHIP, "ceres_render_multi_f32: copy back");
    }
    uint64_t sum[8] = {0};
    std::vector<float> local;
    for (uint32_t r = 0; r < world && !rc; ++r) {
        ceres_scene* s = scenes[r];
        const size_t rows = local_rows_of(H, row_block, r, world);
        uint64_t c[8] = {0};
        (void)hipSetDevice(s->device);
        if (hipMemcpyAsync(c, s->d_counters, sizeof c, hipMemcpyDeviceToHost, s->stream) != hipSuccess) {
            rc = set_error(CERES_EHIP, "ceres_render_multi_f32: counters");
            break;
        }
        if (pixels && rows) {
            local.resize(rows * W * 3);
            if (hipMemcpyAsync(local.data(), s->d_pixels, local.size() * sizeof(float), hipMemcpyDeviceToHost, s->stream) != hipSuccess) {
                rc = set_error(CERES_EHIP, "ceres_render_multi_f32: pixels");
                break;
            }
        }
        if (hipStreamSynchronize(s->stream) != hipSuccess) { rc = set_error(CERES_EHIP, "ceres_render_multi_f32: sync"); break; }
        for (int k = 0; k < 6; ++k) sum[k] += c[k];
        sum[6] |= c[6];
        if (pixels)
            for (size_t k = 0; k < rows; ++k) {                           // local row k -> global row j
                const size_t j = ((k / row_block) * world + r) * row_block + k % row_block;
                std::memcpy(pixels + j * W * 3, local.data() + k * W * 3, W * 3 * sizeof(float));
            }
    }
    if (!rc && rgb8) {
        (void)hipSetDevice(s0->device);
        if (hipStreamSynchronize(s0->stream) != hipSuccess) rc = set_error(CERES_EHIP, "ceres_render_multi_f32: sync");
    }
    cleanup();
    if (rc) return rc;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fill_stats(stats, sum, ms);
    if (sum[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
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
    int rc = launch(s, 1, basis12, sun, mode, W, H, nullptr, nullptr, nullptr, s->d_counters, s->stream, dp, dt, ds);
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
    fill_stats(stats, c, 0.0);
    if (c[6]) return set_error(CERES_ESTACK, "traversal stack overflow");
    return CERES_OK;
}

int ceres_scene_wave_log(ceres_scene* s, uint64_t* out, size_t max_waves, size_t* n_waves) {
    if (!s || !out || !n_waves) return set_error(CERES_EINVAL, "ceres_scene_wave_log: null argument");
    if (!s->d_wave_log) return set_error(CERES_EINVAL, "wave log needs a CERES_SCENE_STATS scene and a full-mode render");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    const size_t n = std::min(max_waves, s->last_grid_waves);
    HIP_TRY(hipMemcpy(out, s->d_wave_log, n * 64, hipMemcpyDeviceToHost));
    *n_waves = n;
    return CERES_OK;
}

int ceres_fetch_counters(int device, uint64_t out[8], int reset) {
    if (!out) return set_error(CERES_EINVAL, "ceres_fetch_counters: null argument");
#if CERES_COUNTING
    static_assert(dev::kFKinds == 8, "ceres_fetch_counters reports 8 kinds");
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long h[dev::kFetchShards][dev::kFKinds];
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(dev::g_fetch), sizeof h));
    for (int k = 0; k < dev::kFKinds; ++k) {
        out[k] = 0;
        for (int q = 0; q < dev::kFetchShards; ++q) out[k] += h[q][k];
    }
    if (reset) {
        std::memset(h, 0, sizeof h);
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(dev::g_fetch), h, sizeof h));
    }
    return CERES_OK;
#else
    (void)device; (void)reset;
    std::memset(out, 0, 8 * sizeof(uint64_t));
    return set_error(CERES_EUNSUPPORTED, "ceres_fetch_counters: only the counting build (make count) tallies fetches");
#endif
}

// Per-launch device timing: while enabled, every render records HIP events around its one
// kernel launch (ceres_fused or ceres_primary) on the launch stream.
int ceres_scene_set_timing(ceres_scene* s, int enable) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    s->timing = enable != 0;
    return CERES_OK;
}

// Synchronises, sums the recorded kernel durations (ms) and recycles the events.  Every render
// is one kernel, so the whole duration is reported as kernel_ms (shadow_ms: always 0, kept for
// the ABI of the former two-kernel path).
int ceres_scene_read_timing(ceres_scene* s, double* kernel_ms, double* shadow_ms, uint64_t* renders) {
    if (!s) return set_error(CERES_EINVAL, "null scene");
    HIP_TRY(hipSetDevice(s->device));
    double p = 0;
    const size_t n = s->ev_used.size() / 2;
    for (size_t k = 0; k < n; ++k) {
        hipEvent_t e0 = s->ev_used[2 * k], e1 = s->ev_used[2 * k + 1];
        HIP_TRY(hipEventSynchronize(e1));
        float a = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, e0, e1));
        p += a;
    }
    for (auto e : s->ev_used) s->ev_pool.push_back(e);
    s->ev_used.clear();
    if (kernel_ms) *kernel_ms = p;
    if (shadow_ms) *shadow_ms = 0.0;
    if (renders) *renders = n;
    return CERES_OK;
}

}  // extern "C"
