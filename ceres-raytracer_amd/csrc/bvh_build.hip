// bvh_build.hip -- the reference's binned-SAH BVH build on gfx950.
//
// Rebuilds BinnedSahBuilder<Bvh,16>::build (binned_sah_builder.hpp:39-234, driven by
// top_down_builder.hpp:43-72) on the GPU with the SAME topology and leaf order as the host
// (reference) build: same bins, same SAH sweeps, same axis choice and fallbacks, same
// std::partition permutation.  Only node NUMBERING differs (the reference's own numbering
// depends on OpenMP task timing); numbering is deterministic here: breadth-first for the
// large nodes, then every small subtree contiguously.
//
// Two regimes:
//   * large items (> kSmall primitives): level-synchronous over all large items of a level,
//     one thread per primitive position.  Bin boxes are reduced with 64-bit keyed atomics
//     (LDS per workgroup, then L2): key = (order-preserving float bits, position), so the
//     reduction is order-independent yet returns exactly what the reference's sequential
//     std::min/std::max loop returns, down to the sign of a zero (the FIRST of equal values in
//     primitive_indices order wins, bounding_box.hpp:23-27 + std::min/max semantics).
//     std::partition (libstdc++ two-pointer swap) is reproduced with a prefix sum: the k-th
//     misplaced "false" from the left swaps with the k-th misplaced "true" from the right.
//   * small items (<= kSmall): one wavefront builds the whole subtree in LDS, binning in the
//     reference's sequential order (lane = axis x bin), partition via __ballot prefix counts.
//
// Compiled with -ffp-contract=off; the only fma in the exact flavour is the reference's
// fast_multiply_add in the bin index (binned_sah_builder.hpp:144-147, a true fmaf under -mfma);
// the CERES_ARITH_FMA flavour adds the SAH-cost contractions of the reference's CMake build.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"
#include "dev_scan.hpp"

#pragma clang fp contract(off)

namespace ceres {
namespace bvhdev {

using namespace devscan;

constexpr int kBins = 16;
constexpr uint32_t kMaxDepth = 64;       // top_down_builder.hpp:36
constexpr uint32_t kMaxLeaf = 16;        // top_down_builder.hpp:41
#ifndef CERES_BVH_SMALL
#define CERES_BVH_SMALL 256
#endif
constexpr uint32_t kSmall = CERES_BVH_SMALL;  // subtree-per-wavefront threshold (primitives)
constexpr int kChunk = 4096;             // positions per binning workgroup (256 threads x 16)
constexpr int kStack = 72;               // small-subtree work stack (depth <= 64 -> <= 66 entries)

// One primitive in position order: centre (the bin key), box, original index.  48 B, moved
// together with the index by the partition so binning reads are coalesced.
struct alignas(16) PrimRec {
    float cx, cy, cz; uint32_t idx;
    float lx, ly, lz, pad0;
    float hx, hy, hz, pad1;
};
static_assert(sizeof(PrimRec) == 48, "PrimRec");

struct BinKeys {                         // keyed bin (large items), 56 B
    unsigned long long lo[3], hi[3];
    uint32_t count, pad;
};

struct Item {                            // one large work item (top_down_builder.hpp:13-24)
    uint32_t node, begin, end, depth;
    float c2b[3], off[3];                // center_to_bin, bin_offset (binned_sah_builder.hpp:144-145)
    uint32_t state;                      // 0 leaf, 1 split candidate, 2 split
    uint32_t axis, split, sah_split;     // final axis, split index, best_splits[axis].second
    uint32_t T, M;                       // #true (left size), #misplaced pairs
    uint32_t next_left, next_right;      // next-level item index of each child, or ~0u (small/leaf)
    uint32_t child;                      // first child node index
};

struct SmallItem { uint32_t node, begin, end, depth; };

struct Counters {                        // host-visible per-level totals
    uint32_t n_items;                    // large items of the next level
    uint32_t n_small;                    // small items so far
    uint32_t n_nodes;                    // top-level nodes so far
    uint32_t pad;
};

// ---- keyed min/max: total order on (float value with -0 == +0, position) --------------------
__device__ __forceinline__ uint32_t ord_bits(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ unsigned long long key_min(float f, uint32_t pos) {
    return (static_cast<unsigned long long>(ord_bits(f)) << 32) | (pos << 1) | (__float_as_uint(f) >> 31);
}
__device__ __forceinline__ unsigned long long key_max(float f, uint32_t pos) {
    return (static_cast<unsigned long long>(ord_bits(f)) << 32) | ((0x7fffffffu - pos) << 1) | (__float_as_uint(f) >> 31);
}
__device__ __forceinline__ float key_value(unsigned long long k) {
    const uint32_t o = uint32_t(k >> 32);
    uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    if (u == 0u && (k & 1ull)) u = 0x80000000u;                    // a -0 that won its tie
    return __uint_as_float(u);
}
constexpr unsigned long long kKeyMinEmpty = (static_cast<unsigned long long>(0xff7fffffu) << 32) | 0xffffffffull;  // FLT_MAX
constexpr unsigned long long kKeyMaxEmpty = (static_cast<unsigned long long>(0x00800000u) << 32);                  // -FLT_MAX

// std::min(a, b) / std::max(a, b) exactly (keep the current value on ties)
__device__ __forceinline__ float lesser(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float greater(float a, float b) { return (a < b) ? b : a; }

// compute_bin_index, binned_sah_builder.hpp:146-149: min(15, size_t(max(0, fmaf(c, c2b, off)))),
// with x86-64's float -> size_t conversion (the reference build is -mavx2, no AVX-512: values
// >= 2^64, infinity included, convert to 0).
__device__ __forceinline__ uint32_t bin_of(float c, float c2b, float off) {
    float f = fmaf(c, c2b, off);
    f = (0.0f < f) ? f : 0.0f;
    if (f >= 18446744073709551616.0f) return 0u;
    if (f >= 15.0f) return kBins - 1;
    return uint32_t(f);
}

__device__ __forceinline__ float half_area(const float lo[3], const float hi[3]) {   // bounding_box.hpp:43-46
    const float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
    return (d0 + d1) * d2 + d0 * d1;
}
// The reference CMake build (g++ -O3 -mfma, CERES_ARITH_FMA: G = true) contracts half_area's FIRST
// product in find_split's sweeps (binned_sah_builder.hpp:98,109), its SECOND in the node's
// max_split_cost (:179), and the sweep cost into fma(count, half_area, right_cost)
// (oracle/contraction_sites.txt)
template <bool G> __device__ __forceinline__ float half_area_sweep(const float lo[3], const float hi[3]) {
    const float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
    return G ? fmaf(d0 + d1, d2, d0 * d1) : (d0 + d1) * d2 + d0 * d1;
}
template <bool G> __device__ __forceinline__ float half_area_node(const float lo[3], const float hi[3]) {
    const float d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
    return G ? fmaf(d0, d1, (d0 + d1) * d2) : (d0 + d1) * d2 + d0 * d1;
}
template <bool G> __device__ __forceinline__ float sweep_cost(float ha, uint32_t cnt, float right) {
    return G ? fmaf(float(cnt), ha, right) : ha * float(cnt) + right;
}

struct BinF { float lo[3], hi[3]; uint32_t count; uint32_t pad; };

// The split decision of BinnedSahBuildTask::build for one node (binned_sah_builder.hpp:86-114,
// 166-196): SAH sweeps per axis, axis choice, leaf test, 0.4-quantile fallback.  `nb` is the
// node box in RefNode order.  Returns false for "make a leaf now".
template <bool G>
__device__ bool sah_decide(const BinF* bins, uint32_t m, const float nb[6], uint32_t& axis_out,
                           uint32_t& split_out, uint32_t& sah_split_out) {
    float best_cost[3];
    uint32_t best_split[3];
    for (int a = 0; a < 3; ++a) {
        const BinF* row = bins + a * kBins;
        float right[kBins];
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        uint32_t cnt = 0;
        for (int i = kBins - 1; i > 0; --i) {
            for (int k = 0; k < 3; ++k) { lo[k] = lesser(lo[k], row[i].lo[k]); hi[k] = greater(hi[k], row[i].hi[k]); }
            cnt += row[i].count;
            right[i] = half_area_sweep<G>(lo, hi) * float(cnt);
        }
        for (int k = 0; k < 3; ++k) { lo[k] = FLT_MAX; hi[k] = -FLT_MAX; }
        cnt = 0;
        best_cost[a] = FLT_MAX;
        best_split[a] = kBins;
        for (int i = 0; i < kBins - 1; ++i) {
            for (int k = 0; k < 3; ++k) { lo[k] = lesser(lo[k], row[i].lo[k]); hi[k] = greater(hi[k], row[i].hi[k]); }
            cnt += row[i].count;
            const float cost = sweep_cost<G>(half_area_sweep<G>(lo, hi), cnt, right[i + 1]);
            if (cost < best_cost[a]) { best_cost[a] = cost; best_split[a] = uint32_t(i + 1); }
        }
    }
    uint32_t axis = 0;
    if (best_cost[0] > best_cost[1]) axis = 1;
    if (best_cost[axis] > best_cost[2]) axis = 2;
    uint32_t split = best_split[axis];
    const float nlo[3] = {nb[0], nb[2], nb[4]}, nhi[3] = {nb[1], nb[3], nb[5]};
    const float leaf_cost = half_area_node<G>(nlo, nhi) * (float(m) - 1.0f);      // traversal_cost = 1
    if (best_split[axis] == kBins || best_cost[axis] >= leaf_cost) {
        if (m <= kMaxLeaf) return false;
        const float d0 = nhi[0] - nlo[0], d1 = nhi[1] - nlo[1], d2 = nhi[2] - nlo[2];   // largest_axis
        const float d[3] = {d0, d1, d2};
        axis = 0;
        if (d[0] < d[1]) axis = 1;
        if (d[axis] < d[2]) axis = 2;
        uint32_t cnt = 0;
        for (int i = 0; i < kBins - 1; ++i) {
            cnt += bins[axis * kBins + i].count;
            if (cnt >= (m * 2u / 5u + 1u)) { split = uint32_t(i + 1); break; }
        }
    }
    axis_out = axis;
    split_out = split;
    sah_split_out = best_split[axis];
    return true;
}

// Child boxes (binned_sah_builder.hpp:216-224), including the reference's use of
// best_splits[axis].second (not the fallback split) as the end of the LEFT range.
__device__ void child_boxes(const BinF* bins, uint32_t axis, uint32_t split, uint32_t sah_split, float lb[6], float rb[6]) {
    float llo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    float rlo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, rhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    const BinF* row = bins + axis * kBins;
    for (uint32_t i = 0; i < sah_split; ++i)
        for (int k = 0; k < 3; ++k) { llo[k] = lesser(llo[k], row[i].lo[k]); lhi[k] = greater(lhi[k], row[i].hi[k]); }
    for (uint32_t i = split; i < uint32_t(kBins); ++i)
        for (int k = 0; k < 3; ++k) { rlo[k] = lesser(rlo[k], row[i].lo[k]); rhi[k] = greater(rhi[k], row[i].hi[k]); }
    for (int k = 0; k < 3; ++k) { lb[2 * k] = llo[k]; lb[2 * k + 1] = lhi[k]; rb[2 * k] = rlo[k]; rb[2 * k + 1] = rhi[k]; }
}

__device__ __forceinline__ float comp3(float x, float y, float z, uint32_t a) { return a == 0 ? x : (a == 1 ? y : z); }
__device__ __forceinline__ uint32_t sel3(uint32_t x, uint32_t y, uint32_t z, uint32_t a) { return a == 0 ? x : (a == 1 ? y : z); }

// ---- init: per-primitive box + centre (triangle.hpp:39-48), root box ---------------------
// Box: p0 extended by p1() = p0 - e1 then p2() = p0 + e2; centre (p0 + p1 + p2) * (1/3).
constexpr int kInitPer = 8;              // primitives per thread in k_init
__global__ void __launch_bounds__(256) k_init(const Tri48* __restrict__ tris, uint32_t n, PrimRec* __restrict__ rec,
                                              int32_t* __restrict__ seg, int32_t seg0,
                                              unsigned long long* __restrict__ root_keys) {
    __shared__ unsigned long long red[6][256];
    unsigned long long k[6] = {kKeyMinEmpty, kKeyMinEmpty, kKeyMinEmpty, kKeyMaxEmpty, kKeyMaxEmpty, kKeyMaxEmpty};
    for (int r = 0; r < kInitPer; ++r) {
        const uint32_t i = (blockIdx.x * kInitPer + uint32_t(r)) * 256u + threadIdx.x;
        if (i >= n) break;
        const Tri48 t = tris[i];
        const float p0[3] = {t.p0[0], t.p0[1], t.p0[2]};
        float p1[3], p2[3], lo[3], hi[3], c[3];
        for (int a = 0; a < 3; ++a) {
            p1[a] = p0[a] - t.e1[a];
            p2[a] = p0[a] + t.e2[a];
            lo[a] = lesser(lesser(p0[a], p1[a]), p2[a]);
            hi[a] = greater(greater(p0[a], p1[a]), p2[a]);
            c[a] = (p0[a] + p1[a] + p2[a]) * (1.0f / 3.0f);
        }
        PrimRec pr;
        pr.cx = c[0]; pr.cy = c[1]; pr.cz = c[2]; pr.idx = i;
        pr.lx = lo[0]; pr.ly = lo[1]; pr.lz = lo[2]; pr.pad0 = 0.f;
        pr.hx = hi[0]; pr.hy = hi[1]; pr.hz = hi[2]; pr.pad1 = 0.f;
        rec[i] = pr;
        seg[i] = seg0;
        for (int a = 0; a < 3; ++a) { k[a] = min(k[a], key_min(lo[a], i)); k[3 + a] = max(k[3 + a], key_max(hi[a], i)); }
    }
    for (int v = 0; v < 6; ++v) red[v][threadIdx.x] = k[v];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < unsigned(s))
            for (int v = 0; v < 6; ++v) {
                const unsigned long long o = red[v][threadIdx.x + s];
                red[v][threadIdx.x] = v < 3 ? min(red[v][threadIdx.x], o) : max(red[v][threadIdx.x], o);
            }
        __syncthreads();
    }
    if (threadIdx.x < 3) atomicMin(&root_keys[threadIdx.x], red[threadIdx.x][0]);
    else if (threadIdx.x < 6) atomicMax(&root_keys[threadIdx.x], red[threadIdx.x][0]);
}

__global__ void k_root(RefNode* nodes, const unsigned long long* root_keys, uint32_t n, Item* items, SmallItem* small,
                       Counters* ctr) {
    if (threadIdx.x != 0) return;
    RefNode r;
    for (int a = 0; a < 3; ++a) { r.bounds[2 * a] = key_value(root_keys[a]); r.bounds[2 * a + 1] = key_value(root_keys[3 + a]); }
    r.primitive_count = 0; r.first_child_or_primitive = 0;
    nodes[0] = r;
    if (n > kSmall) {
        Item it{};
        it.node = 0; it.begin = 0; it.end = n; it.depth = 0;
        items[0] = it;
        ctr->n_items = 1; ctr->n_small = 0;
    } else {
        small[0] = SmallItem{0, 0, n, 0};
        ctr->n_items = 0; ctr->n_small = 1;
    }
    ctr->n_nodes = 1;
}

// ---- large items: one level ------------------------------------------------------------
// per item: bin parameters from the node box, bins cleared
__global__ void k_item_prep(Item* items, uint32_t n_items, const RefNode* nodes, BinKeys* bins) {
    const uint32_t s = blockIdx.x;
    if (s >= n_items) return;
    if (threadIdx.x < 3u * kBins) {
        BinKeys& b = bins[size_t(s) * 3 * kBins + threadIdx.x];
        for (int k = 0; k < 3; ++k) { b.lo[k] = kKeyMinEmpty; b.hi[k] = kKeyMaxEmpty; }
        b.count = 0; b.pad = 0;
    }
    if (threadIdx.x == 0) {
        Item& it = items[s];
        const RefNode& nd = nodes[it.node];
        for (int a = 0; a < 3; ++a) {
            const float lo = nd.bounds[2 * a], hi = nd.bounds[2 * a + 1];
            const float c2b = (1.0f / (hi - lo)) * float(kBins);           // diagonal().inverse() * bin_count
            it.c2b[a] = c2b;
            it.off[a] = (-lo) * c2b;                                       // -bbox.min * center_to_bin
        }
        it.state = 0;
    }
}

// Fill the bins of every large item (binned_sah_builder.hpp:157-164).  A wavefront whose active
// positions all belong to one item reduces each (axis, bin) group of lanes with butterfly
// reductions of the keys (one LDS / L2 atomic per group instead of one per lane); the
// workgroup's first item reduces in LDS, others go straight to L2.  Mixed wavefronts (item
// boundaries) fall back to per-lane atomics.  Keys make every order give the same bins.
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const uint32_t lo = uint32_t(__shfl_xor(int(uint32_t(v)), m));
    const uint32_t hi = uint32_t(__shfl_xor(int(uint32_t(v >> 32)), m));
    return (static_cast<unsigned long long>(hi) << 32) | lo;
}

// Lane (axis, bin) of each wavefront walks the wavefront's positions in order and keeps its
// bin's running box exactly like the reference's sequential loop (ties keep the earlier value),
// remembering which position supplied each bound; the partial bin is flushed as keys when the
// item changes (LDS for the workgroup's first item, else L2).  Reads are LDS broadcasts of
// staged 64-record runs; no atomics conflict inside a wavefront.
__global__ void __launch_bounds__(256) k_bin(const PrimRec* __restrict__ rec, const int32_t* __restrict__ seg, uint32_t n,
                                             const Item* __restrict__ items, BinKeys* __restrict__ bins) {
    __shared__ unsigned long long slo[3 * kBins][3], shi[3 * kBins][3];
    __shared__ uint32_t scount[3 * kBins];
    __shared__ PrimRec stage[4][64];
    __shared__ int32_t sseg[4][64];
    __shared__ int32_t s0_sh;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t blk = blockIdx.x * uint32_t(kChunk);
    const uint32_t base = blk + wave * uint32_t(kChunk / 4);
    const uint32_t my_axis = lane >> 4, my_bin = lane & 15u;
    const bool binlane = lane < 3u * kBins;
    if (threadIdx.x < 3u * kBins) {
        for (int k = 0; k < 3; ++k) { slo[threadIdx.x][k] = kKeyMinEmpty; shi[threadIdx.x][k] = kKeyMaxEmpty; }
        scount[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) s0_sh = blk < n ? seg[blk] : -1;
    __syncthreads();
    const int32_t s0 = s0_sh;
    int32_t cur = -1;
    float mc2b = 0.f, moff = 0.f;
    float lo[3], hi[3];
    uint32_t plo[3], phi[3], cnt = 0;
    auto reset = [&]() {
        for (int k = 0; k < 3; ++k) { lo[k] = FLT_MAX; hi[k] = -FLT_MAX; plo[k] = 0x7fffffffu; phi[k] = 0x7fffffffu; }
        cnt = 0;
    };
    auto flush = [&]() {
        if (cur < 0 || !binlane || cnt == 0) return;
        const uint32_t idx = lane;
        if (cur == s0) {
            atomicAdd(&scount[idx], cnt);
            for (int k = 0; k < 3; ++k) { atomicMin(&slo[idx][k], key_min(lo[k], plo[k])); atomicMax(&shi[idx][k], key_max(hi[k], phi[k])); }
        } else {
            BinKeys& g = bins[size_t(cur) * 3 * kBins + idx];
            atomicAdd(&g.count, cnt);
            for (int k = 0; k < 3; ++k) { atomicMin(&g.lo[k], key_min(lo[k], plo[k])); atomicMax(&g.hi[k], key_max(hi[k], phi[k])); }
        }
    };
    reset();
    for (int r = 0; r < kChunk / 4 / 64; ++r) {
        const uint32_t p0 = base + uint32_t(r) * 64u;
        if (p0 + lane < n) { stage[wave][lane] = rec[p0 + lane]; sseg[wave][lane] = seg[p0 + lane]; }
        else sseg[wave][lane] = -1;
        __syncthreads();
        const int32_t s_run = sseg[wave][0];
        if (__ballot(sseg[wave][lane] == s_run) == ~0ull) {            // one item (or none) in this run
            if (s_run != cur) {
                flush();
                reset();
                cur = s_run;
                if (s_run >= 0) {
                    const Item& it = items[s_run];
                    mc2b = comp3(it.c2b[0], it.c2b[1], it.c2b[2], my_axis);
                    moff = comp3(it.off[0], it.off[1], it.off[2], my_axis);
                }
            }
            if (s_run >= 0 && binlane) {
#pragma unroll 4
                for (uint32_t j = 0; j < 64; ++j) {
                    const PrimRec& pr = stage[wave][j];
                    if (bin_of(comp3(pr.cx, pr.cy, pr.cz, my_axis), mc2b, moff) == my_bin) {
                        const uint32_t p = p0 + j;
                        ++cnt;
                        const float vl[3] = {pr.lx, pr.ly, pr.lz}, vh[3] = {pr.hx, pr.hy, pr.hz};
                        for (int k = 0; k < 3; ++k) {
                            if (vl[k] < lo[k]) { lo[k] = vl[k]; plo[k] = p; }
                            if (hi[k] < vh[k]) { hi[k] = vh[k]; phi[k] = p; }
                        }
                    }
                }
            }
            __syncthreads();
            continue;
        }
        for (uint32_t j = 0; j < 64; ++j) {
            const int32_t sj = sseg[wave][j];
            if (sj != cur) {
                flush();
                reset();
                cur = sj;
                if (sj >= 0) {
                    const Item& it = items[sj];
                    mc2b = comp3(it.c2b[0], it.c2b[1], it.c2b[2], my_axis);
                    moff = comp3(it.off[0], it.off[1], it.off[2], my_axis);
                }
            }
            if (sj < 0) continue;
            const PrimRec& pr = stage[wave][j];
            const float c = comp3(pr.cx, pr.cy, pr.cz, my_axis);
            if (binlane && bin_of(c, mc2b, moff) == my_bin) {
                const uint32_t p = p0 + j;
                ++cnt;
                const float vl[3] = {pr.lx, pr.ly, pr.lz}, vh[3] = {pr.hx, pr.hy, pr.hz};
                for (int k = 0; k < 3; ++k) {
                    if (vl[k] < lo[k]) { lo[k] = vl[k]; plo[k] = p; }
                    if (hi[k] < vh[k]) { hi[k] = vh[k]; phi[k] = p; }
                }
            }
        }
        __syncthreads();
    }
    flush();
    __syncthreads();
    if (s0 >= 0 && threadIdx.x < 3u * kBins && scount[threadIdx.x]) {
        BinKeys& g = bins[size_t(s0) * 3 * kBins + threadIdx.x];
        atomicAdd(&g.count, scount[threadIdx.x]);
        for (int k = 0; k < 3; ++k) { atomicMin(&g.lo[k], slo[threadIdx.x][k]); atomicMax(&g.hi[k], shi[threadIdx.x][k]); }
    }
}

__device__ void decode_bins(const BinKeys* g, BinF* out) {
    for (int b = 0; b < 3 * kBins; ++b) {
        for (int k = 0; k < 3; ++k) { out[b].lo[k] = key_value(g[b].lo[k]); out[b].hi[k] = key_value(g[b].hi[k]); }
        out[b].count = g[b].count;
    }
}

// Split decision per large item (one thread each); leaves are final here.
template <bool G>
__global__ void __launch_bounds__(64) k_split(Item* items, uint32_t n_items, RefNode* nodes, const BinKeys* bins) {
    const uint32_t s = blockIdx.x * 64u + threadIdx.x;
    if (s >= n_items) return;
    Item& it = items[s];
    const uint32_t m = it.end - it.begin;
    RefNode& nd = nodes[it.node];
    if (m <= 1 || it.depth >= kMaxDepth) {
        nd.primitive_count = m; nd.first_child_or_primitive = it.begin;
        it.state = 0;
        return;
    }
    BinF b[3 * kBins];
    decode_bins(bins + size_t(s) * 3 * kBins, b);
    float nb[6];
    for (int k = 0; k < 6; ++k) nb[k] = nd.bounds[k];
    uint32_t axis, split, sah;
    if (!sah_decide<G>(b, m, nb, axis, split, sah)) {
        nd.primitive_count = m; nd.first_child_or_primitive = it.begin;
        it.state = 0;
        return;
    }
    it.axis = axis; it.split = split; it.sah_split = sah;
    it.state = 1;
}

// partition predicate per position of split candidates (binned_sah_builder.hpp:199-201)
__global__ void __launch_bounds__(256) k_flags(const PrimRec* __restrict__ rec, const int32_t* __restrict__ seg, uint32_t n,
                                               const Item* __restrict__ items, uint32_t* __restrict__ flag) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    uint32_t f = 0;
    const int32_t s = seg[p];
    if (s >= 0) {
        const Item& it = items[s];
        if (it.state == 1) {
            const PrimRec& pr = rec[p];
            const float c = comp3(pr.cx, pr.cy, pr.cz, it.axis);
            f = bin_of(c, it.c2b[it.axis], it.off[it.axis]) < it.split ? 1u : 0u;
        }
    }
    flag[p] = f;
}

// ---- per-level plan (one workgroup): finalize splits, allocate child nodes and items ------
__global__ void __launch_bounds__(256) k_plan(Item* items, uint32_t n_items, const uint32_t* __restrict__ X, RefNode* nodes,
                                              Counters* ctr, SmallItem* small) {
    __shared__ uint32_t sh[264];
    __shared__ uint32_t carry_nodes, carry_large, carry_small;
    if (threadIdx.x == 0) { carry_nodes = ctr->n_nodes; carry_large = 0; carry_small = ctr->n_small; }
    __syncthreads();
    for (uint32_t base = 0; base < n_items; base += 256) {
        const uint32_t s = base + threadIdx.x;
        uint32_t split = 0, nlarge = 0, nsmall = 0;
        Item it{};
        if (s < n_items) {
            it = items[s];
            if (it.state == 1) {
                const uint32_t m = it.end - it.begin;
                const uint32_t T = X[it.end] - X[it.begin];
                if (T == 0 || T == m) {                             // one side empty: leaf (:204, :230)
                    nodes[it.node].primitive_count = m;
                    nodes[it.node].first_child_or_primitive = it.begin;
                    it.state = 0;
                } else {
                    it.state = 2;
                    it.T = T;
                    it.M = T - (X[it.begin + T] - X[it.begin]);         // falses left of the split point
                    split = 1;
                    nlarge = (T > kSmall) + (m - T > kSmall);
                    nsmall = 2 - nlarge;
                }
            }
        }
        uint32_t tot;
        const uint32_t ex_split = block_exclusive_scan_256(split, sh, tot);
        const uint32_t tot_split = tot;
        const uint32_t ex_large = block_exclusive_scan_256(nlarge, sh, tot);
        const uint32_t tot_large = tot;
        const uint32_t ex_small = block_exclusive_scan_256(nsmall, sh, tot);
        const uint32_t tot_small = tot;
        if (s < n_items) {
            if (it.state == 2) {
                it.child = carry_nodes + 2 * ex_split;
                const uint32_t m = it.end - it.begin;
                uint32_t lb = carry_large + ex_large, sb = carry_small + ex_small;
                const bool left_large = it.T > kSmall, right_large = m - it.T > kSmall;
                it.next_left = left_large ? lb++ : ~0u;
                it.next_right = right_large ? lb++ : ~0u;
                if (!left_large) small[sb++] = SmallItem{it.child, it.begin, it.begin + it.T, it.depth + 1};
                if (!right_large) small[sb++] = SmallItem{it.child + 1, it.begin + it.T, it.end, it.depth + 1};
            } else {
                it.next_left = it.next_right = ~0u;
            }
            items[s] = it;
        }
        __syncthreads();
        if (threadIdx.x == 0) { carry_nodes += 2 * tot_split; carry_large += tot_large; carry_small += tot_small; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { ctr->n_nodes = carry_nodes; ctr->n_items = carry_large; ctr->n_small = carry_small; }
}

// parent link, child boxes, next-level items (one thread per split item)
__global__ void __launch_bounds__(64) k_emit(const Item* items, uint32_t n_items, RefNode* nodes, const BinKeys* bins,
                                             Item* next) {
    const uint32_t s = blockIdx.x * 64u + threadIdx.x;
    if (s >= n_items) return;
    const Item it = items[s];
    if (it.state != 2) return;
    BinF b[3 * kBins];
    decode_bins(bins + size_t(s) * 3 * kBins, b);
    float lb[6], rb[6];
    child_boxes(b, it.axis, it.split, it.sah_split, lb, rb);
    RefNode& nd = nodes[it.node];
    nd.primitive_count = 0;
    nd.first_child_or_primitive = it.child;
    RefNode l, r;
    for (int k = 0; k < 6; ++k) { l.bounds[k] = lb[k]; r.bounds[k] = rb[k]; }
    l.primitive_count = r.primitive_count = 0;
    l.first_child_or_primitive = r.first_child_or_primitive = 0;
    nodes[it.child] = l;
    nodes[it.child + 1] = r;
    if (it.next_left != ~0u) { Item c{}; c.node = it.child; c.begin = it.begin; c.end = it.begin + it.T; c.depth = it.depth + 1; next[it.next_left] = c; }
    if (it.next_right != ~0u) { Item c{}; c.node = it.child + 1; c.begin = it.begin + it.T; c.end = it.end; c.depth = it.depth + 1; next[it.next_right] = c; }
}

// misplaced elements of each split item: the k-th "false" left of the split point and the
// k-th "true" right of it (counted from the end) are swapped by std::partition.
__global__ void __launch_bounds__(256) k_pos(const int32_t* __restrict__ seg, uint32_t n, const Item* __restrict__ items,
                                             const uint32_t* __restrict__ flag, const uint32_t* __restrict__ X,
                                             uint32_t* __restrict__ posF, uint32_t* __restrict__ posT) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    const int32_t s = seg[p];
    if (s < 0) return;
    const Item& it = items[s];
    if (it.state != 2) return;
    const uint32_t mid = it.begin + it.T;
    const uint32_t tr = X[p] - X[it.begin];                 // trues in [begin, p)
    if (p < mid) {
        if (!flag[p]) posF[it.begin + (p - it.begin - tr)] = p;
    } else {
        if (flag[p]) posT[it.begin + (it.T - 1 - tr)] = p;
    }
}

__global__ void __launch_bounds__(256) k_swap_seg(PrimRec* __restrict__ rec, int32_t* __restrict__ seg, uint32_t n,
                                                  const Item* __restrict__ items, const uint32_t* __restrict__ posF,
                                                  const uint32_t* __restrict__ posT) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    const int32_t s = seg[p];
    if (s < 0) return;
    const Item& it = items[s];
    if (it.state != 2) { seg[p] = -1; return; }
    const uint32_t k = p - it.begin;
    if (k < it.M) {
        const uint32_t a = posF[it.begin + k], b = posT[it.begin + k];
        const PrimRec ra = rec[a], rb = rec[b];
        rec[a] = rb;
        rec[b] = ra;
    }
    const uint32_t nx = p < it.begin + it.T ? it.next_left : it.next_right;
    seg[p] = nx == ~0u ? -1 : int32_t(nx);
}

// ---- small items: one wavefront builds a whole subtree ----------------------------------
// Nodes of the subtree (except its root, a top-level node) go to tnodes[2 * begin + local];
// inner nodes' first_child is local until k_place rebases them.
struct StackEntry { uint32_t begin, end, depth; int32_t local; float box[6]; };

// 16-lane segmented scans over the bins of one axis (lane = axis * 16 + bin).  The combine keeps
// the EARLIER bin on ties, as the reference's ascending extend loops do (sign of zero exact).
struct LaneBox { float lo[3], hi[3]; uint32_t cnt; };

__device__ __forceinline__ LaneBox prefix16(LaneBox v, uint32_t i) {           // bins 0..i
    for (int d = 1; d < 16; d <<= 1) {
        LaneBox u;
        for (int k = 0; k < 3; ++k) { u.lo[k] = __shfl_up(v.lo[k], d, 16); u.hi[k] = __shfl_up(v.hi[k], d, 16); }
        u.cnt = __shfl_up(v.cnt, d, 16);
        if (i >= uint32_t(d)) {
            for (int k = 0; k < 3; ++k) { v.lo[k] = lesser(u.lo[k], v.lo[k]); v.hi[k] = greater(u.hi[k], v.hi[k]); }
            v.cnt += u.cnt;
        }
    }
    return v;
}
__device__ __forceinline__ LaneBox suffix16(LaneBox v, uint32_t i) {           // bins i..15
    for (int d = 1; d < 16; d <<= 1) {
        LaneBox u;
        for (int k = 0; k < 3; ++k) { u.lo[k] = __shfl_down(v.lo[k], d, 16); u.hi[k] = __shfl_down(v.hi[k], d, 16); }
        u.cnt = __shfl_down(v.cnt, d, 16);
        if (i + uint32_t(d) < 16u) {
            for (int k = 0; k < 3; ++k) { v.lo[k] = lesser(v.lo[k], u.lo[k]); v.hi[k] = greater(v.hi[k], u.hi[k]); }
            v.cnt += u.cnt;
        }
    }
    return v;
}
template <bool G> __device__ __forceinline__ float lane_half_area(const LaneBox& b) { return half_area_sweep<G>(b.lo, b.hi); }

// One wavefront builds the whole subtree of a small item.  Bins: keyed LDS atomics (position =
// order of the reference's sequential loop); SAH sweeps: segmented scans, 16 lanes per axis
// (the costs depend only on box values and counts, so they are bit-identical to the sequential
// sweeps of binned_sah_builder.hpp:89-114); the first minimal cost wins (strict <).
template <bool G>
__global__ void __launch_bounds__(64) k_small(PrimRec* __restrict__ rec, const SmallItem* __restrict__ small, uint32_t n_small,
                                              RefNode* __restrict__ nodes, RefNode* __restrict__ tnodes,
                                              uint32_t* __restrict__ small_count, uint32_t* __restrict__ prim_out) {
    __shared__ PrimRec R[kSmall];
    __shared__ StackEntry st[kStack];
    __shared__ unsigned long long klo[3 * kBins][3], khi[3 * kBins][3];
    __shared__ uint32_t kcnt[3 * kBins];
    __shared__ uint16_t posF[kSmall / 2], posT[kSmall / 2];
    const uint32_t s = blockIdx.x;
    if (s >= n_small) return;
    const uint32_t lane = threadIdx.x;
    const SmallItem si = small[s];
    const uint32_t b0 = si.begin, m0 = si.end - si.begin;
    for (uint32_t k = lane; k < m0; k += 64) R[k] = rec[b0 + k];
    if (lane == 0) {
        StackEntry e;
        e.begin = 0; e.end = m0; e.depth = si.depth; e.local = -1;
        for (int k = 0; k < 6; ++k) e.box[k] = nodes[si.node].bounds[k];
        st[0] = e;
    }
    __syncthreads();
    int sp = 1;
    uint32_t nc = 0;                                         // local nodes allocated
    RefNode* const tbase = tnodes + 2 * size_t(b0);
    const uint32_t my_axis = lane >> 4, bi = lane & 15u;     // lanes 48..63: padding group
    while (sp > 0) {
        const StackEntry e = st[--sp];
        __syncthreads();
        RefNode* const nd = e.local < 0 ? nodes + si.node : tbase + e.local;
        const uint32_t m = e.end - e.begin;
        if (m <= 1 || e.depth >= kMaxDepth) {
            if (lane == 0) { nd->primitive_count = m; nd->first_child_or_primitive = b0 + e.begin; }
            continue;
        }
        float c2b[3], off[3];
        for (int a = 0; a < 3; ++a) {
            const float lo = e.box[2 * a], hi = e.box[2 * a + 1];
            c2b[a] = (1.0f / (hi - lo)) * float(kBins);
            off[a] = (-lo) * c2b[a];
        }
        LaneBox v;
        for (int k = 0; k < 3; ++k) { v.lo[k] = FLT_MAX; v.hi[k] = -FLT_MAX; }
        v.cnt = 0;
        {
            if (lane < 3u * kBins) {
                for (int k = 0; k < 3; ++k) { klo[lane][k] = kKeyMinEmpty; khi[lane][k] = kKeyMaxEmpty; }
                kcnt[lane] = 0;
            }
            __syncthreads();
            for (uint32_t p = e.begin + lane; p < e.end; p += 64) {
                const PrimRec& pr = R[p];
                const float c[3] = {pr.cx, pr.cy, pr.cz}, lo[3] = {pr.lx, pr.ly, pr.lz}, hi[3] = {pr.hx, pr.hy, pr.hz};
                for (int a = 0; a < 3; ++a) {
                    const uint32_t b = uint32_t(a) * kBins + bin_of(c[a], c2b[a], off[a]);
                    atomicAdd(&kcnt[b], 1u);
                    for (int k = 0; k < 3; ++k) { atomicMin(&klo[b][k], key_min(lo[k], p)); atomicMax(&khi[b][k], key_max(hi[k], p)); }
                }
            }
            __syncthreads();
            if (lane < 3u * kBins) {
                for (int k = 0; k < 3; ++k) { v.lo[k] = key_value(klo[lane][k]); v.hi[k] = key_value(khi[lane][k]); }
                v.cnt = kcnt[lane];
            }
        }
        const LaneBox L = prefix16(v, bi), Rs = suffix16(v, bi);
        const float rcost = lane_half_area<G>(Rs) * float(Rs.cnt);
        const float rnext = __shfl_down(rcost, 1, 16);
        const float cost = sweep_cost<G>(lane_half_area<G>(L), L.cnt, rnext);
        // first minimal valid cost of this axis (sequential "if (cost < best)" from FLT_MAX)
        const bool valid = bi < 15u && cost < FLT_MAX;
        float bc = valid ? cost : INFINITY;
        uint32_t bs = valid ? bi + 1u : uint32_t(kBins);
        for (int d = 8; d > 0; d >>= 1) {
            const float oc = __shfl_xor(bc, d, 16);
            const uint32_t os = __shfl_xor(bs, d, 16);
            if (oc < bc || (oc == bc && os < bs)) { bc = oc; bs = os; }
        }
        if (bs == uint32_t(kBins)) bc = FLT_MAX;
        const float bcost[3] = {__shfl(bc, 0), __shfl(bc, 16), __shfl(bc, 32)};
        const uint32_t bsplit[3] = {uint32_t(__shfl(int(bs), 0)), uint32_t(__shfl(int(bs), 16)), uint32_t(__shfl(int(bs), 32))};
        uint32_t axis = 0;
        if (bcost[0] > bcost[1]) axis = 1;
        if (comp3(bcost[0], bcost[1], bcost[2], axis) > bcost[2]) axis = 2;
        uint32_t split = sel3(bsplit[0], bsplit[1], bsplit[2], axis);
        const float nlo[3] = {e.box[0], e.box[2], e.box[4]}, nhi[3] = {e.box[1], e.box[3], e.box[5]};
        const float leaf_cost = half_area_node<G>(nlo, nhi) * (float(m) - 1.0f);
        bool make_leaf = false;
        if (split == uint32_t(kBins) || comp3(bcost[0], bcost[1], bcost[2], axis) >= leaf_cost) {
            if (m <= kMaxLeaf) {
                make_leaf = true;
            } else {
                const float d0 = nhi[0] - nlo[0], d1 = nhi[1] - nlo[1], d2 = nhi[2] - nlo[2];   // largest_axis
                axis = 0;
                if (d0 < d1) axis = 1;
                if (comp3(d0, d1, d2, axis) < d2) axis = 2;
                const unsigned long long hit = __ballot(my_axis == axis && bi < 15u && L.cnt >= (m * 2u / 5u + 1u));
                if (hit) split = uint32_t(__ffsll(hit) - 1) - axis * kBins + 1u;
            }
        }
        if (make_leaf) {
            if (lane == 0) { nd->primitive_count = m; nd->first_child_or_primitive = b0 + e.begin; }
            continue;
        }
        const uint32_t sah = sel3(bsplit[0], bsplit[1], bsplit[2], axis);
        const float ac2b = comp3(c2b[0], c2b[1], c2b[2], axis), aoff = comp3(off[0], off[1], off[2], axis);
        // partition: count, then misplaced positions, then swaps (libstdc++ std::partition)
        uint32_t T = 0;
        for (uint32_t base = e.begin; base < e.end; base += 64) {
            const uint32_t p = base + lane;
            const bool f = p < e.end && bin_of(comp3(R[p].cx, R[p].cy, R[p].cz, axis), ac2b, aoff) < split;
            T += uint32_t(__popcll(__ballot(f)));
        }
        if (T == 0 || T == m) {
            if (lane == 0) { nd->primitive_count = m; nd->first_child_or_primitive = b0 + e.begin; }
            continue;
        }
        const uint32_t mid = e.begin + T;
        uint32_t tr = 0, M = 0;
        for (uint32_t base = e.begin; base < e.end; base += 64) {
            const uint32_t p = base + lane;
            const bool f = p < e.end && bin_of(comp3(R[p].cx, R[p].cy, R[p].cz, axis), ac2b, aoff) < split;
            const unsigned long long mask = __ballot(f);
            const uint32_t trp = tr + uint32_t(__popcll(mask & ((1ull << lane) - 1ull)));   // trues in [begin, p)
            if (p < e.end) {
                if (p < mid && !f) posF[(p - e.begin) - trp] = uint16_t(p);
                else if (p >= mid && f) posT[T - 1 - trp] = uint16_t(p);
            }
            M += uint32_t(__popcll(__ballot(p < mid && p < e.end && !f)));
            tr += uint32_t(__popcll(mask));
        }
        __syncthreads();
        for (uint32_t k = lane; k < M; k += 64) {
            const uint32_t a = posF[k], b = posT[k];
            const PrimRec ra = R[a], rb = R[b];
            R[a] = rb;
            R[b] = ra;
        }
        // child boxes (binned_sah_builder.hpp:216-224): left = bins [0, sah), right = bins [split, 16)
        float lb[6], rb[6];
        const int lsrc = int(axis * kBins + sah - 1u), rsrc = int(axis * kBins + split);
        for (int k = 0; k < 3; ++k) {
            lb[2 * k] = __shfl(L.lo[k], lsrc); lb[2 * k + 1] = __shfl(L.hi[k], lsrc);
            rb[2 * k] = __shfl(Rs.lo[k], rsrc); rb[2 * k + 1] = __shfl(Rs.hi[k], rsrc);
        }
        const uint32_t child = nc;
        nc += 2;
        __syncthreads();
        if (lane == 0) {
            RefNode l, r;
            for (int k = 0; k < 6; ++k) { l.bounds[k] = lb[k]; r.bounds[k] = rb[k]; }
            l.primitive_count = r.primitive_count = 0;
            l.first_child_or_primitive = r.first_child_or_primitive = 0;
            tbase[child] = l;
            tbase[child + 1] = r;
            nd->primitive_count = 0;
            nd->first_child_or_primitive = child;
            StackEntry er, el;
            er.begin = mid; er.end = e.end; er.depth = e.depth + 1; er.local = int32_t(child + 1);
            el.begin = e.begin; el.end = mid; el.depth = e.depth + 1; el.local = int32_t(child);
            for (int k = 0; k < 6; ++k) { er.box[k] = rb[k]; el.box[k] = lb[k]; }
            st[sp] = er;
            st[sp + 1] = el;
        }
        sp += 2;
        __syncthreads();
    }
    for (uint32_t k = lane; k < m0; k += 64) prim_out[b0 + k] = R[k].idx;
    if (lane == 0) small_count[s] = nc;
}

// Final permutation for positions that ended in top-level leaves (k_small overwrites its ranges).
__global__ void __launch_bounds__(256) k_prim_out(const PrimRec* __restrict__ rec, uint32_t n, uint32_t* __restrict__ prim_out) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p < n) prim_out[p] = rec[p].idx;
}

// Move each subtree's nodes after the top-level nodes, rebasing local child links.
__global__ void __launch_bounds__(64) k_place(const SmallItem* __restrict__ small, uint32_t n_small, const uint32_t* __restrict__ base,
                                              const RefNode* __restrict__ tnodes, RefNode* __restrict__ nodes, uint32_t top_nodes) {
    const uint32_t s = blockIdx.x;
    if (s >= n_small) return;
    const SmallItem si = small[s];
    const uint32_t cnt = base[s + 1] - base[s];
    const uint32_t dst = top_nodes + base[s];
    const RefNode* src = tnodes + 2 * size_t(si.begin);
    for (uint32_t k = threadIdx.x; k < cnt; k += 64) {
        RefNode r = src[k];
        if (r.primitive_count == 0) r.first_child_or_primitive += dst;
        nodes[dst + k] = r;
    }
    if (threadIdx.x == 0 && cnt) nodes[si.node].first_child_or_primitive = dst;
}

}  // namespace bvhdev
}  // namespace ceres

// --------------------------------------------------------------------------- host side
using namespace ceres;
using namespace ceres::bvhdev;

namespace {

#define BVH_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) { rc = set_error(CERES_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); goto done; } \
    } while (0)

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

extern "C" {

// Device build: d_tri48 = n_tri bvh::Triangle<float> in device memory; d_nodes32 must hold
// 2 * n_tri - 1 RefNodes, d_prim32 n_tri u32.  Stream-ordered; returns after the build
// (the node count is read back).  Workspace comes from hipMallocAsync on `stream`.
int ceres_bvh_build_device_arith(const float* d_tri48, size_t n_tri, uint32_t* d_nodes32, uint32_t* d_prim32,
                                 size_t* n_nodes, void* stream_, int arith) {
    if (!d_tri48 || !d_nodes32 || !d_prim32 || !n_nodes) return set_error(CERES_EINVAL, "ceres_bvh_build_device: null argument");
    if (arith != CERES_ARITH_EXACT && arith != CERES_ARITH_FMA) return set_error(CERES_EINVAL, "unknown arithmetic %d", arith);
    const bool gfma = arith == CERES_ARITH_FMA;
    if (n_tri == 0) return set_error(CERES_EINVAL, "The given scene is empty or cannot be loaded");
    if (n_tri > 0x7fffffffu) return set_error(CERES_EUNSUPPORTED, "more than 2^31 triangles");
    hipStream_t stream = static_cast<hipStream_t>(stream_);
    const uint32_t n = uint32_t(n_tri);
    RefNode* nodes = reinterpret_cast<RefNode*>(d_nodes32);
    const uint32_t cap_items = n / (kSmall + 1) + 2;
    const uint32_t cap_small = uint32_t(std::min<size_t>(n, size_t(128) * n / kSmall + 4));
    const uint32_t scan_blocks = (n + kScanBlock - 1) / kScanBlock;
    const uint32_t chunks = (n + kChunk - 1) / kChunk;
    // workspace layout
    size_t off = 0;
    auto carve = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes); return o; };
    const size_t o_rec = carve(size_t(n) * sizeof(PrimRec));
    const size_t o_seg = carve(size_t(n) * 4);
    const size_t o_flag = carve(size_t(n) * 4);
    const size_t o_X = carve(size_t(n + 1) * 4);
    const size_t o_part = carve(size_t(std::max(scan_blocks, cap_small) + 1) * 4);
    const size_t o_posF = carve(size_t(n) * 4);
    const size_t o_posT = carve(size_t(n) * 4);
    const size_t o_items0 = carve(size_t(cap_items) * sizeof(Item));
    const size_t o_items1 = carve(size_t(cap_items) * sizeof(Item));
    const size_t o_bins = carve(size_t(cap_items) * 3 * kBins * sizeof(BinKeys));
    const size_t o_small = carve(size_t(cap_small) * sizeof(SmallItem));
    const size_t o_scount = carve(size_t(cap_small + 1) * 4);
    const size_t o_tnodes = carve(size_t(2) * n * sizeof(RefNode));
    const size_t o_keys = carve(6 * 8);
    const size_t o_ctr = carve(sizeof(Counters));
    char* ws = nullptr;
    int rc = CERES_OK;
    Counters h{};
    uint32_t n_items = 0;
    int cur = 0;
    BVH_TRY(hipMallocAsync(reinterpret_cast<void**>(&ws), off, stream));
    {
        PrimRec* rec = reinterpret_cast<PrimRec*>(ws + o_rec);
        int32_t* seg = reinterpret_cast<int32_t*>(ws + o_seg);
        uint32_t* flag = reinterpret_cast<uint32_t*>(ws + o_flag);
        uint32_t* X = reinterpret_cast<uint32_t*>(ws + o_X);
        uint32_t* part = reinterpret_cast<uint32_t*>(ws + o_part);
        uint32_t* posF = reinterpret_cast<uint32_t*>(ws + o_posF);
        uint32_t* posT = reinterpret_cast<uint32_t*>(ws + o_posT);
        Item* items[2] = {reinterpret_cast<Item*>(ws + o_items0), reinterpret_cast<Item*>(ws + o_items1)};
        BinKeys* bins = reinterpret_cast<BinKeys*>(ws + o_bins);
        SmallItem* small = reinterpret_cast<SmallItem*>(ws + o_small);
        uint32_t* scount = reinterpret_cast<uint32_t*>(ws + o_scount);
        RefNode* tnodes = reinterpret_cast<RefNode*>(ws + o_tnodes);
        unsigned long long* keys = reinterpret_cast<unsigned long long*>(ws + o_keys);
        Counters* ctr = reinterpret_cast<Counters*>(ws + o_ctr);
        const unsigned long long key_init[6] = {kKeyMinEmpty, kKeyMinEmpty, kKeyMinEmpty, kKeyMaxEmpty, kKeyMaxEmpty, kKeyMaxEmpty};
        BVH_TRY(hipMemcpyAsync(keys, key_init, sizeof key_init, hipMemcpyHostToDevice, stream));
        const uint32_t g256 = (n + 255) / 256;
        hipLaunchKernelGGL(k_init, dim3((n + 256 * kInitPer - 1) / (256 * kInitPer)), dim3(256), 0, stream, reinterpret_cast<const Tri48*>(d_tri48), n, rec, seg,
                           n > kSmall ? 0 : -1, keys);
        BVH_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_root, dim3(1), dim3(64), 0, stream, nodes, keys, n, items[0], small, ctr);
        BVH_TRY(hipGetLastError());
        n_items = n > kSmall ? 1 : 0;
        h.n_small = n > kSmall ? 0 : 1;
        h.n_nodes = 1;
        while (n_items) {
            if (n_items > cap_items) { rc = set_error(CERES_EINVAL, "bvh build: item capacity exceeded"); goto done; }
            Item* it = items[cur];
            hipLaunchKernelGGL(k_item_prep, dim3(n_items), dim3(64), 0, stream, it, n_items, nodes, bins);
            hipLaunchKernelGGL(k_bin, dim3(chunks), dim3(256), 0, stream, rec, seg, n, it, bins);
            if (gfma) hipLaunchKernelGGL(k_split<true>, dim3((n_items + 63) / 64), dim3(64), 0, stream, it, n_items, nodes, bins);
            else hipLaunchKernelGGL(k_split<false>, dim3((n_items + 63) / 64), dim3(64), 0, stream, it, n_items, nodes, bins);
            hipLaunchKernelGGL(k_flags, dim3(g256), dim3(256), 0, stream, rec, seg, n, it, flag);
            hipLaunchKernelGGL(k_scan_reduce, dim3(scan_blocks), dim3(256), 0, stream, flag, n, part);
            hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, stream, part, scan_blocks);
            hipLaunchKernelGGL(k_scan_down, dim3(scan_blocks), dim3(256), 0, stream, flag, n, part, X);
            hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, stream, it, n_items, X, nodes, ctr, small);
            hipLaunchKernelGGL(k_emit, dim3((n_items + 63) / 64), dim3(64), 0, stream, it, n_items, nodes, bins, items[cur ^ 1]);
            hipLaunchKernelGGL(k_pos, dim3(g256), dim3(256), 0, stream, seg, n, it, flag, X, posF, posT);
            hipLaunchKernelGGL(k_swap_seg, dim3(g256), dim3(256), 0, stream, rec, seg, n, it, posF, posT);
            BVH_TRY(hipGetLastError());
            BVH_TRY(hipMemcpyAsync(&h, ctr, sizeof h, hipMemcpyDeviceToHost, stream));
            BVH_TRY(hipStreamSynchronize(stream));
            n_items = h.n_items;
            cur ^= 1;
            if (h.n_small > cap_small) { rc = set_error(CERES_EINVAL, "bvh build: small-item capacity exceeded"); goto done; }
        }
        const uint32_t n_small = h.n_small;
        hipLaunchKernelGGL(k_prim_out, dim3(g256), dim3(256), 0, stream, rec, n, d_prim32);
        uint32_t sub_total = 0;
        if (n_small) {                                   // all-large-leaf builds have no subtrees
            if (gfma) hipLaunchKernelGGL(k_small<true>, dim3(n_small), dim3(64), 0, stream, rec, small, n_small, nodes, tnodes, scount, d_prim32);
            else hipLaunchKernelGGL(k_small<false>, dim3(n_small), dim3(64), 0, stream, rec, small, n_small, nodes, tnodes, scount, d_prim32);
            BVH_TRY(hipGetLastError());
            // exclusive scan of the subtree node counts (n_small + 1 entries)
            BVH_TRY(hipMemcpyAsync(part, scount, size_t(n_small) * 4, hipMemcpyDeviceToDevice, stream));
            hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, stream, part, n_small);
            hipLaunchKernelGGL(k_place, dim3(n_small), dim3(64), 0, stream, small, n_small, part, tnodes, nodes, h.n_nodes);
            BVH_TRY(hipGetLastError());
            BVH_TRY(hipMemcpyAsync(&sub_total, part + n_small, 4, hipMemcpyDeviceToHost, stream));
        }
        BVH_TRY(hipStreamSynchronize(stream));
        *n_nodes = size_t(h.n_nodes) + sub_total;
    }
done:
    if (ws) (void)hipFreeAsync(ws, stream);
    return rc;
}

// Host-buffer convenience with ceres_bvh_build's signature and output: the same BVH as the
// host builder (canonical topology + leaf order), built on `device`.
int ceres_bvh_build_device(const float* d_tri48, size_t n_tri, uint32_t* d_nodes32, uint32_t* d_prim32,
                           size_t* n_nodes, void* stream_) {
    return ceres_bvh_build_device_arith(d_tri48, n_tri, d_nodes32, d_prim32, n_nodes, stream_, CERES_ARITH_EXACT);
}

int ceres_bvh_build_gpu_arith(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64,
                              int device, int arith) {
    if (!tri48 || !nodes32 || !n_nodes || !prim64) return set_error(CERES_EINVAL, "ceres_bvh_build_gpu: null argument");
    if (n_tri == 0) return set_error(CERES_EINVAL, "The given scene is empty or cannot be loaded");
    if (n_tri > 0x7fffffffu) return set_error(CERES_EUNSUPPORTED, "more than 2^31 triangles");
    *nodes32 = nullptr; *prim64 = nullptr; *n_nodes = 0;
    int rc = CERES_OK;
    float* d_tri = nullptr;
    uint32_t* d_nodes = nullptr;
    uint32_t* d_prim = nullptr;
    hipStream_t stream = nullptr;
    uint32_t* hp = nullptr;
    size_t m = 0;
    const size_t cap_nodes = 2 * n_tri - 1;
    BVH_TRY(hipSetDevice(device));
    BVH_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    BVH_TRY(hipMalloc(&d_tri, n_tri * 48));
    BVH_TRY(hipMalloc(&d_nodes, cap_nodes * sizeof(RefNode)));
    BVH_TRY(hipMalloc(&d_prim, n_tri * 4));
    BVH_TRY(hipMemcpyAsync(d_tri, tri48, n_tri * 48, hipMemcpyHostToDevice, stream));
    if ((rc = ceres_bvh_build_device_arith(d_tri, n_tri, d_nodes, d_prim, &m, stream, arith)) != CERES_OK) goto done;
    *nodes32 = static_cast<uint32_t*>(std::malloc(m * sizeof(RefNode)));
    *prim64 = static_cast<uint64_t*>(std::malloc(n_tri * 8));
    hp = static_cast<uint32_t*>(std::malloc(n_tri * 4));
    if (!*nodes32 || !*prim64 || !hp) { rc = set_error(CERES_ENOMEM, "out of host memory"); goto done; }
    BVH_TRY(hipMemcpyAsync(*nodes32, d_nodes, m * sizeof(RefNode), hipMemcpyDeviceToHost, stream));
    BVH_TRY(hipMemcpyAsync(hp, d_prim, n_tri * 4, hipMemcpyDeviceToHost, stream));
    BVH_TRY(hipStreamSynchronize(stream));
    for (size_t i = 0; i < n_tri; ++i) (*prim64)[i] = hp[i];
    *n_nodes = m;
done:
    std::free(hp);
    if (rc != CERES_OK) { std::free(*nodes32); std::free(*prim64); *nodes32 = nullptr; *prim64 = nullptr; }
    if (d_tri) (void)hipFree(d_tri);
    if (d_nodes) (void)hipFree(d_nodes);
    if (d_prim) (void)hipFree(d_prim);
    if (stream) (void)hipStreamDestroy(stream);
    return rc;
}

int ceres_bvh_build_gpu(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64,
                        int device) {
    return ceres_bvh_build_gpu_arith(tri48, n_tri, nodes32, n_nodes, prim64, device, CERES_ARITH_EXACT);
}

}  // extern "C"
