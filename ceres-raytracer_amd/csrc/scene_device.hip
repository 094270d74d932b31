// scene_device.hip -- device-resident scene preparation: the host relayout (relayout_bvh +
// build_shadow_bvh4, scene_host.cpp) rebuilt as gfx950 kernels over device arrays, so the
// whole pre-path (OBJ text -> triangles + normals -> BVH -> GPU layout) can stay in HBM
// (SURVEY.md §8(f) f1/f2).
//
// Same records, numbered differently: the host numbers sibling pairs / BVH4 nodes in a
// depth-first walk; here pair(X) = rank of inner node X among the reachable inner nodes in node
// order and node4(X) = rank among the BVH4 roots.  Traversal order and results depend only on
// the topology (near-first order within a pair, stack order), never on record numbers, so the
// images are identical (tests/test_gpu_scene.py renders through both).
//
// One breadth-first pass over the BVH2 (one launch per level, <= 64 levels) validates the tree
// (child indices in range, leaf ranges inside primitive_indices, no node reached twice), gives
// each inner node its level (the traversal stack needs depth - 1 entries) and its BVH4 role:
// a pair P heads a BVH4 record when it is the root, when its parent pair heads a record and P
// is not collapsed into it, or when its parent was collapsed; collapse(P) = both of P's child
// boxes lie inside P's box (build_shadow_bvh4's exact containment rule).  The BVH4 stack bound
// (most pushes along a root-leaf path) is propagated along the same walk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "dev_scan.hpp"
#include "host_common.hpp"

namespace ceres {
namespace scenedev {

using namespace devscan;

enum : uint32_t { kErrRange = 1, kErrLeaf = 2, kErrShared = 4, kErrPrim = 8, kErrNode4 = 16 };

__device__ __forceinline__ bool inside(const float* c, const float* p) {          // build_shadow_bvh4 `inside`
    return c[0] >= p[0] && c[1] <= p[1] && c[2] >= p[2] && c[3] <= p[3] && c[4] >= p[4] && c[5] <= p[5];
}

// collapse test for inner node q (children q.first, q.first + 1 already range-checked)
__device__ __forceinline__ bool collapses(const RefNode* nodes, uint32_t q) {
    const uint32_t g = nodes[q].first_child_or_primitive;
    return inside(nodes[g].bounds, nodes[q].bounds) && inside(nodes[g + 1].bounds, nodes[q].bounds);
}

struct LevelCtx {
    const RefNode* nodes;
    uint32_t n_nodes, n_tri;
    uint32_t* visited;      // per node: reached
    uint32_t* inner;        // per node: reachable inner node
    uint32_t* is4;          // per node: heads a BVH4 record
    uint32_t* acc_in;       // per BVH4 head: pushes on the stack above it
    uint32_t* stack4;       // max over records of acc_in + max(0, inner entries - 1)
    uint32_t* err;
};

__device__ bool check_child(const LevelCtx& C, uint32_t ch) {
    if (atomicExch(&C.visited[ch], 1u) != 0u) { atomicOr(C.err, uint32_t(kErrShared)); return false; }
    const RefNode& n = C.nodes[ch];
    if (n.primitive_count) {
        if (uint64_t(n.first_child_or_primitive) + n.primitive_count > C.n_tri) { atomicOr(C.err, uint32_t(kErrLeaf)); return false; }
        return true;
    }
    if (uint64_t(n.first_child_or_primitive) + 1 >= C.n_nodes) { atomicOr(C.err, uint32_t(kErrRange)); return false; }
    return true;
}

__global__ void __launch_bounds__(256) k_level(LevelCtx C, const uint32_t* __restrict__ frontier, uint32_t nf,
                                               uint32_t* __restrict__ next, uint32_t* __restrict__ n_next) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= nf) return;
    const uint32_t x = frontier[i];
    const uint32_t c = C.nodes[x].first_child_or_primitive;
    bool ok[2];
    for (int k = 0; k < 2; ++k) ok[k] = check_child(C, c + k);
    if (!ok[0] || !ok[1]) return;
    bool inner[2], col[2] = {false, false};
    for (int k = 0; k < 2; ++k) {
        inner[k] = C.nodes[c + k].primitive_count == 0;
        if (inner[k]) {
            // grandchild indices must be valid before the containment test reads them
            const uint32_t g = C.nodes[c + k].first_child_or_primitive;
            if (uint64_t(g) + 1 >= C.n_nodes) { atomicOr(C.err, uint32_t(kErrRange)); return; }
            col[k] = collapses(C.nodes, c + k);
        }
    }
    if (C.is4[x]) {
        // this record's entries: leaves, collapsed children's two children, other inner children
        uint32_t n_inner = 0;
        for (int k = 0; k < 2; ++k) {
            if (!inner[k]) continue;
            if (col[k]) {
                const uint32_t g = C.nodes[c + k].first_child_or_primitive;
                n_inner += (C.nodes[g].primitive_count == 0) + (C.nodes[g + 1].primitive_count == 0);
            } else {
                n_inner += 1;
            }
        }
        const uint32_t acc = C.acc_in[x] + (n_inner > 1 ? n_inner - 1 : 0);
        atomicMax(C.stack4, acc);
        for (int k = 0; k < 2; ++k) {
            if (!inner[k]) continue;
            if (!col[k]) { C.is4[c + k] = 1; C.acc_in[c + k] = acc; continue; }
            C.is4[c + k] = 0;
            const uint32_t g = C.nodes[c + k].first_child_or_primitive;
            for (int q = 0; q < 2; ++q) if (C.nodes[g + q].primitive_count == 0) C.acc_in[g + q] = acc;
        }
    } else {
        for (int k = 0; k < 2; ++k) if (inner[k]) C.is4[c + k] = 1;   // children of a collapsed pair head records
    }
    for (int k = 0; k < 2; ++k) {
        if (!inner[k]) continue;
        C.inner[c + k] = 1;
        next[atomicAdd(n_next, 1u)] = c + k;
    }
}

__global__ void __launch_bounds__(256) k_flags4(const uint32_t* __restrict__ inner, const uint32_t* __restrict__ is4, uint32_t n,
                                                uint32_t* __restrict__ f4) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) f4[i] = inner[i] && is4[i];
}

// one SiblingPair per reachable inner node (relayout_bvh's record, scene_host.cpp)
__global__ void __launch_bounds__(256) k_pairs(const RefNode* __restrict__ nodes, uint32_t n_nodes, const uint32_t* __restrict__ inner,
                                               const uint32_t* __restrict__ pair_of, SiblingPair* __restrict__ pairs) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= n_nodes || !inner[x]) return;
    const uint32_t c = nodes[x].first_child_or_primitive;
    SiblingPair r;
    for (int k = 0; k < 6; ++k) { r.lb[k] = nodes[c].bounds[k]; r.rb[k] = nodes[c + 1].bounds[k]; }
    const RefNode& L = nodes[c];
    const RefNode& R = nodes[c + 1];
    r.lcount = L.primitive_count; r.lfirst = L.primitive_count ? L.first_child_or_primitive : pair_of[c];
    r.rcount = R.primitive_count; r.rfirst = R.primitive_count ? R.first_child_or_primitive : pair_of[c + 1];
    pairs[pair_of[x]] = r;
}

// one Node4 per BVH4 head (build_shadow_bvh4's record)
__global__ void __launch_bounds__(256) k_nodes4(const RefNode* __restrict__ nodes, uint32_t n_nodes, const uint32_t* __restrict__ f4,
                                                const uint32_t* __restrict__ node4_of, Node4* __restrict__ out,
                                                uint32_t* __restrict__ err) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= n_nodes || !f4[x]) return;
    struct Entry { uint32_t node; };
    uint32_t ent[4];
    int n = 0;
    const uint32_t c = nodes[x].first_child_or_primitive;
    for (int k = 0; k < 2; ++k) {
        const RefNode& ch = nodes[c + k];
        if (ch.primitive_count == 0 && collapses(nodes, c + k)) {
            const uint32_t g = ch.first_child_or_primitive;
            ent[n++] = g;
            ent[n++] = g + 1;
        } else {
            ent[n++] = c + k;
        }
    }
    Node4 r;
    for (int q = 0; q < 4; ++q) {
        if (q >= n) {
            r.lo_x[q] = r.lo_y[q] = r.lo_z[q] = INFINITY;             // the inverted infinite box (build_shadow_bvh4)
            r.hi_x[q] = r.hi_y[q] = r.hi_z[q] = -INFINITY;
            r.child[q] = kNode4Empty;
            continue;
        }
        const RefNode& e = nodes[ent[q]];
        r.lo_x[q] = e.bounds[0]; r.hi_x[q] = e.bounds[1];
        r.lo_y[q] = e.bounds[2]; r.hi_y[q] = e.bounds[3];
        r.lo_z[q] = e.bounds[4]; r.hi_z[q] = e.bounds[5];
        const uint32_t first = e.primitive_count ? e.first_child_or_primitive : node4_of[ent[q]];
        if (e.primitive_count > kNode4MaxCount || first > kNode4MaxFirst) atomicOr(err, uint32_t(kErrNode4));
        r.child[q] = node4_child(e.primitive_count, first);
    }
    node4_leaves_first(r);
    out[node4_of[x]] = r;
}

// triangles in leaf order + original indices (relayout_bvh)
__global__ void __launch_bounds__(256) k_leaf_tris(const Tri48* __restrict__ tris, const uint32_t* __restrict__ prim, uint32_t n_tri,
                                                   Tri48* __restrict__ leaf_tris, uint32_t* __restrict__ orig, uint32_t* __restrict__ err) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n_tri) return;
    const uint32_t p = prim[k];
    if (p >= n_tri) { atomicOr(err, uint32_t(kErrPrim)); return; }
    leaf_tris[k] = tris[p];
    orig[k] = p;
}

}  // namespace scenedev

// Device relayout; outputs are hipMalloc'd (owned by the scene).  Returns CERES_* status.
int relayout_device(const Tri48* d_tris, uint32_t n_tri, const RefNode* d_nodes, uint32_t n_nodes, const uint32_t* d_prim,
                    hipStream_t stream, DeviceLayout& out) {
    using namespace scenedev;
    int rc = CERES_OK;
    uint32_t* ws = nullptr;
    auto fail_hip = [&](hipError_t e, const char* what) { return set_error(CERES_EHIP, "%s: %s", what, hipGetErrorString(e)); };
#define SD_TRY(expr) do { hipError_t e_ = (expr); if (e_ != hipSuccess) { rc = fail_hip(e_, #expr); goto done; } } while (0)
    {
        // workspace: visited, inner, is4, acc_in, f4, pair_of(+1), node4_of(+1), 2 frontiers, counters, partials
        const size_t N = n_nodes;
        const size_t parts = scan_blocks(n_nodes) + 2;
        const size_t words = 7 * (N + 1) + 2 * N + 8 + parts;
        uint32_t *visited, *inner, *is4, *acc_in, *f4, *pair_of, *node4_of, *fr[2], *ctr, *part;
        uint32_t h_ctr[8];
        uint32_t nf = 1, level = 0, cur = 0;
        SD_TRY(hipMallocAsync(reinterpret_cast<void**>(&ws), words * 4, stream));
        SD_TRY(hipMemsetAsync(ws, 0, words * 4, stream));
        visited = ws; inner = visited + N + 1; is4 = inner + N + 1; acc_in = is4 + N + 1; f4 = acc_in + N + 1;
        pair_of = f4 + N + 1; node4_of = pair_of + N + 1; fr[0] = node4_of + N + 1; fr[1] = fr[0] + N;
        ctr = fr[1] + N; part = ctr + 8;          // ctr: [0] next count, [1] stack4, [2] err
        // leaf-order triangles
        SD_TRY(hipMalloc(&out.tris, size_t(n_tri) * sizeof(Tri48)));
        SD_TRY(hipMalloc(&out.orig, size_t(n_tri) * 4));
        hipLaunchKernelGGL(k_leaf_tris, dim3((n_tri + 255) / 256), dim3(256), 0, stream, d_tris, d_prim, n_tri, out.tris, out.orig,
                           ctr + 2);
        SD_TRY(hipGetLastError());
        RefNode root;
        SD_TRY(hipMemcpyAsync(&root, d_nodes, sizeof root, hipMemcpyDeviceToHost, stream));
        SD_TRY(hipStreamSynchronize(stream));
        for (int k = 0; k < 6; ++k) out.root_box[k] = root.bounds[k];
        out.root_leaf_count = out.root_leaf_first = 0;
        if (root.primitive_count) {                                  // the root is a leaf (single_ray_traverser.hpp:72-73)
            if (uint64_t(root.first_child_or_primitive) + root.primitive_count > n_tri) { rc = set_error(CERES_EINVAL, "root leaf range out of bounds"); goto done; }
            out.root_leaf_count = root.primitive_count;
            out.root_leaf_first = root.first_child_or_primitive;
            out.depth = 0;
            out.stack4 = 0;
            out.n_pairs = 1;
            out.n_nodes4 = 1;
            SD_TRY(hipMalloc(&out.pairs, sizeof(SiblingPair)));
            SD_TRY(hipMemsetAsync(out.pairs, 0, sizeof(SiblingPair), stream));
            SD_TRY(hipMalloc(&out.nodes4, sizeof(Node4)));
            SD_TRY(hipMemsetAsync(out.nodes4, 0, sizeof(Node4), stream));
        } else {
            if (uint64_t(root.first_child_or_primitive) + 1 >= n_nodes) { rc = set_error(CERES_EINVAL, "root child index out of range"); goto done; }
            const uint32_t one = 1, zero = 0;
            SD_TRY(hipMemcpyAsync(fr[0], &zero, 4, hipMemcpyHostToDevice, stream));
            SD_TRY(hipMemcpyAsync(visited, &one, 4, hipMemcpyHostToDevice, stream));
            SD_TRY(hipMemcpyAsync(inner, &one, 4, hipMemcpyHostToDevice, stream));
            SD_TRY(hipMemcpyAsync(is4, &one, 4, hipMemcpyHostToDevice, stream));
            LevelCtx C{d_nodes, n_nodes, n_tri, visited, inner, is4, acc_in, ctr + 1, ctr + 2};
            while (nf) {
                if (++level > 65) { rc = set_error(CERES_EINVAL, "BVH deeper than 64 levels or cyclic"); goto done; }
                SD_TRY(hipMemsetAsync(ctr, 0, 4, stream));
                hipLaunchKernelGGL(k_level, dim3((nf + 255) / 256), dim3(256), 0, stream, C, fr[cur], nf, fr[cur ^ 1], ctr);
                SD_TRY(hipGetLastError());
                SD_TRY(hipMemcpyAsync(h_ctr, ctr, 12, hipMemcpyDeviceToHost, stream));
                SD_TRY(hipStreamSynchronize(stream));
                if (h_ctr[2]) break;
                nf = h_ctr[0];
                cur ^= 1;
            }
            if (h_ctr[2]) {
                rc = set_error(CERES_EINVAL, "invalid BVH (%s%s%s%s)", h_ctr[2] & kErrRange ? "child index out of range " : "",
                               h_ctr[2] & kErrLeaf ? "leaf range out of bounds " : "", h_ctr[2] & kErrShared ? "node reached twice " : "",
                               h_ctr[2] & kErrPrim ? "primitive index out of range" : "");
                goto done;
            }
            out.depth = level;                                       // levels of inner nodes (root = 1)
            out.stack4 = h_ctr[1];
            // numbering: pairs over reachable inner nodes, BVH4 records over heads
            SD_TRY(exclusive_scan(inner, n_nodes, pair_of, part, stream));
            hipLaunchKernelGGL(k_flags4, dim3((n_nodes + 255) / 256), dim3(256), 0, stream, inner, is4, n_nodes, f4);
            SD_TRY(exclusive_scan(f4, n_nodes, node4_of, part, stream));
            uint32_t np = 0, n4 = 0;
            SD_TRY(hipMemcpyAsync(&np, pair_of + n_nodes, 4, hipMemcpyDeviceToHost, stream));
            SD_TRY(hipMemcpyAsync(&n4, node4_of + n_nodes, 4, hipMemcpyDeviceToHost, stream));
            SD_TRY(hipStreamSynchronize(stream));
            out.n_pairs = np;
            out.n_nodes4 = std::max<uint32_t>(n4, 1);
            SD_TRY(hipMalloc(&out.pairs, size_t(np) * sizeof(SiblingPair)));
            SD_TRY(hipMalloc(&out.nodes4, size_t(out.n_nodes4) * sizeof(Node4)));
            hipLaunchKernelGGL(k_pairs, dim3((n_nodes + 255) / 256), dim3(256), 0, stream, d_nodes, n_nodes, inner, pair_of, out.pairs);
            hipLaunchKernelGGL(k_nodes4, dim3((n_nodes + 255) / 256), dim3(256), 0, stream, d_nodes, n_nodes, f4, node4_of, out.nodes4,
                               ctr + 2);
            SD_TRY(hipGetLastError());
        }
        uint32_t perr = 0;
        SD_TRY(hipMemcpyAsync(&perr, ctr + 2, 4, hipMemcpyDeviceToHost, stream));
        SD_TRY(hipStreamSynchronize(stream));
        if (perr & kErrPrim) { rc = set_error(CERES_EINVAL, "primitive index out of range"); goto done; }
        if (perr & kErrNode4) {
            // a leaf of more than 31 triangles (coincident centroids: the builder could not split
            // it) does not fit a packed child word; the host collapse turns such leaves into piece
            // nodes (build_shadow_bvh4).  Rare, one-off scene preparation: the pair records go to
            // the host and the BVH4 records come back.
            std::vector<SiblingPair> hp(out.n_pairs);
            std::vector<Node4> n4;
            uint32_t st4 = 0, not_collapsed = 0;
            SD_TRY(hipMemcpyAsync(hp.data(), out.pairs, hp.size() * sizeof(SiblingPair), hipMemcpyDeviceToHost, stream));
            SD_TRY(hipStreamSynchronize(stream));
            if ((rc = build_shadow_bvh4(hp, n4, st4, not_collapsed))) goto done;
            SD_TRY(hipFree(out.nodes4));
            out.nodes4 = nullptr;
            SD_TRY(hipMalloc(&out.nodes4, n4.size() * sizeof(Node4)));
            SD_TRY(hipMemcpyAsync(out.nodes4, n4.data(), n4.size() * sizeof(Node4), hipMemcpyHostToDevice, stream));
            SD_TRY(hipStreamSynchronize(stream));
            out.n_nodes4 = uint32_t(n4.size());
            out.stack4 = st4;
        }
    }
#undef SD_TRY
done:
    if (ws) { (void)hipFreeAsync(ws, stream); (void)hipStreamSynchronize(stream); }
    return rc;
}

}  // namespace ceres
