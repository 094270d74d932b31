// scene_internal.hpp -- the opaque ceres_scene of include/ceres_render.h, shared by the
// translation units that implement the ABI (render_hip.hip: float path, render64.hip: double).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>
#include <vector>

#include "ceres_types.hpp"

using ceres::SiblingPair; using ceres::SiblingPair64; using ceres::Node4; using ceres::Tri48; using ceres::Tri96;
using ceres::Shard;

struct ceres_scene {
    int device = 0;
    uint32_t flags = 0;
    size_t n_tri = 0, n_pairs = 0;
    uint32_t depth = 0, stack_entries = 1, root_leaf_count = 0, root_leaf_first = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};   // root node bounds; root_box_ok: both children inside it
    uint32_t root_box_ok = 0;
    uint32_t shadow_stack_entries = 1;     // BVH4 stack bound of the nearest-first walk (any child order)
    uint32_t shadow_stack_first = 1;       // ... of first-passing-child walks (order_shadow_bvh4; <= the above)
    size_t n_nodes4 = 0;
    SiblingPair* d_pairs = nullptr;
    Node4* d_nodes4 = nullptr;
    ceres::QNode4* d_qnodes4 = nullptr;   // compressed shadow BVH4, built on first CERES_MODE_QBVH4 render
    // fused-kernel tile orders, one per (frame size, tiling, batch, tile), never rewritten or
    // freed while a launch that reads them may be in flight (launches on different streams may
    // read different orders concurrently): an evicted order's buffer goes to `retired` and is
    // freed only once retired buffers exceed kRetiredBytes (counted at the allocation granule) or
    // number kMaxRetired, after one device synchronise -- no
    // per-launch events, and no stall while the working set of shapes fits the cache.
    struct TileOrder {
        size_t W = 0, H = 0;
        uint32_t row_block = 0, rank = 0, world = 0, frames = 0, tile = 0, bands = 0;
        bool packed = false;           // entries (f << 26) | (y << 13) | x (pack_tile) instead of linear ids
        uint32_t* d = nullptr;
        size_t cap = 0;                // entries allocated at d
        uint64_t used = 0;
    };
    std::vector<TileOrder> orders;
    std::vector<uint32_t*> retired;
    size_t retired_bytes = 0;
    uint64_t order_clock = 0;
    Tri48* d_tris = nullptr;
    uint32_t* d_orig = nullptr;
    float* d_norms = nullptr;
    Shard* d_shards = nullptr;
    bool shards_dirty = true;          // shards not known to be zero (see ceres_render_batch)
    uint64_t* d_counters = nullptr;
    float* d_pixels = nullptr;
    uint8_t* d_rgb8 = nullptr;
    size_t px_cap = 0;
    hipStream_t stream = nullptr;
    // host-buffer renders (ceres_render_f32): row bands rendered one after another on `stream`,
    // each band's D2H copy on `copy_stream` as soon as its kernel ends (the copy over the host
    // link, not the kernel, sets the call's length); counters per band
    hipStream_t copy_stream = nullptr;
    uint64_t* d_band_counters = nullptr;
    std::vector<hipEvent_t> band_events;
    // host float framebuffers (ceres_render_f32): the lit pixels -- those with any non-zero bit --
    // compacted on the device into {index, r, g, b} records, copied, and scattered over a host
    // zero fill that overlaps the kernel (host_fill_zero / host_scatter_lit, scene_host.cpp)
    uint4* d_lit = nullptr;
    uint32_t* d_lit_count = nullptr;
    size_t lit_cap = 0;
    uint32_t* h_small = nullptr;       // pinned: lit count + 8 counters
    std::vector<uint4> h_lit;
    uint4* h_lit_pinned = nullptr;     // zero-copy records (pinned host memory the compaction kernel writes)
    bool lit_zc = false;
    double last_lit_frac = 0.0;        // the previous call's lit fraction (dense frames take the full copy)
    uint32_t dense_calls = 0;
    hipEvent_t ev_count = nullptr;
    int num_cus = 256;
    size_t max_lds_per_block = 64 * 1024;   // hipDeviceProp_t::sharedMemPerBlock (set at scene creation)
    unsigned long long* d_wave_log = nullptr;   // stats scenes: per-wave diagnostic records
    size_t wave_log_waves = 0, last_grid_waves = 0;
    // optional per-launch device timing (ceres_scene_set_timing)
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<hipEvent_t> ev_used;   // pairs: before and after the render's kernel
    // double-precision scene (render<double>, render64.hip): set instead of the float layout
    bool f64 = false;
    SiblingPair64* d_pairs64 = nullptr;
    Tri96* d_tris64 = nullptr;
    double* d_norms64 = nullptr;
};

namespace ceres {
// host side of the compacted float readback (scene_host.cpp, OpenMP over the caller's cores)
void host_fill_zero(float* dst, size_t n);
void host_scatter_lit(float* dst, const uint32_t* lit4, size_t n);   // records {pixel, r, g, b}
void scene_release(ceres_scene* s);          // frees every device buffer and the stream (render_hip.hip)
// centre-first, XCD-balanced order of one whole frame's tile x tile tiles (render_hip.hip)
int frame_tile_order(ceres_scene* s, size_t W, size_t H, uint32_t tile, hipStream_t stream, const uint32_t** out);
constexpr size_t kMaxTileOrders = 16;         // cached orders per scene before LRU eviction
constexpr size_t kDramSceneBytes = size_t(64) << 20;   // a scene this large does not stay in the 8 x 4 MB L2s
#ifndef CERES_RETIRED_BYTES
#define CERES_RETIRED_BYTES (64u << 20)
#endif
constexpr size_t kRetiredBytes = CERES_RETIRED_BYTES;   // evicted orders kept until they exceed this ...
constexpr size_t kMaxRetired = 64;                      // ... or number this many buffers
constexpr size_t kAllocGranule = 4096;                  // bytes of a retired buffer counted per started granule
}
