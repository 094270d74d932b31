// ceres_types.hpp -- data layouts shared by the host scene code and the gfx950 kernels.
//
// HBM layout of a device scene (DESIGN.md "Data layout in HBM"):
//
//   pairs[]  64-B SiblingPair records, one per inner node of the reference BVH, holding
//            BOTH children's boxes and links.  The reference traverser always tests the two
//            children of a node together (single_ray_traverser.hpp:85-87) and the reference
//            keeps siblings adjacent (bvh.hpp:9-13, 32 B each), so one traversal step is
//            exactly one 64-B record = four 16-B loads per lane, 64-B aligned (the reference
//            pairs start at odd node indices, i.e. straddle 64-B boundaries).  Records are
//            numbered in depth-first order of the reference topology.
//   tris[]   48-B triangles {p0, e1, e2, n} (triangle.hpp:17-37) permuted into leaf order,
//            so a leaf is a contiguous run: the reference's per-test u64 index gather
//            (primitive_intersectors.hpp:17-20) disappears from the traversal loop.
//   orig[]   u32 original triangle index per leaf slot (read once per primary hit).
//   norms[]  36-B per-triangle vertex normals in ORIGINAL order (obj_norms.hpp:113-115),
//            read only for lit pixels.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace ceres {

struct Tri48 {                 // == bvh::Triangle<float>
    float p0[3], e1[3], e2[3], n[3];
};
static_assert(sizeof(Tri48) == 48, "Tri48");

struct RefNode {               // == bvh::Bvh<float>::Node (bvh.hpp:25-30)
    float bounds[6];           // xmin, xmax, ymin, ymax, zmin, zmax
    uint32_t primitive_count;  // 0 = inner node
    uint32_t first_child_or_primitive;
};
static_assert(sizeof(RefNode) == 32, "RefNode");

struct alignas(16) SiblingPair {
    float lb[6];               // left child bounds  (reference order xmin,xmax,ymin,ymax,zmin,zmax)
    float rb[6];               // right child bounds
    uint32_t lcount, lfirst;   // count 0: inner, first = pair index of its children;
    uint32_t rcount, rfirst;   // count > 0: leaf, first = first leaf slot in tris[]
};
static_assert(sizeof(SiblingPair) == 64, "SiblingPair");

// Double precision (render<double>, anim.cpp -d): the reference's Bvh<double>::Node (64 B),
// Triangle<double> (96 B) and the sibling-pair record with double bounds (112 B = 7 x 16 B).
struct RefNode64 {
    double bounds[6];
    uint64_t primitive_count;
    uint64_t first_child_or_primitive;
};
static_assert(sizeof(RefNode64) == 64, "RefNode64");
struct Tri96 { double p0[3], e1[3], e2[3], n[3]; };
static_assert(sizeof(Tri96) == 96, "Tri96");
struct alignas(16) SiblingPair64 {
    double lb[6], rb[6];
    uint32_t lcount, lfirst, rcount, rfirst;
};
static_assert(sizeof(SiblingPair64) == 112, "SiblingPair64");

// Shadow-ray BVH4 record (build_shadow_bvh4, scene_host.cpp; k_nodes4, scene_device.hip): 4 child
// boxes as SoA float4 rows, then one packed word per child: first << 5 | count (count 0: inner,
// first = Node4 index; 1..31: leaf of `count` triangles from leaf slot `first`), kNode4Empty for
// an unused slot.  One word per child keeps a traversal step at 7 vector loads instead of 8 (the
// kernel pays per load instruction).  128 B = one L2 line.  Children are stored leaves
// first, then inner children, then empty slots (each group in build order: node4_leaves_first),
// and nleaf counts the leaf children -- the packet walk's per-child leaf / inner split is one
// compare against it.  An empty slot holds the inverted infinite box (lo +inf, hi -inf), which
// every slab test fails.
constexpr uint32_t kNode4Empty = 0xffffffffu;
constexpr uint32_t kNode4CountBits = 5;
constexpr uint32_t kNode4MaxCount = (1u << kNode4CountBits) - 1;             // 31
constexpr uint32_t kNode4MaxFirst = (1u << (32 - kNode4CountBits)) - 2;      // keeps clear of kNode4Empty
struct alignas(128) Node4 {
    float lo_x[4], hi_x[4], lo_y[4], hi_y[4], lo_z[4], hi_z[4];
    uint32_t child[4];
    uint32_t nleaf;
    uint32_t unused[3];
};
static_assert(sizeof(Node4) == 128, "Node4");
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t node4_child(uint32_t count, uint32_t first) { return first << kNode4CountBits | count; }

// Reorders a filled record's children: leaves, inner children, empty slots (stable within each
// group, so the walk still meets inner children in build order), sets nleaf, zeroes the rest.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline void node4_leaves_first(Node4& r) {
    Node4 t;
    uint32_t k = 0, nl = 0;
    for (int pass = 0; pass < 3; ++pass)
        for (int c = 0; c < 4; ++c) {
            const uint32_t w = r.child[c];
            const int group = w == kNode4Empty ? 2 : (w & kNode4MaxCount) ? 0 : 1;
            if (group != pass) continue;
            t.lo_x[k] = r.lo_x[c]; t.hi_x[k] = r.hi_x[c];
            t.lo_y[k] = r.lo_y[c]; t.hi_y[k] = r.hi_y[c];
            t.lo_z[k] = r.lo_z[c]; t.hi_z[k] = r.hi_z[c];
            t.child[k] = w;
            nl += group == 0;
            ++k;
        }
    t.nleaf = nl;
    t.unused[0] = t.unused[1] = t.unused[2] = 0;
    r = t;
}

// Compressed shadow BVH4 record (CERES_MODE_QBVH4; quantize_nodes4 in render_hip.hip): the node's
// box origin and a power-of-two scale per axis, each child bound as one byte (4 children's lo_x
// bytes in one word, ...), and the same packed child words as Node4.  Bound = fma(byte, scale,
// origin), rounded outwards on the host (the decoded box always contains the exact one).
// 64 B = four 16-B loads per step instead of seven.
struct alignas(64) QNode4 {
    float ox, oy, oz, sx;
    float sy, sz;
    uint32_t qlx, qhx;           // byte c = child c
    uint32_t qly, qhy, qlz, qhz;
    uint32_t child[4];
};
static_assert(sizeof(QNode4) == 64, "QNode4");

constexpr int kShards = 32;    // counter shards (one 128-B line each), wavefront w adds to shard w % 32
struct alignas(128) Shard {
    uint32_t queued;           // shadow rays traced
    uint32_t error;            // traversal stack overflow flag
    unsigned long long hits;   // primary hits + occluded shadow rays
    unsigned long long pairs;  // node-pair visits (stats variant)
    unsigned long long tests;  // triangle tests (stats variant)
    uint32_t pad[24];
};
static_assert(sizeof(Shard) == 128, "Shard");

constexpr int kMaxFrames = 64;        // frames per batch call (ceres_render_batch_device)
constexpr int kFramesPerLaunch = 56;  // frames per kernel launch (KParams: cameras + cull rects inline, inside the 4 KB
                                      // kernarg limit); a larger batch is two launches on the same stream
struct FrameCam {              // one frame of a batch: eye + the render.hpp:91-97 basis + its sun
    float eye[3], dir[3], iu[3], iv[3], sun[3];
};

// A fused-kernel tile-order entry: frame, tile row and tile column in one word (decoded with bit
// extracts instead of two integer divisions per tile); used when the batch fits the fields.
constexpr uint32_t kTileXBits = 13, kTileYBits = 13;
constexpr uint32_t pack_tile(uint32_t f, uint32_t y, uint32_t x) { return (f << (kTileXBits + kTileYBits)) | (y << kTileXBits) | x; }

struct CullRect { uint16_t i0, i1, j0, j1; };   // pixels (column i, global row j) whose rays may reach the root box

struct KParams {
    FrameCam cam[kFramesPerLaunch];
    CullRect cull_rect[kFramesPerLaunch];        // production kernels: the background cull (tile_misses_root)
    uint32_t frames;                             // frames in this launch (1..kFramesPerLaunch)
    uint32_t W, H;
    uint32_t row_block, rank, world, local_rows; // this rank's rows of every frame (ceres_tiling)
    uint32_t bands;                              // ceres_tiling.bands: frame f renders band (rank + f) % world
    uint32_t band_magic;                         // ... ceil(2^32 / world): (rank + f) / world = umulhi(rank + f, magic)
    uint32_t row_blocks_per_frame;               // 16-row blocks of local rows per frame (primary grid.y)
    uint32_t stack_entries;
    uint32_t root_leaf_count, root_leaf_first;   // root is a leaf (single_ray_traverser.hpp:72-73)
    float root_box[6];                           // the root node's bounds (bvh.hpp:25-30 order) ...
    uint32_t root_box_ok;                        // ... and whether both root children lie inside it
    uint32_t cull;                               // production kernels: background tiles culled (tile_misses_root)
    uint32_t shadow_stack_entries;               // BVH4 traversal stack (shadow rays)
    uint32_t steal_first;                        // work-stealing shadow loop: first passing child, not nearest
    uint32_t packets;                            // batch kernel: wave-wide packets (L2-resident scenes, render_hip.hip)
    uint32_t tiles_x;                            // tile columns per row (fused kernel)
    uint32_t lds_entries;                        // fused kernel: LDS stack slots per lane (24-bit planes)
    uint32_t tile_packed;                        // fused kernel: tile_order entries are pack_tile() words
    const uint32_t* tile_order;                  // fused kernel: block -> batch tile (centre first)
    const SiblingPair* pairs;
    const Node4* nodes4;                         // shadow-ray BVH4 over the same leaf slots
    const QNode4* qnodes4;                       // its compressed copy (CERES_MODE_QBVH4 only)
    const Tri48* tris;
    const uint32_t* orig;
    const float* norms;
    float* pixels;             // [frames][local_rows][W][3] floats, row 0 = bottom (render.hpp:107)
    uint8_t* rgb8;             // [frames][local_rows][W][3] PPM body rows, top row first
    Shard* shards;
    // optional per-pixel hit records (G-buffer / parity output), batch pixel order
    int32_t* rec_prim;         // original triangle index, -1 on a primary miss
    float* rec_tuv;            // t, u, v of the primary hit
    int8_t* rec_shadow;        // -1 no shadow ray, 0 lit, 1 occluded
    // diagnostic (stats scenes only): 8 x u64 per wavefront of the fused kernel
    unsigned long long* wave_log;
};
static_assert(sizeof(KParams) <= 4096, "KParams must fit the 4 KB kernel-argument limit");

// device: reference BVH in HBM -> GPU layout (scene_device.hip); buffers hipMalloc'd
struct DeviceLayout {
    float root_box[6] = {0, 0, 0, 0, 0, 0};      // the reference root node's bounds
    SiblingPair* pairs = nullptr;
    Node4* nodes4 = nullptr;
    Tri48* tris = nullptr;
    uint32_t* orig = nullptr;
    size_t n_pairs = 0, n_nodes4 = 0;
    uint32_t depth = 0, stack4 = 0, root_leaf_count = 0, root_leaf_first = 0;
};
#ifdef __HIPCC__
int relayout_device(const Tri48* d_tris, uint32_t n_tri, const RefNode* d_nodes, uint32_t n_nodes, const uint32_t* d_prim,
                    hipStream_t stream, DeviceLayout& out);
#endif

// host: reference BVH -> GPU layout (scene_host.cpp)
int relayout_bvh(const RefNode* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri48* tris,
                 std::vector<SiblingPair>& pairs, std::vector<Tri48>& leaf_tris, std::vector<uint32_t>& orig,
                 uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first);
int build_shadow_bvh4(const std::vector<SiblingPair>& pairs, std::vector<Node4>& out, uint32_t& stack_bound,
                      uint32_t& not_collapsed);
int order_shadow_bvh4(std::vector<Node4>& nodes, uint32_t& first_bound);
int relayout_bvh64(const RefNode64* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri96* tris,
                   std::vector<SiblingPair64>& pairs, std::vector<Tri96>& leaf_tris, std::vector<uint32_t>& orig,
                   uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first);

}  // namespace ceres
