// scene_host.cpp -- host-side scene preparation of the CERES hot path (product code).
//
// What the reference's callers run before render() (static.cpp:76-107, anim.cpp:38-65):
// OBJ parsing with vertex normals (obj_norms.hpp:57-127), rotate_triangles (render.hpp:24-44),
// the camera basis (render.hpp:91-97) and the binned-SAH BVH (binned_sah_builder.hpp:39-234).
// These stay on the host, as in the north star; they produce the exact bits the gfx950
// kernels consume, so every float operation follows the reference's order (the library is
// compiled with -ffp-contract=off; the reference's explicit fmaf stays an fmaf).
#include <algorithm>
#include <array>
#include <atomic>
#include <cctype>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "host_common.hpp"

namespace ceres {
namespace {

struct Vec { float x, y, z; };
inline float comp(const Vec& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
inline Vec operator+(Vec a, Vec b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec operator-(Vec a, Vec b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec scale(Vec a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float vdot(Vec a, Vec b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
inline Vec vcross(Vec a, Vec b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline Vec vnormalize(Vec v) { float inv = 1.0f / std::sqrt(vdot(v, v)); return scale(v, inv); }

inline Tri48 tri_from_points(Vec p0, Vec p1, Vec p2) {       // Triangle ctor, triangle.hpp:30-34
    Vec e1 = p0 - p1, e2 = p2 - p0, n = vcross(e1, e2);
    return Tri48{{p0.x, p0.y, p0.z}, {e1.x, e1.y, e1.z}, {e2.x, e2.y, e2.z}, {n.x, n.y, n.z}};
}
inline Vec P0(const Tri48& t) { return {t.p0[0], t.p0[1], t.p0[2]}; }
inline Vec E1(const Tri48& t) { return {t.e1[0], t.e1[1], t.e1[2]}; }
inline Vec E2(const Tri48& t) { return {t.e2[0], t.e2[1], t.e2[2]}; }
inline Vec N(const Tri48& t) { return {t.n[0], t.n[1], t.n[2]}; }

// ------------------------------------------------------------------ mesh assembly
// Accumulates fan-triangulated faces and area-weighted (un-normalised, left-handed) face
// normals per vertex in face order, exactly like obj_norms.hpp:84-115.
struct MeshBuilder {
    std::vector<Vec> verts, vn;
    std::vector<Tri48> tris;
    std::vector<uint32_t> corner;     // 3 vertex ids per triangle

    void add_vertex(Vec v) { verts.push_back(v); vn.push_back({0.f, 0.f, 0.f}); }
    void add_triangle(size_t a, size_t b, size_t c) {
        tris.push_back(tri_from_points(verts[a], verts[b], verts[c]));
        Vec n = N(tris.back());
        vn[a] = vn[a] + n; vn[b] = vn[b] + n; vn[c] = vn[c] + n;
        corner.push_back(uint32_t(a)); corner.push_back(uint32_t(b)); corner.push_back(uint32_t(c));
    }
    int finish(float** tri48, float** norm36, size_t* n_tri) {
        for (auto& n : vn) n = vnormalize(n);                // obj_norms.hpp:109-111
        const size_t nt = tris.size();
        *n_tri = nt;
        *tri48 = static_cast<float*>(std::malloc(std::max<size_t>(1, nt * 48)));
        *norm36 = static_cast<float*>(std::malloc(std::max<size_t>(1, nt * 36)));
        if (!*tri48 || !*norm36) { std::free(*tri48); std::free(*norm36); *tri48 = *norm36 = nullptr; return set_error(CERES_ENOMEM, "out of host memory"); }
        std::memcpy(*tri48, tris.data(), nt * 48);
        float* o = *norm36;
        for (size_t t = 0; t < nt; ++t)
            for (int k = 0; k < 3; ++k) {
                const Vec& v = vn[corner[3 * t + k]];
                o[9 * t + 3 * k] = v.x; o[9 * t + 3 * k + 1] = v.y; o[9 * t + 3 * k + 2] = v.z;
            }
        return CERES_OK;
    }
};

// ------------------------------------------------------------------ OBJ text (obj_norms.hpp:12-118)
inline char* skip_space(char* p) { while (std::isspace(static_cast<unsigned char>(*p))) ++p; return p; }
inline void trim_tail(char* p) {
    int i = int(std::strlen(p)) - 1;
    while (i > 0 && std::isspace(static_cast<unsigned char>(p[i]))) p[i--] = '\0';
}
// one face-vertex reference "i", "i/t", "i//n", "i/t/n" (negative = relative); false at end of list
inline bool face_index(char** cursor, long* out) {
    char* p = skip_space(*cursor);
    if (!std::isdigit(static_cast<unsigned char>(*p)) && *p != '-') return false;
    long idx = std::strtol(p, &p, 10);
    p = skip_space(p);
    if (*p == '/') {
        ++p;
        if (*p != '/') std::strtol(p, &p, 10);
        p = skip_space(p);
        if (*p == '/') { ++p; std::strtol(p, &p, 10); }
    }
    *cursor = p;
    *out = static_cast<int>(idx);                           // the reference stores it in an int
    return true;
}

int parse_obj(const char* data, size_t len, MeshBuilder& mb) {
    constexpr size_t kMaxLine = 1024;                       // istream::getline(line, 1024)
    char line[kMaxLine];
    size_t pos = 0;
    while (pos < len) {
        const char* nl = static_cast<const char*>(std::memchr(data + pos, '\n', len - pos));
        size_t n = nl ? size_t(nl - (data + pos)) : len - pos;
        if (n > kMaxLine - 1) break;                        // getline sets failbit: the reference stops reading
        std::memcpy(line, data + pos, n);
        line[n] = '\0';
        pos += n + (nl ? 1 : 0);
        char* p = skip_space(line);
        if (*p == '\0' || *p == '#') continue;
        trim_tail(p);
        if (p[0] == 'v' && std::isspace(static_cast<unsigned char>(p[1]))) {
            char* q = p + 1;
            float x = std::strtof(q, &q);
            float y = std::strtof(q, &q);
            float z = std::strtof(q, &q);
            mb.add_vertex({x, y, z});
        } else if (p[0] == 'f' && std::isspace(static_cast<unsigned char>(p[1]))) {
            char* q = p + 2;
            size_t first = 0, prev = 0;
            for (size_t k = 0;; ++k) {
                long idx;
                if (!face_index(&q, &idx)) break;
                size_t vtx = idx < 0 ? size_t(long(mb.verts.size()) + idx) : size_t(idx - 1);
                if (vtx >= mb.verts.size())
                    return set_error(CERES_EIO, "OBJ face references vertex %ld of %zu", idx, mb.verts.size());
                if (k == 0) first = vtx;
                else if (k == 1) prev = vtx;
                else { mb.add_triangle(first, prev, vtx); prev = vtx; }
            }
        }
    }
    return CERES_OK;
}

// ------------------------------------------------------------------ binned SAH BVH
// Same split rules as BinnedSahBuilder<Bvh,16> so the topology (and leaf order) is the
// reference's: 16 bins per axis on centroids (bin index by fmaf, :144-147), SAH sweeps
// (:89-114), axis choice (:170-174), leaf test with traversal_cost 1 (:179), 0.4-quantile
// fallback above 16 primitives (:180-196), std::partition (:199-201), child boxes from the
// bins (:216-224, including its use of the pre-fallback split count for the left box).
// Subtrees above 1024 primitives become OpenMP tasks (top_down_builder.hpp:63-66).
constexpr size_t kBins = 16, kMaxDepth = 64, kMaxLeaf = 16, kTaskThreshold = 1024;

struct Box { Vec lo, hi; };
inline Box empty_box() { return {{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}}; }
inline float lesser(float a, float b) { return (b < a) ? b : a; }
inline float greater(float a, float b) { return (a < b) ? b : a; }
inline void grow(Box& a, const Box& b) {
    a.lo = {lesser(a.lo.x, b.lo.x), lesser(a.lo.y, b.lo.y), lesser(a.lo.z, b.lo.z)};
    a.hi = {greater(a.hi.x, b.hi.x), greater(a.hi.y, b.hi.y), greater(a.hi.z, b.hi.z)};
}
inline float box_half_area(const Box& b) { Vec d = b.hi - b.lo; return (d.x + d.y) * d.z + d.x * d.y; }

struct SahBuild {
    RefNode* nodes;
    size_t* prim;
    const Box* boxes;
    const Vec* centers;
    std::atomic<size_t> node_count{1};

    static void store_box(RefNode& n, const Box& b) {
        n.bounds[0] = b.lo.x; n.bounds[1] = b.hi.x; n.bounds[2] = b.lo.y;
        n.bounds[3] = b.hi.y; n.bounds[4] = b.lo.z; n.bounds[5] = b.hi.z;
    }
    static Box load_box(const RefNode& n) {
        return {{n.bounds[0], n.bounds[2], n.bounds[4]}, {n.bounds[1], n.bounds[3], n.bounds[5]}};
    }

    struct Task { size_t node, begin, end, depth; };

    // split one node; returns false for a leaf
    bool split(const Task& t, Task& a, Task& b) {
        struct Bin { Box box; size_t count; float right; };
        Bin bins[3][kBins];
        RefNode& node = nodes[t.node];
        const size_t n = t.end - t.begin;
        auto make_leaf = [&] { node.first_child_or_primitive = uint32_t(t.begin); node.primitive_count = uint32_t(n); return false; };
        if (n <= 1 || t.depth >= kMaxDepth) return make_leaf();
        const Box bb = load_box(node);
        const Vec diag = bb.hi - bb.lo;
        const Vec c2b = scale(Vec{1.0f / diag.x, 1.0f / diag.y, 1.0f / diag.z}, float(kBins));
        const Vec off = {(-bb.lo.x) * c2b.x, (-bb.lo.y) * c2b.y, (-bb.lo.z) * c2b.z};
        auto bin_index = [&](const Vec& c, int axis) -> size_t {
            float f = std::fmaf(comp(c, axis), comp(c2b, axis), comp(off, axis));
            return std::min(kBins - 1, size_t(std::max(0.0f, f)));
        };
        for (auto& row : bins) for (auto& bin : row) { bin.box = empty_box(); bin.count = 0; bin.right = 0.f; }
        for (size_t i = t.begin; i < t.end; ++i) {
            const size_t p = prim[i];
            for (int axis = 0; axis < 3; ++axis) { Bin& bin = bins[axis][bin_index(centers[p], axis)]; bin.count++; grow(bin.box, boxes[p]); }
        }
        float best_cost[3]; size_t best_split[3];
        for (int axis = 0; axis < 3; ++axis) {
            Bin* row = bins[axis];
            Box acc = empty_box(); size_t cnt = 0;
            for (size_t i = kBins - 1; i > 0; --i) { grow(acc, row[i].box); cnt += row[i].count; row[i].right = box_half_area(acc) * cnt; }
            acc = empty_box(); cnt = 0;
            best_cost[axis] = FLT_MAX; best_split[axis] = kBins;
            for (size_t i = 0; i + 1 < kBins; ++i) {
                grow(acc, row[i].box); cnt += row[i].count;
                float cost = box_half_area(acc) * cnt + row[i + 1].right;
                if (cost < best_cost[axis]) { best_cost[axis] = cost; best_split[axis] = i + 1; }
            }
        }
        int axis = 0;
        if (best_cost[0] > best_cost[1]) axis = 1;
        if (best_cost[axis] > best_cost[2]) axis = 2;
        size_t split_at = best_split[axis];
        const float leaf_cost = box_half_area(bb) * (n - 1.0f);   // traversal_cost = 1
        if (best_split[axis] == kBins || best_cost[axis] >= leaf_cost) {
            if (n <= kMaxLeaf) return make_leaf();
            // largest_axis (bounding_box.hpp:53-59), then the 0.4 quantile of the bin counts
            axis = 0;
            if (diag.x < diag.y) axis = 1;
            if (comp(diag, axis) < diag.z) axis = 2;
            for (size_t i = 0, cnt = 0; i + 1 < kBins; ++i) {
                cnt += bins[axis][i].count;
                if (cnt >= (n * 2 / 5 + 1)) { split_at = i + 1; break; }
            }
        }
        size_t* mid = std::partition(prim + t.begin, prim + t.end,
                                     [&](size_t p) { return bin_index(centers[p], axis) < split_at; });
        const size_t m = size_t(mid - prim);
        if (m <= t.begin || m >= t.end) return make_leaf();
        const size_t child = node_count.fetch_add(2);
        node.first_child_or_primitive = uint32_t(child);
        node.primitive_count = 0;
        Box lb = empty_box(), rb = empty_box();
        for (size_t i = 0; i < best_split[axis]; ++i) grow(lb, bins[axis][i].box);
        for (size_t i = split_at; i < kBins; ++i) grow(rb, bins[axis][i].box);
        store_box(nodes[child], lb);
        store_box(nodes[child + 1], rb);
        a = {child, t.begin, m, t.depth + 1};
        b = {child + 1, m, t.end, t.depth + 1};
        return true;
    }

    void run(Task root) {
        std::vector<Task> stack{root};
        while (!stack.empty()) {
            Task t = stack.back(); stack.pop_back();
            Task a, b;
            if (!split(t, a, b)) continue;
            if (a.end - a.begin > b.end - b.begin) std::swap(a, b);
            stack.push_back(b);
            if (a.end - a.begin > kTaskThreshold) {
                #pragma omp task firstprivate(a)
                run(a);
            } else {
                stack.push_back(a);
            }
        }
    }
};

}  // namespace

// Re-lay the reference BVH (nodes32 + prim64) as depth-first SiblingPair records and the
// triangles in leaf order (DESIGN.md "Data layout in HBM"), validating ranges and cycles.
int relayout_bvh(const RefNode* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri48* tris,
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


// Shadow-ray BVH4: each record holds up to 4 boxes, obtained by collapsing a sibling pair's
// inner children into THEIR children (the grandchildren) when both grandchild boxes lie inside
// the child's box (exact float comparison).  The slab test is monotone in the box bounds, so
// with containment a grandchild box passing implies its parent box passing, and an any-hit
// traversal of the BVH4 tests exactly the triangles of the leaves whose own boxes pass -- the
// same set, with the same per-triangle arithmetic, as the BVH2 traversal of
// single_ray_traverser.hpp:68-126 with tmax fixed at FLT_MAX (any-hit never lowers it before
// it returns).  A child whose grandchildren are not contained (e.g. a box quirk of the builder's
// quantile fallback) stays an entry of its own, so the equivalence holds unconditionally.
// stack_bound: the most entries the traversal can ever hold (pushes along any root-leaf path).
int build_shadow_bvh4(const std::vector<SiblingPair>& pairs, std::vector<Node4>& out, uint32_t& stack_bound,
                      uint32_t& not_collapsed) {
    struct Entry { const float* box; uint32_t count, first; };   // count 0: first = pair index
    auto inside = [](const float* c, const float* p) {
        return c[0] >= p[0] && c[1] <= p[1] && c[2] >= p[2] && c[3] <= p[3] && c[4] >= p[4] && c[5] <= p[5];
    };
    out.clear();
    out.reserve(pairs.size() / 2 + 1);
    stack_bound = 0;
    not_collapsed = 0;
    struct Item { uint32_t pair, node4, acc; };
    std::vector<Item> st;
    out.emplace_back();
    st.push_back({0, 0, 0});
    while (!st.empty()) {
        const Item it = st.back(); st.pop_back();
        const SiblingPair& P = pairs[it.pair];
        Entry ents[4];
        int n = 0;
        const float* side_box[2] = {P.lb, P.rb};
        const uint32_t side_cnt[2] = {P.lcount, P.rcount}, side_first[2] = {P.lfirst, P.rfirst};
        for (int k = 0; k < 2; ++k) {
            if (side_cnt[k]) { ents[n++] = {side_box[k], side_cnt[k], side_first[k]}; continue; }
            const SiblingPair& Q = pairs[side_first[k]];
            if (inside(Q.lb, side_box[k]) && inside(Q.rb, side_box[k])) {
                ents[n++] = {Q.lb, Q.lcount, Q.lfirst};
                ents[n++] = {Q.rb, Q.rcount, Q.rfirst};
            } else {
                ents[n++] = {side_box[k], 0, side_first[k]};
                ++not_collapsed;
            }
        }
        int inner = 0;
        for (int c = 0; c < n; ++c) inner += ents[c].count == 0;
        const uint32_t acc = it.acc + uint32_t(std::max(0, inner - 1));
        stack_bound = std::max(stack_bound, acc);
        Node4 rec{};
        for (int c = 0; c < 4; ++c) {
            if (c >= n) { rec.count[c] = kNode4Empty; rec.first[c] = 0; continue; }
            rec.lo_x[c] = ents[c].box[0]; rec.hi_x[c] = ents[c].box[1];
            rec.lo_y[c] = ents[c].box[2]; rec.hi_y[c] = ents[c].box[3];
            rec.lo_z[c] = ents[c].box[4]; rec.hi_z[c] = ents[c].box[5];
            rec.count[c] = ents[c].count;
            if (ents[c].count) {
                rec.first[c] = ents[c].first;
            } else {
                rec.first[c] = uint32_t(out.size());
                out.emplace_back();
                st.push_back({ents[c].first, rec.first[c], acc});
            }
        }
        out[it.node4] = rec;
    }
    return CERES_OK;
}

}  // namespace ceres

using namespace ceres;

extern "C" {

void ceres_free(void* p) { std::free(p); }

int ceres_obj_load(const char* path, float** tri48, float** norm36, size_t* n_tri) {
    if (!path || !tri48 || !norm36 || !n_tri) return set_error(CERES_EINVAL, "ceres_obj_load: null argument");
    *tri48 = *norm36 = nullptr; *n_tri = 0;
    std::vector<char> buf;
    if (FILE* f = std::fopen(path, "rb")) {
        char chunk[1 << 16];
        size_t got;
        while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
        std::fclose(f);
    }   // unreadable file: empty mesh, like obj_norms.hpp:123-126
    MeshBuilder mb;
    int rc = parse_obj(buf.data(), buf.size(), mb);
    if (rc) return rc;
    return mb.finish(tri48, norm36, n_tri);
}

int ceres_proc_mesh(int n, float** tri48, float** norm36, size_t* n_tri) {
    if (n < 2 || !tri48 || !norm36 || !n_tri) return set_error(CERES_EINVAL, "ceres_proc_mesh: need n >= 2");
    MeshBuilder mb;
    const size_t nv = size_t(n) * size_t(n);
    mb.verts.reserve(nv); mb.vn.reserve(nv);
    mb.tris.reserve(2 * size_t(n - 1) * size_t(n - 1));
    mb.corner.reserve(6 * size_t(n - 1) * size_t(n - 1));
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double x = double(i) / double(n - 1), y = double(j) / double(n - 1);
            double z = 0.05 * (std::sin(40.0 * x) + std::cos(37.0 * y)) + 0.01 * std::sin(400.0 * x + 300.0 * y);
            mb.add_vertex({float(x), float(y), float(z)});
        }
    for (int j = 0; j + 1 < n; ++j)
        for (int i = 0; i + 1 < n; ++i) {
            size_t a = size_t(j) * n + i, b = a + 1, c = a + n + 1, d = a + n;
            mb.add_triangle(a, b, c);
            mb.add_triangle(a, c, d);
        }
    return mb.finish(tri48, norm36, n_tri);
}

int ceres_rotate_triangles(float* tri48, size_t n_tri, int axis, float degrees) {
    if ((!tri48 && n_tri) || axis < 0 || axis > 2) return set_error(CERES_EINVAL, "ceres_rotate_triangles: bad argument");
    const float pi = float(3.14159265359);
    const float c = std::cos(degrees * pi / float(180));
    const float s = std::sin(degrees * pi / float(180));
    auto rot = [&](Vec p) -> Vec {
        if (axis == 0) return {p.x, p.y * c - p.z * s, p.y * s + p.z * c};
        if (axis == 1) return {p.x * c + p.z * s, p.y, -p.x * s + p.z * c};
        return {p.x * c - p.y * s, p.x * s + p.y * c, p.z};
    };
    Tri48* t = reinterpret_cast<Tri48*>(tri48);
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n_tri; ++i) {
        const Vec p0 = P0(t[i]), p1 = P0(t[i]) - E1(t[i]), p2 = P0(t[i]) + E2(t[i]);   // p1(), p2()
        t[i] = tri_from_points(rot(p0), rot(p1), rot(p2));
    }
    return CERES_OK;
}

int ceres_bvh_build(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64) {
    if (!tri48 || !nodes32 || !n_nodes || !prim64) return set_error(CERES_EINVAL, "ceres_bvh_build: null argument");
    if (n_tri == 0) return set_error(CERES_EINVAL, "The given scene is empty or cannot be loaded");
    if (n_tri > 0x7fffffffu) return set_error(CERES_EUNSUPPORTED, "more than 2^31 triangles");
    const Tri48* t = reinterpret_cast<const Tri48*>(tri48);
    std::vector<Box> boxes(n_tri);
    std::vector<Vec> centers(n_tri);
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n_tri; ++i) {                   // Triangle::bounding_box / center, triangle.hpp:39-48
        const Vec p0 = P0(t[i]), p1 = P0(t[i]) - E1(t[i]), p2 = P0(t[i]) + E2(t[i]);
        Box b{p0, p0};
        grow(b, Box{p1, p1});
        grow(b, Box{p2, p2});
        boxes[i] = b;
        centers[i] = scale(p0 + p1 + p2, float(1.0) / float(3.0));
    }
    Box global = empty_box();
    for (size_t i = 0; i < n_tri; ++i) grow(global, boxes[i]);
    std::vector<RefNode> nodes(2 * n_tri + 1);
    std::vector<size_t> prim(n_tri);
    for (size_t i = 0; i < n_tri; ++i) prim[i] = i;
    SahBuild sb;
    sb.nodes = nodes.data(); sb.prim = prim.data(); sb.boxes = boxes.data(); sb.centers = centers.data();
    SahBuild::store_box(nodes[0], global);
    #pragma omp parallel
    #pragma omp single
    sb.run({0, 0, n_tri, 0});
    const size_t m = sb.node_count.load();
    *n_nodes = m;
    *nodes32 = static_cast<uint32_t*>(std::malloc(m * sizeof(RefNode)));
    *prim64 = static_cast<uint64_t*>(std::malloc(n_tri * 8));
    if (!*nodes32 || !*prim64) { std::free(*nodes32); std::free(*prim64); return set_error(CERES_ENOMEM, "out of host memory"); }
    std::memcpy(*nodes32, nodes.data(), m * sizeof(RefNode));
    for (size_t i = 0; i < n_tri; ++i) (*prim64)[i] = prim[i];
    return CERES_OK;
}

int ceres_camera_basis(const float eye[3], const float dir[3], const float up[3], float fov_deg,
                       size_t width, size_t height, float out9[9]) {
    (void)eye;
    if (!dir || !up || !out9 || !width || !height) return set_error(CERES_EINVAL, "ceres_camera_basis: bad argument");
    const Vec d = vnormalize({dir[0], dir[1], dir[2]});
    Vec u = vnormalize(vcross(d, {up[0], up[1], up[2]}));
    Vec v = vnormalize(vcross(u, d));
    const float w = std::tan(fov_deg * float(3.14159265 * (1.0 / 180.0) * 0.5));
    const float ratio = float(height) / float(width);
    u = scale(u, w);
    v = scale(scale(v, w), ratio);
    const float o[9] = {d.x, d.y, d.z, u.x, u.y, u.z, v.x, v.y, v.z};
    std::memcpy(out9, o, sizeof o);
    return CERES_OK;
}

// The orbit of anim.cpp:76-88: t = Transform<float>().rotate(axis, step / 180 * pi)
// (transform.hpp:67-104, Markley-Crassidis matrix composed onto the identity) applied to the
// camera eye, camera dir and sun once per frame; `up` is not rotated.  rotate_first = 1 is
// anim.cpp's order (rotate, then render); 0 renders frame 0 at the start pose.
int ceres_orbit_cameras(const float eye[3], const float dir[3], const float up[3], const float sun[3], float fov_deg,
                        size_t width, size_t height, const float axis[3], float step_deg, uint32_t n_frames,
                        int rotate_first, float* basis12, float* sun3, float* dir3) {
    if (!eye || !dir || !up || !sun || !axis || !basis12 || !sun3 || !width || !height)
        return set_error(CERES_EINVAL, "ceres_orbit_cameras: bad argument");
    const float pi = float(3.14159265359);
    const float angle = step_deg / 180.0f * pi;
    const Vec n = vnormalize({axis[0], axis[1], axis[2]});
    const float s = std::sin(angle), c = std::cos(angle);
    const float m[3][3] = {
        {c + (1 - c) * n.x * n.x, (1 - c) * n.x * n.y + s * n.z, (1 - c) * n.x * n.z - s * n.y},
        {(1 - c) * n.y * n.x - s * n.z, c + (1 - c) * n.y * n.y, (1 - c) * n.y * n.z + s * n.x},
        {(1 - c) * n.z * n.x + s * n.y, (1 - c) * n.z * n.y - s * n.x, c + (1 - c) * n.z * n.z}};
    float a[3][3];                                          // identity * m, summed like transform.hpp:96-102
    const float id[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int r = 0; r < 3; ++r)
        for (int col = 0; col < 3; ++col) {
            float acc = 0;
            for (int i = 0; i < 3; ++i) acc += id[r][i] * m[i][col];
            a[r][col] = acc;
        }
    auto apply = [&](Vec p) -> Vec {                        // operator(), transform.hpp:106-112 (v = 0)
        return {a[0][0] * p.x + a[0][1] * p.y + a[0][2] * p.z + 0.0f,
                a[1][0] * p.x + a[1][1] * p.y + a[1][2] * p.z + 0.0f,
                a[2][0] * p.x + a[2][1] * p.y + a[2][2] * p.z + 0.0f};
    };
    Vec e{eye[0], eye[1], eye[2]}, d{dir[0], dir[1], dir[2]}, l{sun[0], sun[1], sun[2]};
    for (uint32_t f = 0; f < n_frames; ++f) {
        if (rotate_first || f > 0) { e = apply(e); d = apply(d); l = apply(l); }
        const float ev[3] = {e.x, e.y, e.z}, dv[3] = {d.x, d.y, d.z};
        basis12[12 * f] = e.x; basis12[12 * f + 1] = e.y; basis12[12 * f + 2] = e.z;
        if (int rc = ceres_camera_basis(ev, dv, up, fov_deg, width, height, basis12 + 12 * f + 3)) return rc;
        sun3[3 * f] = l.x; sun3[3 * f + 1] = l.y; sun3[3 * f + 2] = l.z;
        if (dir3) { dir3[3 * f] = d.x; dir3[3 * f + 1] = d.y; dir3[3 * f + 2] = d.z; }
    }
    return CERES_OK;
}

}  // extern "C"
