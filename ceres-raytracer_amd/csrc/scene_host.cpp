// scene_host.cpp -- host-side scene preparation of the CERES hot path (product code).
//
// What the reference's callers run before render() (static.cpp:76-107, anim.cpp:38-65):
// OBJ parsing with vertex normals (obj_norms.hpp:57-127), rotate_triangles (render.hpp:24-44),
// the camera basis (render.hpp:91-97) and the binned-SAH BVH (binned_sah_builder.hpp:39-234).
// These stay on the host, as in the north star; they produce the exact bits the gfx950
// kernels consume, so every float operation follows the reference's order (the library is
// compiled with -ffp-contract=off; the reference's explicit fmaf stays an fmaf).  Every step
// comes in two arithmetic flavours (template G, CERES_ARITH_*): G = false is the reference
// without contraction, G = true the reference as its own CMake build (g++ -O3 -mfma) compiles it,
// an explicit fma at exactly the sites where GCC contracts (oracle/contraction_sites.txt).
#include <algorithm>
#include <array>
#include <atomic>
#include <cctype>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
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

// Scalar-generic vector (S = float: render<float>, static.cpp; S = double: render<double>,
// anim.cpp -d).  Every operation keeps the reference's order (vector.hpp:136-153).
template <class S> struct V3 { S x, y, z; };
template <class S> inline S comp(const V3<S>& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
template <class S> inline V3<S> operator+(V3<S> a, V3<S> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class S> inline V3<S> operator-(V3<S> a, V3<S> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class S> inline V3<S> scale(V3<S> a, S s) { return {a.x * s, a.y * s, a.z * s}; }
template <class S> inline S vdot(V3<S> a, V3<S> b) { S s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
template <class S> inline V3<S> vcross(V3<S> a, V3<S> b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
template <class S> inline V3<S> vnormalize(V3<S> v) { S inv = S(1) / std::sqrt(vdot(v, v)); return scale(v, inv); }
// GCC-contracted forms: dot -> fma(a2,b2, fma(a0,b0, a1 b1)); cross a_j b_k - a_k b_j ->
// fma(a_j, b_k, -(a_k b_j)) (vector.hpp:134-167 as the reference's build fuses them)
template <bool G, class S> inline S gdot(V3<S> a, V3<S> b) {
    if constexpr (G) return std::fma(a.z, b.z, std::fma(a.x, b.x, a.y * b.y));
    else return vdot(a, b);
}
template <bool G, class S> inline V3<S> gcross(V3<S> a, V3<S> b) {
    if constexpr (G) return {std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)), std::fma(a.x, b.y, -(a.y * b.x))};
    else return vcross(a, b);
}
template <bool G, class S> inline V3<S> gnormalize(V3<S> v) { S inv = S(1) / std::sqrt(gdot<G>(v, v)); return scale(v, inv); }
// a * b + c * d (sub: a * b - c * d) with GCC's fusion of the first product
template <bool G, class S> inline S gmad2(S a, S b, S c, S d, bool sub) {
    if constexpr (G) return std::fma(a, b, sub ? -(c * d) : c * d);
    else return sub ? a * b - c * d : a * b + c * d;
}
using Vec = V3<float>;

template <class S> struct TriT { S p0[3], e1[3], e2[3], n[3]; };     // bvh::Triangle<S>
static_assert(sizeof(TriT<float>) == sizeof(Tri48), "Tri48");
template <class S> struct NodeT;                                     // bvh::Bvh<S>::Node (bvh.hpp:25-30)
template <> struct NodeT<float> { float bounds[6]; uint32_t primitive_count, first_child_or_primitive; };
template <> struct NodeT<double> { double bounds[6]; uint64_t primitive_count, first_child_or_primitive; };
static_assert(sizeof(NodeT<float>) == 32 && sizeof(NodeT<double>) == 64, "Node");

template <bool G, class S> inline TriT<S> tri_from_points(V3<S> p0, V3<S> p1, V3<S> p2) {   // Triangle ctor, triangle.hpp:30-34
    V3<S> e1 = p0 - p1, e2 = p2 - p0, n = gcross<G>(e1, e2);
    return TriT<S>{{p0.x, p0.y, p0.z}, {e1.x, e1.y, e1.z}, {e2.x, e2.y, e2.z}, {n.x, n.y, n.z}};
}
template <class S> inline V3<S> P0(const TriT<S>& t) { return {t.p0[0], t.p0[1], t.p0[2]}; }
template <class S> inline V3<S> E1(const TriT<S>& t) { return {t.e1[0], t.e1[1], t.e1[2]}; }
template <class S> inline V3<S> E2(const TriT<S>& t) { return {t.e2[0], t.e2[1], t.e2[2]}; }
template <class S> inline V3<S> N(const TriT<S>& t) { return {t.n[0], t.n[1], t.n[2]}; }

// ------------------------------------------------------------------ mesh assembly
// Accumulates fan-triangulated faces and area-weighted (un-normalised, left-handed) face
// normals per vertex in face order, exactly like obj_norms.hpp:84-115.  Vertex coordinates
// are floats from strtof (obj_norms.hpp:78-80), widened for S = double.
template <class S, bool G>
struct MeshBuilder {
    std::vector<V3<S>> verts, vn;
    std::vector<TriT<S>> tris;
    std::vector<uint32_t> corner;     // 3 vertex ids per triangle

    void add_vertex(V3<S> v) { verts.push_back(v); vn.push_back({S(0), S(0), S(0)}); }
    void add_triangle(size_t a, size_t b, size_t c) {
        tris.push_back(tri_from_points<G>(verts[a], verts[b], verts[c]));
        V3<S> n = N(tris.back());
        vn[a] = vn[a] + n; vn[b] = vn[b] + n; vn[c] = vn[c] + n;
        corner.push_back(uint32_t(a)); corner.push_back(uint32_t(b)); corner.push_back(uint32_t(c));
    }
    int finish(S** tri, S** norm, size_t* n_tri) {
        for (auto& n : vn) n = gnormalize<G>(n);             // obj_norms.hpp:109-111
        const size_t nt = tris.size();
        *n_tri = nt;
        *tri = static_cast<S*>(std::malloc(std::max<size_t>(1, nt * sizeof(TriT<S>))));
        *norm = static_cast<S*>(std::malloc(std::max<size_t>(1, nt * 9 * sizeof(S))));
        if (!*tri || !*norm) { std::free(*tri); std::free(*norm); *tri = *norm = nullptr; return set_error(CERES_ENOMEM, "out of host memory"); }
        if (nt) std::memcpy(*tri, tris.data(), nt * sizeof(TriT<S>));   // (an empty mesh has no data())
        S* o = *norm;
        for (size_t t = 0; t < nt; ++t)
            for (int k = 0; k < 3; ++k) {
                const V3<S>& v = vn[corner[3 * t + k]];
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

template <class S, bool G>
int parse_obj(const char* data, size_t len, MeshBuilder<S, G>& mb) {
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
            mb.add_vertex({S(x), S(y), S(z)});
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

template <class S, bool G = false>
int obj_load(const char* path, S** tri, S** norm, size_t* n_tri) {
    if (!path || !tri || !norm || !n_tri) return set_error(CERES_EINVAL, "ceres_obj_load: null argument");
    *tri = *norm = nullptr; *n_tri = 0;
    std::vector<char> buf;
    if (FILE* f = std::fopen(path, "rb")) {
        char chunk[1 << 16];
        size_t got;
        while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
        std::fclose(f);
    }   // unreadable file: empty mesh, like obj_norms.hpp:123-126
    MeshBuilder<S, G> mb;
    int rc = parse_obj(buf.data(), buf.size(), mb);
    if (rc) return rc;
    return mb.finish(tri, norm, n_tri);
}

template <class S, bool G = false>
int proc_mesh(int n, S** tri, S** norm, size_t* n_tri) {
    if (n < 2 || !tri || !norm || !n_tri) return set_error(CERES_EINVAL, "ceres_proc_mesh: need n >= 2");
    MeshBuilder<S, G> mb;
    const size_t nv = size_t(n) * size_t(n);
    mb.verts.reserve(nv); mb.vn.reserve(nv);
    mb.tris.reserve(2 * size_t(n - 1) * size_t(n - 1));
    mb.corner.reserve(6 * size_t(n - 1) * size_t(n - 1));
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double x = double(i) / double(n - 1), y = double(j) / double(n - 1);
            double z = 0.05 * (std::sin(40.0 * x) + std::cos(37.0 * y)) + 0.01 * std::sin(400.0 * x + 300.0 * y);
            mb.add_vertex({S(float(x)), S(float(y)), S(float(z))});   // the OBJ-text values (%.9g floats)
        }
    for (int j = 0; j + 1 < n; ++j)
        for (int i = 0; i + 1 < n; ++i) {
            size_t a = size_t(j) * n + i, b = a + 1, c = a + n + 1, d = a + n;
            mb.add_triangle(a, b, c);
            mb.add_triangle(a, c, d);
        }
    return mb.finish(tri, norm, n_tri);
}

template <class S, bool G = false>
int rotate_triangles(S* tri, size_t n_tri, int axis, S degrees) {         // render.hpp:24-44
    if ((!tri && n_tri) || axis < 0 || axis > 2) return set_error(CERES_EINVAL, "ceres_rotate_triangles: bad argument");
    const S pi = S(3.14159265359);
    const S c = std::cos(degrees * pi / S(180));
    const S s = std::sin(degrees * pi / S(180));
    auto rot = [&](V3<S> p) -> V3<S> {                      // (GCC fuses each coordinate's first product)
        if (axis == 0) return {p.x, gmad2<G>(p.y, c, p.z, s, true), gmad2<G>(p.y, s, p.z, c, false)};
        if (axis == 1) return {gmad2<G>(p.x, c, p.z, s, false), p.y, gmad2<G>(-p.x, s, p.z, c, false)};
        return {gmad2<G>(p.x, c, p.y, s, true), gmad2<G>(p.x, s, p.y, c, false), p.z};
    };
    TriT<S>* t = reinterpret_cast<TriT<S>*>(tri);
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n_tri; ++i) {
        const V3<S> p0 = P0(t[i]), p1 = P0(t[i]) - E1(t[i]), p2 = P0(t[i]) + E2(t[i]);   // p1(), p2()
        t[i] = tri_from_points<G>(rot(p0), rot(p1), rot(p2));
    }
    return CERES_OK;
}

// ------------------------------------------------------------------ binned SAH BVH
// Same split rules as BinnedSahBuilder<Bvh,16> so the topology (and leaf order) is the
// reference's: 16 bins per axis on centroids (bin index by fma, :144-147), SAH sweeps
// (:89-114), axis choice (:170-174), leaf test with traversal_cost 1 (:179), 0.4-quantile
// fallback above 16 primitives (:180-196), std::partition (:199-201), child boxes from the
// bins (:216-224, including its use of the pre-fallback split count for the left box).
// Subtrees above 1024 primitives become OpenMP tasks (top_down_builder.hpp:63-66).
constexpr size_t kBins = 16, kMaxDepth = 64, kMaxLeaf = 16, kTaskThreshold = 1024;

template <class S> struct BoxT { V3<S> lo, hi; };
template <class S> inline BoxT<S> empty_box() {
    const S m = std::numeric_limits<S>::max();
    return {{m, m, m}, {-m, -m, -m}};
}
template <class S> inline S lesser(S a, S b) { return (b < a) ? b : a; }
template <class S> inline S greater(S a, S b) { return (a < b) ? b : a; }
template <class S> inline void grow(BoxT<S>& a, const BoxT<S>& b) {
    a.lo = {lesser(a.lo.x, b.lo.x), lesser(a.lo.y, b.lo.y), lesser(a.lo.z, b.lo.z)};
    a.hi = {greater(a.hi.x, b.hi.x), greater(a.hi.y, b.hi.y), greater(a.hi.z, b.hi.z)};
}
template <class S> inline S box_half_area(const BoxT<S>& b) { V3<S> d = b.hi - b.lo; return (d.x + d.y) * d.z + d.x * d.y; }
// GCC fuses half_area's FIRST product in find_split's sweeps (binned_sah_builder.hpp:98,109) and
// its SECOND in the node's max_split_cost (:179); the sweep's cost is fma(count, ha, right_cost)
template <bool G, class S> inline S half_area_sweep(const BoxT<S>& b) {
    V3<S> d = b.hi - b.lo;
    if constexpr (G) return std::fma(d.x + d.y, d.z, d.x * d.y);
    else return (d.x + d.y) * d.z + d.x * d.y;
}
template <bool G, class S> inline S half_area_node(const BoxT<S>& b) {
    V3<S> d = b.hi - b.lo;
    if constexpr (G) return std::fma(d.x, d.y, (d.x + d.y) * d.z);
    else return (d.x + d.y) * d.z + d.x * d.y;
}

template <class S, bool G>
struct SahBuild {
    using Node = NodeT<S>;
    using Box = BoxT<S>;
    using Vs = V3<S>;
    Node* nodes;
    size_t* prim;
    const Box* boxes;
    const Vs* centers;
    std::atomic<size_t> node_count{1};

    static void store_box(Node& n, const Box& b) {
        n.bounds[0] = b.lo.x; n.bounds[1] = b.hi.x; n.bounds[2] = b.lo.y;
        n.bounds[3] = b.hi.y; n.bounds[4] = b.lo.z; n.bounds[5] = b.hi.z;
    }
    static Box load_box(const Node& n) {
        return {{n.bounds[0], n.bounds[2], n.bounds[4]}, {n.bounds[1], n.bounds[3], n.bounds[5]}};
    }

    struct Task { size_t node, begin, end, depth; };

    // split one node; returns false for a leaf
    bool split(const Task& t, Task& a, Task& b) {
        struct Bin { Box box; size_t count; S right; };
        Bin bins[3][kBins];
        Node& node = nodes[t.node];
        const size_t n = t.end - t.begin;
        auto make_leaf = [&] { node.first_child_or_primitive = t.begin; node.primitive_count = n; return false; };
        if (n <= 1 || t.depth >= kMaxDepth) return make_leaf();
        const Box bb = load_box(node);
        const Vs diag = bb.hi - bb.lo;
        const Vs c2b = scale(Vs{S(1) / diag.x, S(1) / diag.y, S(1) / diag.z}, S(kBins));
        const Vs off = {(-bb.lo.x) * c2b.x, (-bb.lo.y) * c2b.y, (-bb.lo.z) * c2b.z};
        auto bin_index = [&](const Vs& c, int axis) -> size_t {
            S f = std::fma(comp(c, axis), comp(c2b, axis), comp(off, axis));
            return std::min(kBins - 1, size_t(std::max(S(0), f)));
        };
        for (auto& row : bins) for (auto& bin : row) { bin.box = empty_box<S>(); bin.count = 0; bin.right = S(0); }
        for (size_t i = t.begin; i < t.end; ++i) {
            const size_t p = prim[i];
            for (int axis = 0; axis < 3; ++axis) { Bin& bin = bins[axis][bin_index(centers[p], axis)]; bin.count++; grow(bin.box, boxes[p]); }
        }
        S best_cost[3]; size_t best_split[3];
        for (int axis = 0; axis < 3; ++axis) {
            Bin* row = bins[axis];
            Box acc = empty_box<S>(); size_t cnt = 0;
            for (size_t i = kBins - 1; i > 0; --i) { grow(acc, row[i].box); cnt += row[i].count; row[i].right = half_area_sweep<G>(acc) * S(cnt); }
            acc = empty_box<S>(); cnt = 0;
            best_cost[axis] = std::numeric_limits<S>::max(); best_split[axis] = kBins;
            for (size_t i = 0; i + 1 < kBins; ++i) {
                grow(acc, row[i].box); cnt += row[i].count;
                S cost = G ? std::fma(S(cnt), half_area_sweep<G>(acc), row[i + 1].right) : box_half_area(acc) * S(cnt) + row[i + 1].right;
                if (cost < best_cost[axis]) { best_cost[axis] = cost; best_split[axis] = i + 1; }
            }
        }
        int axis = 0;
        if (best_cost[0] > best_cost[1]) axis = 1;
        if (best_cost[axis] > best_cost[2]) axis = 2;
        size_t split_at = best_split[axis];
        const S leaf_cost = half_area_node<G>(bb) * (S(n) - S(1));   // traversal_cost = 1
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
        node.first_child_or_primitive = child;
        node.primitive_count = 0;
        Box lb = empty_box<S>(), rb = empty_box<S>();
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

template <class S, bool G = false>
int bvh_build(const S* tri, size_t n_tri, NodeT<S>** nodes_out, size_t* n_nodes, uint64_t** prim64) {
    if (!tri || !nodes_out || !n_nodes || !prim64) return set_error(CERES_EINVAL, "ceres_bvh_build: null argument");
    if (n_tri == 0) return set_error(CERES_EINVAL, "The given scene is empty or cannot be loaded");
    if (n_tri > 0x7fffffffu) return set_error(CERES_EUNSUPPORTED, "more than 2^31 triangles");
    const TriT<S>* t = reinterpret_cast<const TriT<S>*>(tri);
    std::vector<BoxT<S>> boxes(n_tri);
    std::vector<V3<S>> centers(n_tri);
    #pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n_tri; ++i) {                   // Triangle::bounding_box / center, triangle.hpp:39-48
        const V3<S> p0 = P0(t[i]), p1 = P0(t[i]) - E1(t[i]), p2 = P0(t[i]) + E2(t[i]);
        BoxT<S> b{p0, p0};
        grow(b, BoxT<S>{p1, p1});
        grow(b, BoxT<S>{p2, p2});
        boxes[i] = b;
        centers[i] = scale(p0 + p1 + p2, S(1.0) / S(3.0));
    }
    BoxT<S> global = empty_box<S>();
    for (size_t i = 0; i < n_tri; ++i) grow(global, boxes[i]);
    std::vector<NodeT<S>> nodes(2 * n_tri + 1);
    std::vector<size_t> prim(n_tri);
    for (size_t i = 0; i < n_tri; ++i) prim[i] = i;
    SahBuild<S, G> sb;
    sb.nodes = nodes.data(); sb.prim = prim.data(); sb.boxes = boxes.data(); sb.centers = centers.data();
    SahBuild<S, G>::store_box(nodes[0], global);
    #pragma omp parallel
    #pragma omp single
    sb.run({0, 0, n_tri, 0});
    const size_t m = sb.node_count.load();
    *n_nodes = m;
    *nodes_out = static_cast<NodeT<S>*>(std::malloc(m * sizeof(NodeT<S>)));
    *prim64 = static_cast<uint64_t*>(std::malloc(n_tri * 8));
    if (!*nodes_out || !*prim64) { std::free(*nodes_out); std::free(*prim64); return set_error(CERES_ENOMEM, "out of host memory"); }
    std::memcpy(*nodes_out, nodes.data(), m * sizeof(NodeT<S>));
    for (size_t i = 0; i < n_tri; ++i) (*prim64)[i] = prim[i];
    return CERES_OK;
}

// render.hpp:91-97 (the basis; eye is passed through by the callers)
template <class S, bool G = false>
int camera_basis(const S dir[3], const S up[3], S fov_deg, size_t width, size_t height, S out9[9]) {
    if (!dir || !up || !out9 || !width || !height) return set_error(CERES_EINVAL, "ceres_camera_basis: bad argument");
    const V3<S> d = gnormalize<G>(V3<S>{dir[0], dir[1], dir[2]});
    V3<S> u = gnormalize<G>(gcross<G>(d, V3<S>{up[0], up[1], up[2]}));
    V3<S> v = gnormalize<G>(gcross<G>(u, d));
    const S w = std::tan(fov_deg * S(3.14159265 * (1.0 / 180.0) * 0.5));
    const S ratio = S(height) / S(width);
    u = scale(u, w);
    v = scale(scale(v, w), ratio);
    const S o[9] = {d.x, d.y, d.z, u.x, u.y, u.z, v.x, v.y, v.z};
    std::memcpy(out9, o, sizeof o);
    return CERES_OK;
}

// The orbit of anim.cpp:76-88: t = Transform<S>().rotate(axis, step / 180 * pi)
// (transform.hpp:67-104, Markley-Crassidis matrix composed onto the identity) applied to the
// camera eye, camera dir and sun once per frame; `up` is not rotated.
template <class S, bool G = false>
int orbit_cameras(const S eye[3], const S dir[3], const S up[3], const S sun[3], S fov_deg, size_t width, size_t height,
                  const S axis[3], S step_deg, uint32_t n_frames, int rotate_first, S* basis12, S* sun3, S* dir3) {
    if (!eye || !dir || !up || !sun || !axis || !basis12 || !sun3 || !width || !height)
        return set_error(CERES_EINVAL, "ceres_orbit_cameras: bad argument");
    const S pi = S(3.14159265359);
    const S angle = step_deg / 180.0f * pi;                  // anim.cpp:77, a float literal 180
    const V3<S> n = gnormalize<G>(V3<S>{axis[0], axis[1], axis[2]});
    const S s = std::sin(angle), c = std::cos(angle);
    // transform.hpp:80-96; GCC fuses every entry's outer (1-c) n_r * n_k product
    auto ent = [&](S nr, S nk, S add, bool sub) -> S {       // (1-c) nr nk +/- add
        const S cr = (1 - c) * nr;
        if constexpr (G) return std::fma(cr, nk, sub ? -add : add);
        else return sub ? cr * nk - add : cr * nk + add;
    };
    auto diag = [&](S nr) -> S {                             // c + (1-c) nr nr
        const S cr = (1 - c) * nr;
        if constexpr (G) return std::fma(cr, nr, c);
        else return c + cr * nr;
    };
    const S m[3][3] = {
        {diag(n.x), ent(n.x, n.y, s * n.z, false), ent(n.x, n.z, s * n.y, true)},
        {ent(n.y, n.x, s * n.z, true), diag(n.y), ent(n.y, n.z, s * n.x, false)},
        {ent(n.z, n.x, s * n.y, false), ent(n.z, n.y, s * n.x, true), diag(n.z)}};
    S a[3][3];                                              // identity * m, summed like transform.hpp:96-102
    const S id[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int r = 0; r < 3; ++r)
        for (int col = 0; col < 3; ++col) {
            S acc = 0;
            for (int i = 0; i < 3; ++i) acc += id[r][i] * m[i][col];
            a[r][col] = acc;
        }
    auto apply = [&](V3<S> p) -> V3<S> {                    // operator(), transform.hpp:111-118 (v = 0)
        return {gdot<G>(V3<S>{a[0][0], a[0][1], a[0][2]}, p) + S(0),
                gdot<G>(V3<S>{a[1][0], a[1][1], a[1][2]}, p) + S(0),
                gdot<G>(V3<S>{a[2][0], a[2][1], a[2][2]}, p) + S(0)};
    };
    V3<S> e{eye[0], eye[1], eye[2]}, d{dir[0], dir[1], dir[2]}, l{sun[0], sun[1], sun[2]};
    for (uint32_t f = 0; f < n_frames; ++f) {
        if (rotate_first || f > 0) { e = apply(e); d = apply(d); l = apply(l); }
        const S dv[3] = {d.x, d.y, d.z};
        basis12[12 * f] = e.x; basis12[12 * f + 1] = e.y; basis12[12 * f + 2] = e.z;
        if (int rc = camera_basis<S, G>(dv, up, fov_deg, width, height, basis12 + 12 * f + 3)) return rc;
        sun3[3 * f] = l.x; sun3[3 * f + 1] = l.y; sun3[3 * f + 2] = l.z;
        if (dir3) { dir3[3 * f] = d.x; dir3[3 * f + 1] = d.y; dir3[3 * f + 2] = d.z; }
    }
    return CERES_OK;
}

}  // namespace

// Re-lay the reference BVH (nodes + prim64) as depth-first SiblingPair records and the
// triangles in leaf order (DESIGN.md "Data layout in HBM"), validating ranges and cycles.
// Node / Pair / Tri: float (RefNode, SiblingPair, Tri48) or double (RefNode64, SiblingPair64, Tri96).
template <class Node, class Pair, class Tri>
static int relayout_t(const Node* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri* tris,
                      std::vector<Pair>& pairs, std::vector<Tri>& leaf_tris, std::vector<uint32_t>& orig,
                      uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first) {
    leaf_tris.resize(n_tri);
    orig.resize(n_tri);
    for (size_t k = 0; k < n_tri; ++k) {
        if (prim[k] >= n_tri) return set_error(CERES_EINVAL, "primitive_indices[%zu] = %llu out of range", k, (unsigned long long)prim[k]);
        leaf_tris[k] = tris[prim[k]];
        orig[k] = uint32_t(prim[k]);
    }
    auto check_leaf = [&](const Node& n) -> bool {
        return uint64_t(n.first_child_or_primitive) + uint64_t(n.primitive_count) <= n_tri;
    };
    depth = 0;
    root_leaf_count = root_leaf_first = 0;
    if (nodes[0].primitive_count) {
        if (!check_leaf(nodes[0])) return set_error(CERES_EINVAL, "root leaf range out of bounds");
        root_leaf_count = uint32_t(nodes[0].primitive_count);
        root_leaf_first = uint32_t(nodes[0].first_child_or_primitive);
        pairs.assign(1, Pair{});
        return CERES_OK;
    }
    // pre-order DFS over inner nodes; each inner node's children become one record
    struct Item { uint64_t node; uint32_t pair, level; };
    pairs.clear();
    pairs.reserve(n_nodes / 2 + 1);
    std::vector<Item> st;
    if (uint64_t(nodes[0].first_child_or_primitive) + 1 >= n_nodes) return set_error(CERES_EINVAL, "root child index out of range");
    pairs.emplace_back();
    st.push_back({0, 0, 1});
    size_t visited = 0;
    while (!st.empty()) {
        const Item it = st.back(); st.pop_back();
        if (++visited > n_nodes) return set_error(CERES_EINVAL, "BVH has a cycle");
        const Node& n = nodes[it.node];
        const uint64_t c = n.first_child_or_primitive;
        depth = std::max(depth, it.level);
        Pair& rec = pairs[it.pair];
        std::memcpy(rec.lb, nodes[c].bounds, sizeof rec.lb);
        std::memcpy(rec.rb, nodes[c + 1].bounds, sizeof rec.rb);
        const Node* ch[2] = {&nodes[c], &nodes[c + 1]};
        uint32_t cnt[2], first[2];
        Item push[2]; int npush = 0;
        for (int k = 0; k < 2; ++k) {
            cnt[k] = uint32_t(ch[k]->primitive_count);
            if (ch[k]->primitive_count) {
                if (!check_leaf(*ch[k])) return set_error(CERES_EINVAL, "leaf range out of bounds");
                first[k] = uint32_t(ch[k]->first_child_or_primitive);
            } else {
                const uint64_t gc = ch[k]->first_child_or_primitive;
                if (gc + 1 >= n_nodes) return set_error(CERES_EINVAL, "child index out of range");
                first[k] = uint32_t(pairs.size());
                pairs.emplace_back();
                push[npush++] = {c + uint64_t(k), first[k], it.level + 1};
            }
        }
        Pair& r2 = pairs[it.pair];                                   // (emplace_back may have moved rec)
        r2.lcount = cnt[0]; r2.lfirst = first[0];
        r2.rcount = cnt[1]; r2.rfirst = first[1];
        for (int k = npush - 1; k >= 0; --k) st.push_back(push[k]);   // left subtree first
    }
    return CERES_OK;
}

int relayout_bvh(const RefNode* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri48* tris,
                 std::vector<SiblingPair>& pairs, std::vector<Tri48>& leaf_tris, std::vector<uint32_t>& orig,
                 uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first) {
    return relayout_t(nodes, n_nodes, prim, n_tri, tris, pairs, leaf_tris, orig, depth, root_leaf_count, root_leaf_first);
}

int relayout_bvh64(const RefNode64* nodes, size_t n_nodes, const uint64_t* prim, size_t n_tri, const Tri96* tris,
                   std::vector<SiblingPair64>& pairs, std::vector<Tri96>& leaf_tris, std::vector<uint32_t>& orig,
                   uint32_t& depth, uint32_t& root_leaf_count, uint32_t& root_leaf_first) {
    return relayout_t(nodes, n_nodes, prim, n_tri, tris, pairs, leaf_tris, orig, depth, root_leaf_count, root_leaf_first);
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
//
// A child word packs a leaf as (first << 5 | count), so a leaf holds at most 31 triangles.  The
// reference builder makes bigger leaves when no split separates the centroids (coincident
// triangles; binned_sah_builder.hpp:179-196 falls back, top_down_builder.hpp:36 caps the depth),
// so such a leaf becomes a "piece" node: an extra Node4 whose children are runs of <= 31 of the
// leaf's triangles (or further piece nodes), every one with the leaf's own box.  Equal boxes
// pass or fail together, so the triangles tested -- and the any-hit answer -- are unchanged.
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
    auto set_box = [](Node4& rec, int c, const float* b) {
        rec.lo_x[c] = b[0]; rec.hi_x[c] = b[1]; rec.lo_y[c] = b[2]; rec.hi_y[c] = b[3]; rec.lo_z[c] = b[4]; rec.hi_z[c] = b[5];
    };
    // an empty slot: kNode4Empty and the inverted infinite box (lo +inf, hi -inf), which every
    // octant-selected slab test fails (render_hip.hip packet_any4 tests no child word)
    auto set_empty = [](Node4& rec, int c) {
        rec.lo_x[c] = rec.lo_y[c] = rec.lo_z[c] = INFINITY;
        rec.hi_x[c] = rec.hi_y[c] = rec.hi_z[c] = -INFINITY;
        rec.child[c] = kNode4Empty;
    };
    // child word of a leaf of `count` triangles from slot `first` reached with `acc` stack entries
    // held above it; oversized leaves are split into piece nodes (recursively, 4 ways)
    std::function<int(const float*, uint32_t, uint32_t, uint32_t, uint32_t&)> leaf_word =
        [&](const float* box, uint32_t count, uint32_t first, uint32_t acc, uint32_t& word) -> int {
        if (first > kNode4MaxFirst) return set_error(CERES_EUNSUPPORTED, "shadow BVH4: leaf slot %u at or above 2^27", first);
        if (count <= kNode4MaxCount) { word = node4_child(count, first); return CERES_OK; }
        if (out.size() > kNode4MaxFirst) return set_error(CERES_EUNSUPPORTED, "shadow BVH4: more than 2^27 records");
        const uint32_t idx = uint32_t(out.size());
        out.emplace_back();
        const uint32_t parts = count <= 4 * kNode4MaxCount ? (count + kNode4MaxCount - 1) / kNode4MaxCount : 4;
        const uint32_t per = (count + parts - 1) / parts;
        const uint32_t inner = count <= 4 * kNode4MaxCount ? 0 : parts;      // pieces that are piece nodes again
        const uint32_t acc2 = acc + (inner > 1 ? inner - 1 : 0);
        stack_bound = std::max(stack_bound, acc2);
        Node4 rec{};
        for (uint32_t c = 0; c < 4; ++c) {
            const uint32_t lo = c * per, n = c < parts && lo < count ? std::min(per, count - lo) : 0;
            if (!n) { set_empty(rec, int(c)); continue; }
            set_box(rec, int(c), box);
            uint32_t w = 0;
            if (int rc = leaf_word(box, n, first + lo, acc2, w)) return rc;
            rec.child[c] = w;
        }
        node4_leaves_first(rec);
        out[idx] = rec;
        word = node4_child(0, idx);
        return CERES_OK;
    };
    struct Item { uint32_t pair, node4, acc; };
    std::vector<Item> st;
    out.emplace_back();
    st.push_back({0, 0, 0});
    size_t collapsed_records = 1;     // records made from sibling pairs (piece nodes excluded): a tree has at most one per pair
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
        for (int c = 0; c < n; ++c) inner += ents[c].count == 0 || ents[c].count > kNode4MaxCount;   // piece nodes are inner
        const uint32_t acc = it.acc + uint32_t(std::max(0, inner - 1));
        stack_bound = std::max(stack_bound, acc);
        Node4 rec{};
        for (int c = 0; c < 4; ++c) {
            if (c >= n) { set_empty(rec, c); continue; }
            set_box(rec, c, ents[c].box);
            if (ents[c].count) {
                uint32_t w = 0;
                if (int rc = leaf_word(ents[c].box, ents[c].count, ents[c].first, acc, w)) return rc;
                rec.child[c] = w;
            } else {
                if (collapsed_records >= pairs.size() || ents[c].first >= pairs.size())   // a tree has no more records than pairs
                    return set_error(CERES_EINVAL, "build_shadow_bvh4: sibling pairs do not form a tree");
                ++collapsed_records;
                if (out.size() > kNode4MaxFirst) return set_error(CERES_EUNSUPPORTED, "shadow BVH4: more than 2^27 records");
                const uint32_t idx = uint32_t(out.size());
                rec.child[c] = node4_child(0, idx);
                out.emplace_back();
                st.push_back({ents[c].first, idx, acc});
            }
        }
        node4_leaves_first(rec);
        out[it.node4] = rec;
    }
    return CERES_OK;
}

// Inner-child order of the shadow BVH4 for a small traversal stack.  The BVH4 walks that descend
// into the FIRST passing inner child and push the other passing ones in slot order (trace_any4,
// packet_any4, and the work-stealing loop when KParams::steal_first) pop the highest slot first,
// so a record's inner child in slot j (of k) starts with at most max(k-1-j, j-1) of the record's
// own entries below it: k-1-j when it is the first passing child (every later one pushed), j-1
// when it is pushed (every earlier one pushed before it).  need(r) = max_j (w_j + need(child_j))
// is then the exact worst case over every set of passing children, and putting the children with
// the largest need in the slots with the smallest weight minimises it (weights k=4: 3,2,1,2).
// The leaves-first layout is kept (inner slots nleaf..nleaf+k-1, empties after); children of a
// record always have larger indices (build_shadow_bvh4 appends them), so one backward sweep
// sees every child's need first.  Any-hit answers do not depend on the order.  C5: 37 -> 27
// entries (the nearest-first bound, `stack_bound` of build_shadow_bvh4, stays the sum over a path
// of k-1).
int order_shadow_bvh4(std::vector<Node4>& nodes, uint32_t& first_bound) {
    std::vector<uint32_t> need(nodes.size(), 0);
    for (size_t r = nodes.size(); r-- > 0;) {
        Node4& n = nodes[r];
        uint32_t slot[4], cneed[4], k = 0;
        for (uint32_t c = n.nleaf; c < 4; ++c) {
            const uint32_t w = n.child[c];
            if (w == kNode4Empty || (w & kNode4MaxCount)) break;
            const uint32_t ch = w >> kNode4CountBits;
            if (ch <= r || ch >= nodes.size()) return set_error(CERES_EINVAL, "shadow BVH4: child record %u of %zu", ch, r);
            slot[k] = c; cneed[k] = need[ch]; ++k;
        }
        if (!k) continue;
        uint32_t by_need[4] = {0, 1, 2, 3}, by_weight[4] = {0, 1, 2, 3}, wt[4];
        for (uint32_t j = 0; j < k; ++j) wt[j] = std::max<int>(int(k) - 1 - int(j), int(j) - 1);
        std::stable_sort(by_need, by_need + k, [&](uint32_t a, uint32_t b) { return cneed[a] > cneed[b]; });
        std::stable_sort(by_weight, by_weight + k, [&](uint32_t a, uint32_t b) { return wt[a] < wt[b]; });
        const Node4 old = n;
        uint32_t worst = 0;
        for (uint32_t i = 0; i < k; ++i) {
            const uint32_t from = slot[by_need[i]], to = slot[by_weight[i]];
            n.lo_x[to] = old.lo_x[from]; n.hi_x[to] = old.hi_x[from];
            n.lo_y[to] = old.lo_y[from]; n.hi_y[to] = old.hi_y[from];
            n.lo_z[to] = old.lo_z[from]; n.hi_z[to] = old.hi_z[from];
            n.child[to] = old.child[from];
            worst = std::max(worst, wt[by_weight[i]] + cneed[by_need[i]]);
        }
        need[r] = worst;
    }
    first_bound = nodes.empty() ? 0 : need[0];
    return CERES_OK;
}



}  // namespace ceres

using namespace ceres;

extern "C" {

void ceres_free(void* p) { std::free(p); }

int ceres_obj_load(const char* path, float** tri48, float** norm36, size_t* n_tri) { return obj_load<float>(path, tri48, norm36, n_tri); }
int ceres_obj_load_f64(const char* path, double** tri96, double** norm72, size_t* n_tri) { return obj_load<double>(path, tri96, norm72, n_tri); }
int ceres_proc_mesh(int n, float** tri48, float** norm36, size_t* n_tri) { return proc_mesh<float>(n, tri48, norm36, n_tri); }
int ceres_proc_mesh_f64(int n, double** tri96, double** norm72, size_t* n_tri) { return proc_mesh<double>(n, tri96, norm72, n_tri); }
int ceres_rotate_triangles(float* tri48, size_t n_tri, int axis, float degrees) { return rotate_triangles<float>(tri48, n_tri, axis, degrees); }
int ceres_rotate_triangles_f64(double* tri96, size_t n_tri, int axis, double degrees) { return rotate_triangles<double>(tri96, n_tri, axis, degrees); }

int ceres_bvh_build(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64) {
    if (!nodes32) return set_error(CERES_EINVAL, "ceres_bvh_build: null argument");
    NodeT<float>* nodes = nullptr;
    const int rc = bvh_build<float>(tri48, n_tri, &nodes, n_nodes, prim64);
    *nodes32 = reinterpret_cast<uint32_t*>(nodes);
    return rc;
}
int ceres_bvh_build_f64(const double* tri96, size_t n_tri, uint64_t** nodes64, size_t* n_nodes, uint64_t** prim64) {
    if (!nodes64) return set_error(CERES_EINVAL, "ceres_bvh_build_f64: null argument");
    NodeT<double>* nodes = nullptr;
    const int rc = bvh_build<double>(tri96, n_tri, &nodes, n_nodes, prim64);
    *nodes64 = reinterpret_cast<uint64_t*>(nodes);
    return rc;
}

int ceres_camera_basis(const float eye[3], const float dir[3], const float up[3], float fov_deg,
                       size_t width, size_t height, float out9[9]) {
    (void)eye;
    return camera_basis<float>(dir, up, fov_deg, width, height, out9);
}
int ceres_camera_basis_f64(const double eye[3], const double dir[3], const double up[3], double fov_deg,
                           size_t width, size_t height, double out9[9]) {
    (void)eye;
    return camera_basis<double>(dir, up, fov_deg, width, height, out9);
}

int ceres_orbit_cameras(const float eye[3], const float dir[3], const float up[3], const float sun[3], float fov_deg,
                        size_t width, size_t height, const float axis[3], float step_deg, uint32_t n_frames,
                        int rotate_first, float* basis12, float* sun3, float* dir3) {
    return orbit_cameras<float>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames, rotate_first,
                                basis12, sun3, dir3);
}
int ceres_orbit_cameras_f64(const double eye[3], const double dir[3], const double up[3], const double sun[3],
                            double fov_deg, size_t width, size_t height, const double axis[3], double step_deg,
                            uint32_t n_frames, int rotate_first, double* basis12, double* sun3, double* dir3) {
    return orbit_cameras<double>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames, rotate_first,
                                 basis12, sun3, dir3);
}

// Content hash for the drop-in render.hpp's per-call scene check (render.hpp:86-156 reads the
// caller's arrays on every call): 64-bit multiply-mix over 8-byte words in 256-KiB chunks hashed
// in parallel (OpenMP), chunk hashes folded in order -- deterministic for a given byte string.
uint64_t ceres_content_hash(const void* p, size_t bytes) {
    if (!p || !bytes) return 0x9e3779b97f4a7c15ull ^ bytes;
    constexpr size_t kChunk = 256 << 10;
    const size_t n_chunks = (bytes + kChunk - 1) / kChunk;
    auto mix = [](uint64_t h, uint64_t w) {
        h ^= w * 0x9e3779b97f4a7c15ull;
        h = (h << 31) | (h >> 33);
        return h * 0xbf58476d1ce4e5b9ull;
    };
    auto chunk_hash = [&](size_t c) {
        const unsigned char* b = static_cast<const unsigned char*>(p) + c * kChunk;
        const size_t n = std::min(kChunk, bytes - c * kChunk);
        uint64_t h[4] = {0x243f6a8885a308d3ull, 0x13198a2e03707344ull, 0xa4093822299f31d0ull, 0x082efa98ec4e6c89ull};
        size_t i = 0;
        for (; i + 32 <= n; i += 32) {
            uint64_t w[4];
            std::memcpy(w, b + i, 32);
            for (int k = 0; k < 4; ++k) h[k] = mix(h[k], w[k]);
        }
        for (; i < n; i += 8) {                                  // < 32 bytes left: zero-padded words
            uint64_t w = 0;
            std::memcpy(&w, b + i, std::min<size_t>(8, n - i));
            h[0] = mix(h[0], w);
        }
        return mix(mix(mix(mix(h[0], h[1]), h[2]), h[3]), n);
    };
    std::vector<uint64_t> hs(n_chunks);
    #pragma omp parallel for schedule(static) if (n_chunks > 4)
    for (size_t c = 0; c < n_chunks; ++c) hs[c] = chunk_hash(c);
    uint64_t h = 0x6a09e667f3bcc908ull ^ bytes;
    for (uint64_t x : hs) h = mix(h, x);
    return h;
}

// ---- the same steps in a chosen arithmetic (CERES_ARITH_EXACT / CERES_ARITH_FMA) ----
static int bad_arith(int arith) {
    return arith == CERES_ARITH_EXACT || arith == CERES_ARITH_FMA ? 0 : set_error(CERES_EINVAL, "unknown arithmetic %d", arith);
}
int ceres_obj_load_arith(const char* path, float** tri48, float** norm36, size_t* n_tri, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? obj_load<float, true>(path, tri48, norm36, n_tri) : obj_load<float, false>(path, tri48, norm36, n_tri);
}
int ceres_proc_mesh_arith(int n, float** tri48, float** norm36, size_t* n_tri, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? proc_mesh<float, true>(n, tri48, norm36, n_tri) : proc_mesh<float, false>(n, tri48, norm36, n_tri);
}
int ceres_rotate_triangles_arith(float* tri48, size_t n_tri, int axis, float degrees, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? rotate_triangles<float, true>(tri48, n_tri, axis, degrees) : rotate_triangles<float, false>(tri48, n_tri, axis, degrees);
}
int ceres_bvh_build_arith(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    if (!nodes32) return set_error(CERES_EINVAL, "ceres_bvh_build: null argument");
    NodeT<float>* nodes = nullptr;
    const int rc = arith ? bvh_build<float, true>(tri48, n_tri, &nodes, n_nodes, prim64)
                         : bvh_build<float, false>(tri48, n_tri, &nodes, n_nodes, prim64);
    *nodes32 = reinterpret_cast<uint32_t*>(nodes);
    return rc;
}
int ceres_camera_basis_arith(const float eye[3], const float dir[3], const float up[3], float fov_deg,
                             size_t width, size_t height, float out9[9], int arith) {
    (void)eye;
    if (int rc = bad_arith(arith)) return rc;
    return arith ? camera_basis<float, true>(dir, up, fov_deg, width, height, out9)
                 : camera_basis<float, false>(dir, up, fov_deg, width, height, out9);
}
int ceres_orbit_cameras_arith(const float eye[3], const float dir[3], const float up[3], const float sun[3], float fov_deg,
                              size_t width, size_t height, const float axis[3], float step_deg, uint32_t n_frames,
                              int rotate_first, float* basis12, float* sun3, float* dir3, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? orbit_cameras<float, true>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames,
                                              rotate_first, basis12, sun3, dir3)
                 : orbit_cameras<float, false>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames,
                                               rotate_first, basis12, sun3, dir3);
}

// render<double> in the reference CMake build's arithmetic (anim.cpp -d compiled with -mfma,
// CMakeLists.txt:11): GCC fuses the double host steps at the same sites as the float ones
// (oracle/contraction_sites.txt; the double dump's FMA sites -- triangle normals, rotation, vertex
// normals, SAH costs -- carry the same expressions), so the G = true templates serve both scalars.
int ceres_obj_load_f64_arith(const char* path, double** tri96, double** norm72, size_t* n_tri, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? obj_load<double, true>(path, tri96, norm72, n_tri) : obj_load<double, false>(path, tri96, norm72, n_tri);
}
int ceres_proc_mesh_f64_arith(int n, double** tri96, double** norm72, size_t* n_tri, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? proc_mesh<double, true>(n, tri96, norm72, n_tri) : proc_mesh<double, false>(n, tri96, norm72, n_tri);
}
int ceres_rotate_triangles_f64_arith(double* tri96, size_t n_tri, int axis, double degrees, int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? rotate_triangles<double, true>(tri96, n_tri, axis, degrees)
                 : rotate_triangles<double, false>(tri96, n_tri, axis, degrees);
}
int ceres_bvh_build_f64_arith(const double* tri96, size_t n_tri, uint64_t** nodes64, size_t* n_nodes, uint64_t** prim64,
                              int arith) {
    if (int rc = bad_arith(arith)) return rc;
    if (!nodes64) return set_error(CERES_EINVAL, "ceres_bvh_build_f64: null argument");
    NodeT<double>* nodes = nullptr;
    const int rc = arith ? bvh_build<double, true>(tri96, n_tri, &nodes, n_nodes, prim64)
                         : bvh_build<double, false>(tri96, n_tri, &nodes, n_nodes, prim64);
    *nodes64 = reinterpret_cast<uint64_t*>(nodes);
    return rc;
}
int ceres_camera_basis_f64_arith(const double eye[3], const double dir[3], const double up[3], double fov_deg,
                                 size_t width, size_t height, double out9[9], int arith) {
    (void)eye;
    if (int rc = bad_arith(arith)) return rc;
    return arith ? camera_basis<double, true>(dir, up, fov_deg, width, height, out9)
                 : camera_basis<double, false>(dir, up, fov_deg, width, height, out9);
}
int ceres_orbit_cameras_f64_arith(const double eye[3], const double dir[3], const double up[3], const double sun[3],
                                  double fov_deg, size_t width, size_t height, const double axis[3], double step_deg,
                                  uint32_t n_frames, int rotate_first, double* basis12, double* sun3, double* dir3,
                                  int arith) {
    if (int rc = bad_arith(arith)) return rc;
    return arith ? orbit_cameras<double, true>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames,
                                               rotate_first, basis12, sun3, dir3)
                 : orbit_cameras<double, false>(eye, dir, up, sun, fov_deg, width, height, axis, step_deg, n_frames,
                                                rotate_first, basis12, sun3, dir3);
}

}  // extern "C"

// ---------------------------------------------------------------- compacted float readback
// render.hpp:86-89 writes every pixel of the caller's float framebuffer; ceres_render_f32 sends
// only the lit pixels over the host link (a C3 frame: ~7 % of them) and writes the rest here as
// zeros -- the bits the reference stores for a miss or a shadowed hit (render.hpp:116-117,147-150).
// The fill runs on the caller's cores while the kernel runs.
namespace ceres {
static int host_threads() {
    const int t = omp_get_max_threads();
    return t < 1 ? 1 : t > 16 ? 16 : t;
}
void host_fill_zero(float* dst, size_t n) {
    const size_t chunk = size_t(1) << 16;                            // 256 KB per task
    const long long nc = (long long)((n + chunk - 1) / chunk);
    #pragma omp parallel for schedule(static) num_threads(host_threads())
    for (long long c = 0; c < nc; ++c) {
        const size_t a = size_t(c) * chunk, b = std::min(n, a + chunk);
        std::memset(dst + a, 0, (b - a) * sizeof(float));
    }
}
void host_scatter_lit(float* dst, const uint32_t* lit4, size_t n) {    // records {pixel, r, g, b} (bits)
    #pragma omp parallel for schedule(static) num_threads(host_threads()) if (n > 16384)
    for (long long k = 0; k < (long long)n; ++k) {
        const uint32_t* r = lit4 + 4 * size_t(k);
        uint32_t* q = reinterpret_cast<uint32_t*>(dst + 3 * size_t(r[0]));
        q[0] = r[1]; q[1] = r[2]; q[2] = r[3];
    }
}
}  // namespace ceres
