// oracle/oracle.cpp -- CPU RESTATEMENT OF THE REFERENCE HOT PATH.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library, and only as the checker.  The product (ceres-raytracer_amd/) never links it.
//
// A from-scratch restatement (not a copy) of iracigt/ceres-raytracer's render() path,
// written so that every floating-point operation happens in the same order as in the
// reference.  Compiled with -ffp-contract=off, and every function comes in two arithmetic
// flavours selected by a `contract` argument:
//   contract = 0  bit-identical to the reference headers compiled with -ffp-contract=off
//                 (oracle/_ref/ref_render_exact);
//   contract = 1  bit-identical to the reference as its own CMake build compiles it
//                 (CMakeLists.txt:11-13, -O3 -mavx2 -mfma: GCC 11 fuses a*b+c into FMA at the
//                 sites its widening_mul pass picks, oracle/_ref/ref_render).  Each such site is
//                 an explicit fmaf here, read from `g++ -fdump-tree-widening_mul-lineno` of the
//                 reference build (oracle/contraction_sites.txt lists them with file:line).
//
// Parity is PINNED: tests/test_oracle_golden.py checks this library against the golden
// fixtures generated from the reference itself (tests/golden/make_golden.py): PPM
// sha256, ray/hit counts, traversal statistics, camera basis bits, rotated-triangle and
// normal bits, canonical BVH topology and per-pixel {prim,t,u,v,shadow,rgb} records.
//
// Citations (file:line) are into /root/reference.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cfloat>
#include <cctype>
#include <algorithm>
#include <array>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct V3 { float x, y, z; };
inline float at(const V3& a, int i) { return i == 0 ? a.x : i == 1 ? a.y : a.z; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }        // vector.hpp:122-132
inline float dot(V3 a, V3 b) { float s = a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }   // vector.hpp:134-141
inline V3 cross(V3 a, V3 b) {                                                 // vector.hpp:159-167
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline V3 normalize(V3 v) { float inv = 1.0f / std::sqrt(dot(v, v)); return mul(v, inv); }   // vector.hpp:143-154

// GCC-contracted forms (G = true) of the same expressions.  dot (vector.hpp:134-141) is
// ((a0 b0 + a1 b1) + a2 b2); GCC fuses it as fma(a2, b2, fma(a0, b0, a1 b1)) ("A") everywhere
// but in Triangle::intersect's v = dot(r, e1), where it fuses fma(a2, b2, fma(a1, b1, a0 b0))
// ("B").  cross (vector.hpp:159-167) a_j b_k - a_k b_j becomes fma(a_j, b_k, -(a_k b_j)).
template <bool G> inline float dotA(V3 a, V3 b) { return G ? std::fmaf(a.z, b.z, std::fmaf(a.x, b.x, a.y * b.y)) : dot(a, b); }
template <bool G> inline float dotB(V3 a, V3 b) { return G ? std::fmaf(a.z, b.z, std::fmaf(a.y, b.y, a.x * b.x)) : dot(a, b); }
template <bool G> inline V3 crossG(V3 a, V3 b) {
    if (!G) return cross(a, b);
    return {std::fmaf(a.y, b.z, -(a.z * b.y)), std::fmaf(a.z, b.x, -(a.x * b.z)), std::fmaf(a.x, b.y, -(a.y * b.x))};
}
template <bool G> inline V3 normalizeG(V3 v) { float inv = 1.0f / std::sqrt(dotA<G>(v, v)); return mul(v, inv); }

// Triangle (triangle.hpp:17-37): p0, e1 = p0 - p1, e2 = p2 - p0, n = cross(e1, e2); 48 bytes.
struct Tri { V3 p0, e1, e2, n; };
static_assert(sizeof(Tri) == 48, "Triangle layout");
template <bool G> inline Tri make_tri(V3 p0, V3 p1, V3 p2) { Tri t; t.p0 = p0; t.e1 = sub(p0, p1); t.e2 = sub(p2, p0); t.n = crossG<G>(t.e1, t.e2); return t; }
inline V3 tri_p1(const Tri& t) { return sub(t.p0, t.e1); }                   // triangle.hpp:36
inline V3 tri_p2(const Tri& t) { return add(t.p0, t.e2); }                   // triangle.hpp:37

// Bvh::Node (bvh.hpp:25-30): bounds {xmin,xmax,ymin,ymax,zmin,zmax}, u32 count, u32 first.
struct Node { float b[6]; uint32_t count, first; };
static_assert(sizeof(Node) == 32, "Node layout");

struct Box { V3 lo, hi; };
inline Box box_empty() { return {{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}}; }   // bounding_box.hpp:76-80
inline float fmin_std(float a, float b) { return (b < a) ? b : a; }          // std::min
inline float fmax_std(float a, float b) { return (a < b) ? b : a; }          // std::max
inline void box_extend(Box& a, const Box& b) {                               // bounding_box.hpp:21-25
    a.lo = {fmin_std(a.lo.x, b.lo.x), fmin_std(a.lo.y, b.lo.y), fmin_std(a.lo.z, b.lo.z)};
    a.hi = {fmax_std(a.hi.x, b.hi.x), fmax_std(a.hi.y, b.hi.y), fmax_std(a.hi.z, b.hi.z)};
}
inline void box_extend(Box& a, V3 v) { box_extend(a, Box{v, v}); }
inline float half_area(const Box& b) { V3 d = sub(b.hi, b.lo); return (d.x + d.y) * d.z + d.x * d.y; }   // bounding_box.hpp:43-46
// GCC fuses half_area's first product inside find_split's sweeps (binned_sah_builder.hpp:98,109)
// and its second product in the node's max_split_cost (:179)
template <bool G> inline float half_area_sweep(const Box& b) { V3 d = sub(b.hi, b.lo); return G ? std::fmaf(d.x + d.y, d.z, d.x * d.y) : half_area(b); }
template <bool G> inline float half_area_node(const Box& b) { V3 d = sub(b.hi, b.lo); return G ? std::fmaf(d.x, d.y, (d.x + d.y) * d.z) : half_area(b); }
inline int largest_axis(const Box& b) {                                      // bounding_box.hpp:53-59
    V3 d = sub(b.hi, b.lo); int a = 0;
    if (d.x < d.y) a = 1;
    if (at(d, a) < d.z) a = 2;
    return a;
}

thread_local std::string g_err;

// ---------------------------------------------------------------- OBJ loader (obj_norms.hpp)
void remove_eol(char* p) {                                                   // obj_norms.hpp:12-20
    int i = 0; while (p[i]) i++; i--;
    while (i > 0 && std::isspace((unsigned char)p[i])) { p[i] = '\0'; i--; }
}
char* skip_ws(char* p) { while (std::isspace((unsigned char)*p)) p++; return p; }   // obj_norms.hpp:22-25
bool read_index(char** pp, int* out) {                                       // obj_norms.hpp:27-55
    char* b = skip_ws(*pp);
    if (!std::isdigit((unsigned char)*b) && *b != '-') return false;
    int idx = (int)std::strtol(b, &b, 10);
    b = skip_ws(b);
    if (*b == '/') {
        b++;
        if (*b != '/') std::strtol(b, &b, 10);
        b = skip_ws(b);
        if (*b == '/') { b++; std::strtol(b, &b, 10); }
    }
    *pp = b; *out = idx; return true;
}

struct Mesh { std::vector<Tri> tris; std::vector<std::array<V3, 3>> norms; };

template <bool G> int load_stream(std::istream& is, Mesh& m) {                                 // obj_norms.hpp:57-118
    static constexpr size_t max_line = 1024;
    char line[max_line];
    std::vector<V3> verts, vnorm;
    std::vector<std::array<size_t, 3>> tidx;
    while (is.getline(line, max_line)) {
        char* p = skip_ws(line);
        if (*p == '\0' || *p == '#') continue;
        remove_eol(p);
        if (*p == 'v' && std::isspace((unsigned char)p[1])) {
            float x = std::strtof(p + 1, &p); float y = std::strtof(p, &p); float z = std::strtof(p, &p);
            verts.push_back({x, y, z}); vnorm.push_back({0.f, 0.f, 0.f});
        } else if (*p == 'f' && std::isspace((unsigned char)p[1])) {
            V3 pts[2]; size_t id[2] = {0, 0};
            p += 2;
            for (size_t i = 0;; ++i) {
                int index;
                if (!read_index(&p, &index)) break;
                size_t j = index < 0 ? verts.size() + index : size_t(index - 1);
                if (j >= verts.size()) { g_err = "OBJ face index out of range"; return -2; }   // obj_norms.hpp:90 assert
                V3 v = verts[j];
                if (i >= 2) {                                                // fan triangulation, obj_norms.hpp:92-98
                    m.tris.push_back(make_tri<G>(pts[0], pts[1], v));
                    V3 n = m.tris.back().n;
                    vnorm[id[0]] = add(vnorm[id[0]], n);
                    vnorm[id[1]] = add(vnorm[id[1]], n);
                    vnorm[j] = add(vnorm[j], n);
                    tidx.push_back({id[0], id[1], j});
                    pts[1] = v; id[1] = j;
                } else { pts[i] = v; id[i] = j; }
            }
        }
    }
    for (auto& n : vnorm) n = normalizeG<G>(n);                              // obj_norms.hpp:109-111
    m.norms.reserve(tidx.size());
    for (auto& t : tidx) m.norms.push_back({vnorm[t[0]], vnorm[t[1]], vnorm[t[2]]});   // obj_norms.hpp:113-115
    return 0;
}

int export_mesh(Mesh& m, float** tri48, float** norm36, size_t* n) {
    *n = m.tris.size();
    *tri48 = (float*)std::malloc(std::max<size_t>(1, m.tris.size() * sizeof(Tri)));
    *norm36 = (float*)std::malloc(std::max<size_t>(1, m.norms.size() * 36));
    if (!*tri48 || !*norm36) { g_err = "out of memory"; return -3; }
    std::memcpy(*tri48, m.tris.data(), m.tris.size() * sizeof(Tri));
    std::memcpy(*norm36, m.norms.data(), m.norms.size() * 36);
    return 0;
}

// ---------------------------------------------------------------- binned SAH (binned_sah_builder.hpp)
constexpr size_t kBins = 16;
struct Bin { Box box; size_t count; float right_cost; };
struct Item { size_t node, begin, end, depth; size_t size() const { return end - begin; } };

template <bool G> struct Builder {
    std::vector<Node> nodes;
    std::vector<size_t> prim;
    const Box* boxes; const V3* centers;
    size_t node_count = 1;
    const size_t max_depth = 64, max_leaf = 16;                              // top_down_builder.hpp:36,41
    const float traversal_cost = 1;                                          // sah_based_algorithm.hpp:16
    Bin bins[3][kBins];

    static void set_box(Node& n, const Box& b) { n.b[0] = b.lo.x; n.b[1] = b.hi.x; n.b[2] = b.lo.y; n.b[3] = b.hi.y; n.b[4] = b.lo.z; n.b[5] = b.hi.z; }
    static Box get_box(const Node& n) { return {{n.b[0], n.b[2], n.b[4]}, {n.b[1], n.b[3], n.b[5]}}; }

    std::pair<float, size_t> find_split(int axis) {                          // binned_sah_builder.hpp:89-114
        Bin* b = bins[axis];
        Box cur = box_empty(); size_t cnt = 0;
        for (size_t i = kBins - 1; i > 0; --i) { box_extend(cur, b[i].box); cnt += b[i].count; b[i].right_cost = half_area_sweep<G>(cur) * cnt; }
        cur = box_empty(); cnt = 0;
        std::pair<float, size_t> best(FLT_MAX, kBins);
        for (size_t i = 0; i < kBins - 1; ++i) {
            box_extend(cur, b[i].box); cnt += b[i].count;
            float cost = G ? std::fmaf(float(cnt), half_area_sweep<G>(cur), b[i + 1].right_cost)
                           : half_area(cur) * cnt + b[i + 1].right_cost;
            if (cost < best.first) best = {cost, i + 1};
        }
        return best;
    }

    // returns true and two children items when split
    bool step(const Item& it, Item& l, Item& r) {                            // binned_sah_builder.hpp:123-234
        Node& node = nodes[it.node];
        auto leaf = [&]() { node.first = uint32_t(it.begin); node.count = uint32_t(it.size()); };
        if (it.size() <= 1 || it.depth >= max_depth) { leaf(); return false; }
        Box bb = get_box(node);
        V3 d = sub(bb.hi, bb.lo);
        V3 c2b = mul(V3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z}, float(kBins));   // diagonal().inverse() * bin_count
        V3 off = {(-bb.lo.x) * c2b.x, (-bb.lo.y) * c2b.y, (-bb.lo.z) * c2b.z};
        auto bin_of = [&](const V3& c, int a) -> size_t {
            float bi = std::fmaf(at(c, a), at(c2b, a), at(off, a));          // fast_multiply_add, utilities.hpp:37-44
            return std::min(kBins - 1, size_t(std::max(0.0f, bi)));
        };
        for (int a = 0; a < 3; ++a) for (auto& b : bins[a]) { b.box = box_empty(); b.count = 0; }
        for (size_t i = it.begin; i < it.end; ++i) {
            size_t p = prim[i];
            for (int a = 0; a < 3; ++a) { Bin& b = bins[a][bin_of(centers[p], a)]; b.count++; box_extend(b.box, boxes[p]); }
        }
        std::pair<float, size_t> best[3];
        for (int a = 0; a < 3; ++a) best[a] = find_split(a);
        int ax = 0;
        if (best[0].first > best[1].first) ax = 1;
        if (best[ax].first > best[2].first) ax = 2;
        size_t split = best[ax].second;
        float max_cost = half_area_node<G>(bb) * (it.size() - traversal_cost);
        if (best[ax].second == kBins || best[ax].first >= max_cost) {
            if (it.size() > max_leaf) {                                      // median-ish fallback, :180-196
                ax = largest_axis(bb);
                for (size_t i = 0, cnt = 0; i < kBins - 1; ++i) {
                    cnt += bins[ax][i].count;
                    if (cnt >= (it.size() * 2 / 5 + 1)) { split = i + 1; break; }
                }
            } else { leaf(); return false; }
        }
        size_t mid = std::partition(prim.data() + it.begin, prim.data() + it.end,
                                    [&](size_t i) { return bin_of(centers[i], ax) < split; }) - prim.data();
        if (mid > it.begin && mid < it.end) {
            size_t fc = node_count; node_count += 2;
            node.first = uint32_t(fc); node.count = 0;
            Box lb = box_empty(), rb = box_empty();
            for (size_t i = 0; i < best[ax].second; ++i) box_extend(lb, bins[ax][i].box);   // note: best split index, :216-220
            for (size_t i = split; i < kBins; ++i) box_extend(rb, bins[ax][i].box);
            set_box(nodes[fc], lb); set_box(nodes[fc + 1], rb);
            l = {fc, it.begin, mid, it.depth + 1}; r = {fc + 1, mid, it.end, it.depth + 1};
            return true;
        }
        leaf(); return false;
    }
};

// ---------------------------------------------------------------- traversal (single_ray_traverser.hpp)
struct Hit { uint32_t prim; float t, u, v; };
struct Ctx {
    const Tri* tris; const Node* nodes; const uint64_t* prim;
};

// Triangle::intersect, triangle.hpp:95-115 (left-handed normal)
template <bool G> inline bool tri_hit(const Tri& tr, V3 o, V3 d, float tmin, float tmax, float* t, float* u, float* v) {
    V3 c = sub(tr.p0, o);
    V3 r = crossG<G>(d, c);
    float inv_det = 1.0f / dotA<G>(tr.n, d);
    float uu = dotA<G>(r, tr.e2) * inv_det;
    float vv = dotB<G>(r, tr.e1) * inv_det;
    float ww = 1.0f - uu - vv;
    if (uu >= 0 && vv >= 0 && ww >= 0) {
        float tt = dotA<G>(tr.n, c) * inv_det;
        if (tt >= tmin && tt <= tmax) { *t = tt; *u = uu; *v = vv; return true; }
    }
    return false;
}

// Closest-hit traversal with statistics; returns true on hit.  Stack overflow sets *ovf.
template <bool G> bool traverse(const Ctx& cx, V3 o, V3 d, Hit* best, uint64_t* pairs, uint64_t* tests, bool* ovf, bool robust = false) {
    float tmin = 0.0f, tmax = FLT_MAX;                                       // ray.hpp:17-21
    bool have = false;
    auto leaf = [&](const Node& n) {                                         // intersect_leaf :43-63
        size_t b = n.first, e = b + n.count;
        *tests += e - b;
        for (size_t i = b; i < e; ++i) {
            size_t idx = size_t(cx.prim[i]);                                 // primitive_at, primitive_intersectors.hpp:17-20
            float t, u, v;
            if (tri_hit<G>(cx.tris[idx], o, d, tmin, tmax, &t, &u, &v)) { *best = {uint32_t(idx), t, u, v}; have = true; tmax = t; }
        }
    };
    if (cx.nodes[0].count != 0) { leaf(cx.nodes[0]); return have; }          // root-is-leaf, :72-73
    // FastNodeIntersector (node_intersectors.hpp:83-103): octant + safe_inverse + scaled origin
    int oct[3] = {std::signbit(d.x), std::signbit(d.y), std::signbit(d.z)};
    const float eps = FLT_EPSILON;
    auto sinv = [&](float x) { return 1.0f / (std::fabs(x) < eps ? std::copysign(eps, x) : x); };   // vector.hpp:69-74
    V3 inv = {sinv(d.x), sinv(d.y), sinv(d.z)};
    V3 so = {(-o.x) * inv.x, (-o.y) * inv.y, (-o.z) * inv.z};
    auto rmax = [](float x, float y) { return x > y ? x : y; };              // utilities.hpp:57-67
    auto rmin = [](float x, float y) { return x < y ? x : y; };
    // RobustNodeIntersector (node_intersectors.hpp:54-79): plain inverse, exit slabs scaled by the
    // inverse padded by 2 ulps of magnitude (add_ulp_magnitude, utilities.hpp:102-106)
    auto pad2 = [](float x) { uint32_t u; std::memcpy(&u, &x, 4); u += 2; float r; std::memcpy(&r, &u, 4); return std::isfinite(x) ? r : x; };
    const V3 rinv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const V3 pinv = {pad2(rinv.x), pad2(rinv.y), pad2(rinv.z)};
    auto box = [&](const Node& n, float* en, float* ex) {                    // node_intersectors.hpp:35-47
        float e0, e1, e2, x0, x1, x2;
        if (robust) {                                                        // (p - o) * inv, :70-73
            e0 = (n.b[0 + oct[0]] - o.x) * rinv.x; x0 = (n.b[1 - oct[0]] - o.x) * pinv.x;
            e1 = (n.b[2 + oct[1]] - o.y) * rinv.y; x1 = (n.b[3 - oct[1]] - o.y) * pinv.y;
            e2 = (n.b[4 + oct[2]] - o.z) * rinv.z; x2 = (n.b[5 - oct[2]] - o.z) * pinv.z;
        } else {
            e0 = std::fmaf(n.b[0 + oct[0]], inv.x, so.x);
            e1 = std::fmaf(n.b[2 + oct[1]], inv.y, so.y);
            e2 = std::fmaf(n.b[4 + oct[2]], inv.z, so.z);
            x0 = std::fmaf(n.b[1 - oct[0]], inv.x, so.x);
            x1 = std::fmaf(n.b[3 - oct[1]], inv.y, so.y);
            x2 = std::fmaf(n.b[5 - oct[2]], inv.z, so.z);
        }
        *en = rmax(e0, rmax(e1, rmax(e2, tmin)));
        *ex = rmin(x0, rmin(x1, rmin(x2, tmax)));
    };
    uint32_t stack[64]; size_t sp = 0;                                       // Stack, :22-39
    const Node* left = &cx.nodes[cx.nodes[0].first];
    while (true) {                                                           // :82-123
        ++*pairs;
        const Node* right = left + 1;
        float ln, lx, rn, rx;
        box(*left, &ln, &lx);
        box(*right, &rn, &rx);
        if (ln <= lx) { if (left->count != 0) { leaf(*left); left = nullptr; } } else left = nullptr;
        if (rn <= rx) { if (right->count != 0) { leaf(*right); right = nullptr; } } else right = nullptr;
        if (left) {
            if (right) {
                if (ln > rn) std::swap(left, right);
                if (sp >= 64) { *ovf = true; return have; }
                stack[sp++] = right->first;
            }
            left = &cx.nodes[left->first];
        } else if (right) {
            left = &cx.nodes[right->first];
        } else {
            if (sp == 0) break;
            left = &cx.nodes[stack[--sp]];
        }
    }
    return have;
}

// ---------------------------------------------------------------- shading (render.hpp:46-84)
// lambertian's sum (render.hpp:48) contracts like dot "A"; in smooth_shading GCC fuses
// amb + 0.5 lam into fma(lam, 0.5, amb) and each channel's (amb + diffuse) * k + specular into
// fma(amb + diffuse, k, specular) (render.hpp:67-81); the c[] accumulation stays unfused.
template <bool G> inline float lambertian(V3 s, V3 n) { return G ? std::fabs(dotA<true>(s, n)) : std::fabs(s.x * n.x + s.y * n.y + s.z * n.z); }
template <bool G> inline float blinn_phong_spec(V3 s, V3 n, V3 view) { return (float)std::pow((double)dotA<G>(n, normalizeG<G>(add(s, view))), 24.0); }
inline float clampf(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }   // std::clamp
template <bool G> inline void smooth_shading(V3 sun_line, const std::array<V3, 3>& N, V3 view, float u, float v, float c[3]) {
    c[0] = c[1] = c[2] = 0.f;
    const float amb = 0.2;
    const V3 vneg = mul(view, -1.0f);
    const float w[3] = {u, v, 1 - u - v};
    for (int k = 0; k < 3; ++k) {
        const float lam = lambertian<G>(sun_line, N[k]);
        float specular = 0.8f * blinn_phong_spec<G>(sun_line, N[k], vneg);
        const float base = G ? std::fmaf(lam, 0.5f, amb) : amb + 0.5f * lam;
        const float kr = G ? std::fmaf(base, 0.5f, specular) : base * 0.5f + specular;
        const float kg = G ? std::fmaf(base, 0.0f, specular) : base * 0.0f + specular;
        const float kb = G ? std::fmaf(base, 0.8f, specular) : base * 0.8f + specular;
        c[0] += w[k] * clampf(kr, 0.f, 1.f);
        c[1] += w[k] * clampf(kg, 0.f, 1.f);
        c[2] += w[k] * clampf(kb, 0.f, 1.f);
    }
}

inline uint8_t quantize(float x) {                                           // static.cpp:141-143
    float a = x * 255; float m = (255.f < a) ? 255.f : a; float q = (m < 0.f) ? 0.f : m;
    return static_cast<uint8_t>(q);
}

}  // namespace

extern "C" {

const char* oracle_last_error(void) { return g_err.c_str(); }
void oracle_free(void* p) { std::free(p); }

// Numbering-independent serialisation of a bvh::Bvh<float> (bvh.hpp:25-79): pre-order DFS from
// the root, per node its 6 bounds + primitive_count (7 x 4 B), leaves followed by their
// primitive_indices (u64).  Same byte stream as tests/golden/make_golden.py canonical_bvh_sha,
// in C so 10M-node trees take milliseconds.  *out is malloc'd.
int oracle_bvh_canonical(const uint32_t* nodes32, size_t n_nodes, const uint64_t* prim, size_t n_prim,
                         uint8_t** out, size_t* out_len) {
    std::vector<uint8_t> buf;
    buf.reserve(n_nodes * 28 + n_prim * 8);
    std::vector<uint32_t> st{0};
    size_t visited = 0;
    while (!st.empty()) {
        const uint32_t k = st.back(); st.pop_back();
        if (k >= n_nodes || ++visited > n_nodes) { g_err = "bad BVH"; return -1; }
        const uint32_t* n = nodes32 + 8 * size_t(k);
        const uint8_t* b = reinterpret_cast<const uint8_t*>(n);
        buf.insert(buf.end(), b, b + 28);
        const uint32_t cnt = n[6], first = n[7];
        if (cnt) {
            if (size_t(first) + cnt > n_prim) { g_err = "bad leaf"; return -1; }
            const uint8_t* q = reinterpret_cast<const uint8_t*>(prim + first);
            buf.insert(buf.end(), q, q + 8 * size_t(cnt));
        } else {
            st.push_back(first + 1);
            st.push_back(first);
        }
    }
    *out = static_cast<uint8_t*>(std::malloc(std::max<size_t>(1, buf.size())));
    if (!*out) { g_err = "out of memory"; return -3; }
    std::memcpy(*out, buf.data(), buf.size());
    *out_len = buf.size();
    return 0;
}

int oracle_load_obj(const char* path, float** tri48, float** norm36, size_t* n_tri, int contract) {   // obj_norms.hpp:120-127
    std::ifstream is(path);
    Mesh m;
    if (is) { int rc = contract ? load_stream<true>(is, m) : load_stream<false>(is, m); if (rc) return rc; }
    return export_mesh(m, tri48, norm36, n_tri);
}

int oracle_load_obj_text(const char* text, size_t len, float** tri48, float** norm36, size_t* n_tri, int contract) {
    std::istringstream is(std::string(text, len));
    Mesh m;
    int rc = contract ? load_stream<true>(is, m) : load_stream<false>(is, m);
    if (rc) return rc;
    return export_mesh(m, tri48, norm36, n_tri);
}

}  // extern "C"

namespace {
template <bool G> int proc_mesh(int n, float** tri48, float** norm36, size_t* n_tri) {
    if (n < 2) { g_err = "proc mesh needs n >= 2"; return -1; }
    std::vector<V3> verts(size_t(n) * n), vnorm(size_t(n) * n, V3{0.f, 0.f, 0.f});
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double x = double(i) / double(n - 1), y = double(j) / double(n - 1);
            double z = 0.05 * (std::sin(40.0 * x) + std::cos(37.0 * y)) + 0.01 * std::sin(400.0 * x + 300.0 * y);
            verts[size_t(j) * n + i] = {(float)x, (float)y, (float)z};
        }
    Mesh m;
    size_t nt = size_t(n - 1) * (n - 1) * 2;
    m.tris.reserve(nt);
    std::vector<std::array<size_t, 3>> tidx; tidx.reserve(nt);
    for (int j = 0; j + 1 < n; ++j)
        for (int i = 0; i + 1 < n; ++i) {
            size_t a = size_t(j) * n + i, b = a + 1, c = a + n + 1, d = a + n;
            const size_t f[2][3] = {{a, b, c}, {a, c, d}};
            for (auto& q : f) {
                m.tris.push_back(make_tri<G>(verts[q[0]], verts[q[1]], verts[q[2]]));
                V3 nn = m.tris.back().n;
                for (int k = 0; k < 3; ++k) vnorm[q[k]] = add(vnorm[q[k]], nn);
                tidx.push_back({q[0], q[1], q[2]});
            }
        }
    for (auto& v : vnorm) v = normalizeG<G>(v);
    m.norms.reserve(nt);
    for (auto& t : tidx) m.norms.push_back({vnorm[t[0]], vnorm[t[1]], vnorm[t[2]]});
    return export_mesh(m, tri48, norm36, n_tri);
}

// rotate_triangles<Axis> (render.hpp:24-44).  GCC fuses each rotated coordinate's first product:
// p1 c - p2 s -> fma(p1, c, -(p2 s)), p1 s + p2 c -> fma(p1, s, p2 c), -p0 s + p2 c -> fma(-p0, s, p2 c).
template <bool G> void rotate(float* tri48, size_t n, int axis, float degrees) {
    const float pi = float(3.14159265359);
    float c = std::cos(degrees * pi / float(180));
    float s = std::sin(degrees * pi / float(180));
    auto f2 = [](float a, float b, float x, float y, bool minus) {      // a*b -/+ x*y
        if (G) return std::fmaf(a, b, minus ? -(x * y) : x * y);
        return minus ? a * b - x * y : a * b + x * y;
    };
    auto rot = [&](V3 p) -> V3 {
        if (axis == 0) return {p.x, f2(p.y, c, p.z, s, true), f2(p.y, s, p.z, c, false)};
        if (axis == 1) return {f2(p.x, c, p.z, s, false), p.y, f2(-p.x, s, p.z, c, false)};
        return {f2(p.x, c, p.y, s, true), f2(p.x, s, p.y, c, false), p.z};
    };
    Tri* t = reinterpret_cast<Tri*>(tri48);
    #pragma omp parallel for
    for (size_t i = 0; i < n; ++i) {
        V3 p0 = rot(t[i].p0), p1 = rot(tri_p1(t[i])), p2 = rot(tri_p2(t[i]));
        t[i] = make_tri<G>(p0, p1, p2);
    }
}

template <bool G> int build_bvh(const float* tri48, size_t n, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64) {
    if (n == 0) { g_err = "empty scene"; return -1; }
    const Tri* t = reinterpret_cast<const Tri*>(tri48);
    std::vector<Box> boxes(n); std::vector<V3> centers(n);
    for (size_t i = 0; i < n; ++i) {
        Box b{t[i].p0, t[i].p0}; box_extend(b, tri_p1(t[i])); box_extend(b, tri_p2(t[i]));   // triangle.hpp:39-44
        boxes[i] = b;
        centers[i] = mul(add(add(t[i].p0, tri_p1(t[i])), tri_p2(t[i])), float(1.0) / float(3.0));   // triangle.hpp:46-48
    }
    Box global = box_empty();
    for (size_t i = 0; i < n; ++i) box_extend(global, boxes[i]);
    Builder<G> B;
    B.nodes.assign(2 * n + 1, Node{});
    B.prim.resize(n);
    for (size_t i = 0; i < n; ++i) B.prim[i] = i;
    B.boxes = boxes.data(); B.centers = centers.data();
    Builder<G>::set_box(B.nodes[0], global);
    std::vector<Item> stack{{0, 0, n, 0}};                                   // top_down_builder.hpp:47-72
    while (!stack.empty()) {
        Item it = stack.back(); stack.pop_back();
        Item l, r;
        if (B.step(it, l, r)) {
            if (l.size() > r.size()) std::swap(l, r);
            stack.push_back(r);
            stack.push_back(l);
        }
    }
    *n_nodes = B.node_count;
    *nodes32 = (uint32_t*)std::malloc(B.node_count * sizeof(Node));
    *prim64 = (uint64_t*)std::malloc(n * 8);
    std::memcpy(*nodes32, B.nodes.data(), B.node_count * sizeof(Node));
    for (size_t i = 0; i < n; ++i) (*prim64)[i] = B.prim[i];
    return 0;
}

// Transform::rotate (transform.hpp:67-104) then operator() (:111-118).  GCC fuses every matrix
// entry's (1-c) n_r * n_k product (c + (1-c) n_r n_r -> fma((1-c) n_r, n_r, c); off-diagonal
// fma((1-c) n_r, n_k, +/-(s n_j))) and applies the rows as dot "A" (then + v = 0).
template <bool G> void orbit(const float axis[3], float step_deg, int count, float eye[3], float dir[3], float sun[3]) {
    const float pi = float(3.14159265359);
    const float angle = step_deg / 180.0f * pi;
    const V3 n = normalizeG<G>(V3{axis[0], axis[1], axis[2]});
    const float nv[3] = {n.x, n.y, n.z};
    const float s = std::sin(angle), c = std::cos(angle);
    float m[3][3];
    const float sn[3] = {s * nv[0], s * nv[1], s * nv[2]};
    // Markley-Crassidis: diagonal c + (1-c) n_r n_r; off-diagonal (1-c) n_r n_k -/+ s n_j
    const float sign[3][3] = {{0, 1, -1}, {-1, 0, 1}, {1, -1, 0}};
    const int other[3][3] = {{0, 2, 1}, {2, 0, 0}, {1, 0, 0}};
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            const float cr = (1 - c) * nv[r];
            if (r == k) m[r][k] = G ? std::fmaf(cr, nv[k], c) : c + cr * nv[k];
            else {
                const float t = sign[r][k] > 0 ? sn[other[r][k]] : -sn[other[r][k]];
                m[r][k] = G ? std::fmaf(cr, nv[k], t) : (sign[r][k] > 0 ? cr * nv[k] + sn[other[r][k]] : cr * nv[k] - sn[other[r][k]]);
            }
        }
    float a[3][3];
    for (int r = 0; r < 3; ++r)                    // ret.a = identity * mat, accumulated from 0
        for (int k = 0; k < 3; ++k) {
            float acc = 0.0f;
            for (int i = 0; i < 3; ++i) acc += (r == i ? 1.0f : 0.0f) * m[i][k];
            a[r][k] = acc;
        }
    auto apply = [&](float* p) {
        float q[3];
        for (int r = 0; r < 3; ++r) q[r] = dotA<G>(V3{a[r][0], a[r][1], a[r][2]}, V3{p[0], p[1], p[2]}) + 0.0f;
        p[0] = q[0]; p[1] = q[1]; p[2] = q[2];
    };
    for (int k = 0; k < count; ++k) { apply(eye); apply(dir); apply(sun); }
}

// Camera basis, render.hpp:91-97.  out = {dir, image_u*w, image_v*w*ratio}.
template <bool G> void camera_basis(const float dir[3], const float up[3], float fov, size_t W, size_t H, float out[9]) {
    V3 d = normalizeG<G>(V3{dir[0], dir[1], dir[2]});
    V3 u = normalizeG<G>(crossG<G>(d, V3{up[0], up[1], up[2]}));
    V3 v = normalizeG<G>(crossG<G>(u, d));
    float w = std::tan(fov * float(3.14159265 * (1.0 / 180.0) * 0.5));
    float ratio = float(H) / float(W);
    u = mul(u, w);
    v = mul(mul(v, w), ratio);
    float o[9] = {d.x, d.y, d.z, u.x, u.y, u.z, v.x, v.y, v.z};
    std::memcpy(out, o, sizeof o);
}
}  // namespace

extern "C" {

// Procedural heightfield: n x n vertices on [0,1]^2, two triangles per
// quad ("f a b c" / "f a c d"), vertex = float(x), float(y), float(z(x,y)) computed in double
// without contraction (the mesh is an input, the same in both arithmetic flavours).
// Equivalent to feeding the OBJ text of oracle/ref_harness.cpp:proc_obj through the loader.
int oracle_proc_mesh(int n, float** tri48, float** norm36, size_t* n_tri, int contract) {
    return contract ? proc_mesh<true>(n, tri48, norm36, n_tri) : proc_mesh<false>(n, tri48, norm36, n_tri);
}

// rotate_triangles<Axis> (render.hpp:24-44): cos/sin of degrees*pi/180 in float, then rebuild
// each Triangle from p0, p1() = p0 - e1, p2() = p0 + e2.
void oracle_rotate(float* tri48, size_t n, int axis, float degrees, int contract) {
    if (contract) rotate<true>(tri48, n, axis, degrees); else rotate<false>(tri48, n, axis, degrees);
}

// compute_bounding_boxes_and_centers + compute_bounding_boxes_union (utilities.hpp:142-171)
// + BinnedSahBuilder<Bvh,16>::build (binned_sah_builder.hpp:39-66), single-threaded:
// the topology (and leaf primitive order) is the reference's; node numbering may differ.
int oracle_build_bvh(const float* tri48, size_t n, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64, int contract) {
    return contract ? build_bvh<true>(tri48, n, nodes32, n_nodes, prim64) : build_bvh<false>(tri48, n, nodes32, n_nodes, prim64);
}

// anim.cpp:76-88 orbit step: Transform<float>().rotate(axis, step/180*pi) (transform.hpp:67-104)
// then operator() (transform.hpp:106-112) on eye, dir and sun, `count` times, in place.
void oracle_orbit(const float axis[3], float step_deg, int count, float eye[3], float dir[3], float sun[3], int contract) {
    if (contract) orbit<true>(axis, step_deg, count, eye, dir, sun); else orbit<false>(axis, step_deg, count, eye, dir, sun);
}

void oracle_camera_basis(const float eye[3], const float dir[3], const float up[3], float fov,
                         size_t W, size_t H, float out[9], int contract) {
    (void)eye;
    if (contract) camera_basis<true>(dir, up, fov, W, H, out); else camera_basis<false>(dir, up, fov, W, H, out);
}

// render() (render.hpp:86-156) over the full framebuffer.
//   mode 0: primary + shadow + smooth shading; mode 1: primary only, pixel = |normalize(n)|;
//   | 0x10: RobustNodeIntersector traversal instead of FastNodeIntersector
//   | 0x20: the reference-flag arithmetic (GCC contraction, see the header)
//   pixels: 3*W*H floats (row j=0 at the bottom, render.hpp:107) or null
//   ppm:    3*W*H bytes of the P6 body (rows top-down, static.cpp:137-145) or null
//   rec_*:  optional per-pixel records (prim -1 on miss; shadow -1 none / 0 lit / 1 occluded)
//   counts: {rays, hits, primary_pairs, primary_tests, shadow_pairs, shadow_tests}
}  // extern "C"

namespace {
template <bool G>
int render_impl(const float* tri48, const float* norm36, size_t n_tri, const uint32_t* nodes32, size_t n_nodes,
                const uint64_t* prim64, const float eye[3], const float basis[9], const float sun[3], int mode,
                size_t W, size_t H, float* pixels, uint8_t* ppm, int32_t* rec_prim, float* rec_tuv,
                int8_t* rec_shadow, uint64_t counts[6], int threads, uint32_t* rec_pairs) {
    if (n_tri == 0 || n_nodes == 0) { g_err = "empty scene"; return -1; }
    const bool robust = (mode & 0x10) != 0;
    mode &= 0xf;
    Ctx cx{reinterpret_cast<const Tri*>(tri48), reinterpret_cast<const Node*>(nodes32), prim64};
    const auto* norms = reinterpret_cast<const std::array<V3, 3>*>(norm36);
    const V3 E{eye[0], eye[1], eye[2]}, D{basis[0], basis[1], basis[2]}, IU{basis[3], basis[4], basis[5]},
        IV{basis[6], basis[7], basis[8]}, S{sun[0], sun[1], sun[2]};
    uint64_t rays = 0, hits = 0, pp = 0, pt = 0, sp_ = 0, st = 0;
    int ovf_any = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    #pragma omp parallel for collapse(2) schedule(dynamic, 64) reduction(+: rays, hits, pp, pt, sp_, st) reduction(|: ovf_any)
    for (size_t i = 0; i < W; ++i) {
        for (size_t j = 0; j < H; ++j) {
            size_t index = 3 * (W * j + i);
            float u = 2 * (i + float(0.5)) / float(W) - float(1);          // render.hpp:109-111
            float v = 2 * (j + float(0.5)) / float(H) - float(1);
            // iu*u + iv*v + dir; GCC fuses the iv*v product: dir + fma(iv, v, iu*u)
            V3 view = G ? normalizeG<G>(V3{D.x + std::fmaf(IV.x, v, IU.x * u), D.y + std::fmaf(IV.y, v, IU.y * u),
                                            D.z + std::fmaf(IV.z, v, IU.z * u)})
                        : normalize(add(add(mul(IU, u), mul(IV, v)), D));
            Hit h{}; bool ovf = false;
            const uint64_t pp0 = pp, sp0 = sp_;
            bool hit = traverse<G>(cx, E, view, &h, &pp, &pt, &ovf, robust);
            rays++;
            float c[3] = {0.f, 0.f, 0.f};
            int32_t rp = -1; int8_t rs = -1;
            if (hit) {
                hits++;
                rp = int32_t(h.prim);
                const Tri& tr = cx.tris[h.prim];
                V3 normal = normalizeG<G>(tr.n);
                if (mode == 1) {                                             // render.hpp:123-125
                    c[0] = std::fabs(normal.x); c[1] = std::fabs(normal.y); c[2] = std::fabs(normal.z);
                } else {
                    float hu = h.u, hv = h.v;                                // render.hpp:127-135
                    float scale = -0.00001;
                    V3 p;
                    if (G) {                                                 // fma(n, scale, fma(w, p2, fma(v, p1, u p0)))
                        const float w = 1 - hu - hv;
                        const V3 p1 = tri_p1(tr), p2 = tri_p2(tr);
                        p = {std::fmaf(normal.x, scale, std::fmaf(w, p2.x, std::fmaf(hv, p1.x, hu * tr.p0.x))),
                             std::fmaf(normal.y, scale, std::fmaf(w, p2.y, std::fmaf(hv, p1.y, hu * tr.p0.y))),
                             std::fmaf(normal.z, scale, std::fmaf(w, p2.z, std::fmaf(hv, p1.z, hu * tr.p0.z)))};
                    } else {
                        p = add(add(mul(tr.p0, hu), mul(tri_p1(tr), hv)), mul(tri_p2(tr), 1 - hu - hv));
                        p = add(p, mul(normal, scale));
                    }
                    V3 sun_line = normalizeG<G>(sub(S, p));
                    Hit h2{};
                    bool sh = traverse<G>(cx, p, sun_line, &h2, &sp_, &st, &ovf, robust);   // render.hpp:136-138
                    rays++;
                    if (!sh) { smooth_shading<G>(sun_line, norms[h.prim], view, hu, hv, c); rs = 0; }
                    else { hits++; rs = 1; }
                }
            }
            if (ovf) ovf_any = 1;
            if (pixels) { pixels[index] = c[0]; pixels[index + 1] = c[1]; pixels[index + 2] = c[2]; }
            if (ppm) {
                size_t o = 3 * (W * (H - 1 - j) + i);
                ppm[o] = quantize(c[0]); ppm[o + 1] = quantize(c[1]); ppm[o + 2] = quantize(c[2]);
            }
            size_t pix = W * j + i;
            if (rec_prim) rec_prim[pix] = rp;
            if (rec_pairs) { rec_pairs[2 * pix] = uint32_t(pp - pp0); rec_pairs[2 * pix + 1] = uint32_t(sp_ - sp0); }
            if (rec_shadow) rec_shadow[pix] = rs;
            if (rec_tuv) { rec_tuv[3 * pix] = hit ? h.t : 0.f; rec_tuv[3 * pix + 1] = hit ? h.u : 0.f; rec_tuv[3 * pix + 2] = hit ? h.v : 0.f; }
        }
    }
    if (counts) { counts[0] = rays; counts[1] = hits; counts[2] = pp; counts[3] = pt; counts[4] = sp_; counts[5] = st; }
    if (ovf_any) { g_err = "traversal stack overflow (64 entries)"; return -4; }
    return 0;
}
}  // namespace

extern "C" int oracle_render(const float* tri48, const float* norm36, size_t n_tri, const uint32_t* nodes32, size_t n_nodes,
                             const uint64_t* prim64, const float eye[3], const float basis[9], const float sun[3], int mode,
                             size_t W, size_t H, float* pixels, uint8_t* ppm, int32_t* rec_prim, float* rec_tuv,
                             int8_t* rec_shadow, uint64_t counts[6], int threads, uint32_t* rec_pairs) {
    auto f = (mode & 0x20) ? render_impl<true> : render_impl<false>;
    return f(tri48, norm36, n_tri, nodes32, n_nodes, prim64, eye, basis, sun, mode & ~0x20, W, H, pixels, ppm,
             rec_prim, rec_tuv, rec_shadow, counts, threads, rec_pairs);
}
