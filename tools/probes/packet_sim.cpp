// Packet vs per-lane traversal step counts on the CPU (docs/EXPERIMENTS.md "Wave-wide packets").
// For every 8x8 tile of the first views of a bench step: the per-lane loops' wave iterations (the
// longest lane) and leaf trips (the longest lane's trip count per iteration), against a wave-wide
// masked packet's node visits and leaf trips -- closest hit over the BVH2 in each lane's own
// near-first order (lanes disagreeing on a node's near child split the mask), any-hit over a
// 4-wide collapse of it.  Plain float arithmetic: step counts, not the product's bits.
// Inputs: tools/packet_sim.py dumps the scene, BVH and views and runs this.
// Shadow-ray packet simulation: per-lane any-hit BVH4 (current batch kernel) vs wave-wide masked
// packet traversal over the same BVH4.  Counts wave iterations / triangle trips.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <cfloat>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>
static int popcount64(uint64_t x) { return __builtin_popcountll(x); }
struct V3 { float x, y, z; };
static V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V3 norm(V3 v) { float l = 1.f / std::sqrt(dot(v, v)); return v * l; }
struct Node { float b[6]; uint32_t cnt, first; };
struct Tri { V3 p0, e1, e2, n; };
std::vector<Tri> tris; std::vector<Node> nodes; std::vector<uint64_t> prim;
template <class T> std::vector<T> rd(const std::string& p) {
    FILE* f = fopen(p.c_str(), "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    std::vector<T> v(n / sizeof(T)); if (fread(v.data(), 1, n, f) != size_t(n)) v.clear(); fclose(f); return v; }
struct Ray { V3 o, d, inv; };
static Ray mk(V3 o, V3 d) { Ray r{o, d, {}}; auto si = [](float x) { return 1.f / (std::fabs(x) < FLT_EPSILON ? std::copysign(FLT_EPSILON, x) : x); };
    r.inv = {si(d.x), si(d.y), si(d.z)}; return r; }
static bool box(const Ray& r, const float* b, float tmax, float* ent = nullptr) {
    float tx0 = (b[0] - r.o.x) * r.inv.x, tx1 = (b[1] - r.o.x) * r.inv.x;
    float ty0 = (b[2] - r.o.y) * r.inv.y, ty1 = (b[3] - r.o.y) * r.inv.y;
    float tz0 = (b[4] - r.o.z) * r.inv.z, tz1 = (b[5] - r.o.z) * r.inv.z;
    float e = std::max(std::max(std::min(tx0, tx1), std::min(ty0, ty1)), std::max(std::min(tz0, tz1), 0.f));
    float x = std::min(std::min(std::max(tx0, tx1), std::max(ty0, ty1)), std::min(std::max(tz0, tz1), tmax));
    if (ent) *ent = e; return e <= x; }
static bool tri(const Tri& t, const Ray& r, float tmax, float& tt) {
    V3 c = t.p0 - r.o, rc = cross(r.d, c); float det = dot(t.n, r.d); float inv = 1.f / det;
    float u = dot(rc, t.e2) * inv, v = dot(rc, t.e1) * inv, w = 1 - u - v;
    if (u >= 0 && v >= 0 && w >= 0) { tt = dot(t.n, c) * inv; return tt >= 0 && tt <= tmax; } return false; }
// closest hit, BVH2
static bool closest(const Ray& r, uint32_t& best, float& bt) {
    bt = FLT_MAX; bool have = false; uint32_t stk[64]; int sp = 0; uint32_t cur = nodes[0].first;
    if (!box(r, nodes[0].b, bt)) return false;
    while (true) {
        const Node &L = nodes[cur], &R = nodes[cur + 1]; float el, er;
        bool hl = box(r, L.b, bt, &el), hr = box(r, R.b, bt, &er);
        if (hl && L.cnt) { for (uint32_t k = L.first; k < L.first + L.cnt; ++k) { float t; if (tri(tris[prim[k]], r, bt, t)) { bt = t; best = prim[k]; have = true; } } hl = false; }
        if (hr && R.cnt) { for (uint32_t k = R.first; k < R.first + R.cnt; ++k) { float t; if (tri(tris[prim[k]], r, bt, t)) { bt = t; best = prim[k]; have = true; } } hr = false; }
        if (hl && hr) { if (el > er) { stk[sp++] = L.first; cur = R.first; } else { stk[sp++] = R.first; cur = L.first; } }
        else if (hl) cur = L.first; else if (hr) cur = R.first;
        else { if (!sp) break; cur = stk[--sp]; }
    }
    return have; }
// BVH4: node = up to 4 BVH2 node indices
struct N4 { int n; uint32_t c[4]; };
std::vector<N4> n4; std::vector<int32_t> n4_of;   // bvh2 inner node (index of its first child pair) -> n4 index
static bool inside(const float* a, const float* b) { return a[0] >= b[0] && a[1] <= b[1] && a[2] >= b[2] && a[3] <= b[3] && a[4] >= b[4] && a[5] <= b[5]; }
static int build4(uint32_t node) {   // node: bvh2 inner node index; returns n4 index
    N4 q; q.n = 2; q.c[0] = nodes[node].first; q.c[1] = nodes[node].first + 1;
    bool grew = true;
    while (q.n < 4 && grew) { grew = false;
        for (int i = 0; i < q.n && q.n < 4; ++i) { const Node& c = nodes[q.c[i]];
            if (c.cnt) continue; const Node &a = nodes[c.first], &b = nodes[c.first + 1];
            if (inside(a.b, c.b) && inside(b.b, c.b)) { uint32_t f = c.first; q.c[i] = f; q.c[q.n++] = f + 1; grew = true; } } }
    int id = n4.size(); n4.push_back(q);
    return id; }
std::vector<int32_t> map4;   // bvh2 node -> n4 index (for inner children)
static void build_all() { map4.assign(nodes.size(), -1);
    std::vector<uint32_t> todo{0};
    while (!todo.empty()) { uint32_t v = todo.back(); todo.pop_back(); int id = build4(v); map4[v] = id;
        for (int i = 0; i < n4[id].n; ++i) if (!nodes[n4[id].c[i]].cnt) todo.push_back(n4[id].c[i]); } }
// per-lane any-hit: returns steps; tri counts per step appended
static bool anyhit(const Ray& r, std::vector<int>& per_step) {
    uint32_t stk[256]; int sp = 0; int cur = map4[0];
    if (!box(r, nodes[0].b, FLT_MAX)) { per_step.push_back(0); return false; }
    while (true) { const N4& q = n4[cur]; int trips = 0; int inner[4], ni = 0; bool occ = false;
        for (int i = 0; i < q.n && !occ; ++i) { const Node& c = nodes[q.c[i]]; if (!box(r, c.b, FLT_MAX)) continue;
            if (c.cnt) { for (uint32_t k = c.first; k < c.first + c.cnt; ++k) { ++trips; float t; if (tri(tris[prim[k]], r, FLT_MAX, t)) { occ = true; break; } } }
            else inner[ni++] = map4[q.c[i]]; }
        per_step.push_back(trips); if (occ) return true;
        if (ni) { for (int i = 1; i < ni; ++i) stk[sp++] = inner[i]; cur = inner[0]; }
        else { if (!sp) return false; cur = stk[--sp]; } } }
// packet any-hit over lanes (mask): returns visits, trips
static void packet(const std::vector<Ray>& rays, uint64_t mask, long& visits, long& trips, long& lane_node_tests, long& lane_tri_tests) {
    uint64_t occluded = 0; struct E { int n; uint64_t m; }; std::vector<E> stk; int cur = map4[0]; uint64_t m = 0;
    for (int l = 0; l < 64; ++l) if ((mask >> l & 1) && box(rays[l], nodes[0].b, FLT_MAX)) m |= 1ull << l;
    visits++; if (!m) return;
    while (true) { const N4& q = n4[cur]; visits++; uint64_t cm[4] = {0, 0, 0, 0};
        for (int i = 0; i < q.n; ++i) for (int l = 0; l < 64; ++l) if (m >> l & 1) { lane_node_tests++; if (box(rays[l], nodes[q.c[i]].b, FLT_MAX)) cm[i] |= 1ull << l; }
        int inner[4]; uint64_t im[4]; int ni = 0;
        for (int i = 0; i < q.n; ++i) { if (!cm[i]) continue; const Node& c = nodes[q.c[i]];
            if (c.cnt) { uint64_t lm = cm[i] & ~occluded;
                for (uint32_t k = c.first; k < c.first + c.cnt && lm; ++k) { ++trips;
                    for (int l = 0; l < 64; ++l) if (lm >> l & 1) { lane_tri_tests++; float t; if (tri(tris[prim[k]], rays[l], FLT_MAX, t)) { occluded |= 1ull << l; } }
                    lm &= ~occluded; } }
            else { inner[ni] = map4[q.c[i]]; im[ni++] = cm[i]; } }
        int best = -1; for (int i = 0; i < ni; ++i) { uint64_t mm = im[i] & ~occluded; if (!mm) continue; if (best < 0) { best = i; } else stk.push_back({inner[i], mm}); }
        if (best >= 0) { cur = inner[best]; m = im[best] & ~occluded; continue; }
        bool got = false; while (!stk.empty()) { E e = stk.back(); stk.pop_back(); e.m &= ~occluded; if (e.m) { cur = e.n; m = e.m; got = true; break; } }
        if (!got) break; } }

// primary: per-lane BVH2 closest hit in reference order, recording leaf tests per step
static int prim_lane(const Ray& r, std::vector<int>& per_step, uint32_t& best, float& bt) {
    bt = FLT_MAX; uint32_t stk[64]; int sp = 0; uint32_t cur = nodes[0].first; int steps = 0;
    while (true) { ++steps;
        const Node &L = nodes[cur], &R = nodes[cur + 1]; float el, er;
        bool hl = box(r, L.b, bt, &el), hr = box(r, R.b, bt, &er); int trips = 0;
        bool gl = hl && !L.cnt, gr = hr && !R.cnt;
        if (hl && L.cnt) for (uint32_t k = L.first; k < L.first + L.cnt; ++k) { ++trips; float t; if (tri(tris[prim[k]], r, bt, t)) { bt = t; best = prim[k]; } }
        if (hr && R.cnt) for (uint32_t k = R.first; k < R.first + R.cnt; ++k) { ++trips; float t; if (tri(tris[prim[k]], r, bt, t)) { bt = t; best = prim[k]; } }
        per_step.push_back(trips);
        if (gl && gr) { if (el > er) { stk[sp++] = L.first; cur = R.first; } else { stk[sp++] = R.first; cur = L.first; } }
        else if (gl) cur = L.first; else if (gr) cur = R.first;
        else { if (!sp) break; cur = stk[--sp]; } }
    return steps; }
static void prim_packet(const std::vector<Ray>& rays, uint64_t mask, long& visits, long& trips, long& splits) {
    float bt[64]; for (int l = 0; l < 64; ++l) bt[l] = FLT_MAX;
    struct E { uint32_t n; uint64_t m; }; std::vector<E> stk; uint32_t cur = nodes[0].first; uint64_t m = mask;
    while (true) { visits++; const Node &L = nodes[cur], &R = nodes[cur + 1];
        uint64_t ml = 0, mr = 0, sw = 0;
        for (int l = 0; l < 64; ++l) if (m >> l & 1) { float el, er; bool hl = box(rays[l], L.b, bt[l], &el), hr = box(rays[l], R.b, bt[l], &er);
            if (hl) ml |= 1ull << l; if (hr) mr |= 1ull << l; if (el > er) sw |= 1ull << l; }
        if (L.cnt && ml) for (uint32_t k = L.first; k < L.first + L.cnt; ++k) { ++trips; for (int l = 0; l < 64; ++l) if (ml >> l & 1) { float t; if (tri(tris[prim[k]], rays[l], bt[l], t)) bt[l] = t; } }
        if (R.cnt && mr) for (uint32_t k = R.first; k < R.first + R.cnt; ++k) { ++trips; for (int l = 0; l < 64; ++l) if (mr >> l & 1) { float t; if (tri(tris[prim[k]], rays[l], bt[l], t)) bt[l] = t; } }
        uint64_t gl = L.cnt ? 0 : ml, gr = R.cnt ? 0 : mr;
        uint64_t both = gl & gr, onlyl = gl & ~gr, onlyr = gr & ~gl;
        uint64_t A = both & ~sw, B = both & sw;   // A: left first, B: right first
        // lanes: A -> L then R ; B -> R then L ; onlyl -> L ; onlyr -> R
        // packet: go to the child with the larger mask first
        uint64_t goL = A | onlyl, goR = B | onlyr;   // first visits
        if (A && B) splits++;
        if (!goL && !goR) { bool got = false; while (!stk.empty()) { E e = stk.back(); stk.pop_back(); if (e.m) { cur = e.n; m = e.m; got = true; break; } } if (!got) break; continue; }
        // order: choose first = L with goL; pushes: (L, B) pushed first (deepest), (R, A) ... general:
        // if goL first: push (L_again? no) -> stack: [.., (L,B), (R, goR | A)] then go L with goL
        if (popcount64(goL) >= popcount64(goR)) { if (B) stk.push_back({L.first, B}); if (goR | A) stk.push_back({R.first, goR | A}); cur = L.first; m = goL; if (!goL) { E e = stk.back(); stk.pop_back(); cur = e.n; m = e.m; } }
        else { if (A) stk.push_back({R.first, A}); if (goL | B) stk.push_back({L.first, goL | B}); cur = R.first; m = goR; if (!goR) { E e = stk.back(); stk.pop_back(); cur = e.n; m = e.m; } }
    } }

int main(int argc, char** argv) {
    std::string base = argv[1]; int W = atoi(argv[2]), H = atoi(argv[3]), F = atoi(argv[4]); int fmax = argc > 5 ? atoi(argv[5]) : F;
    auto tf = rd<float>(base + ".tri"); tris.resize(tf.size() / 12); for (size_t i = 0; i < tris.size(); ++i) { const float* p = &tf[12 * i]; tris[i] = {{p[0], p[1], p[2]}, {p[3], p[4], p[5]}, {p[6], p[7], p[8]}, {p[9], p[10], p[11]}}; }
    auto nu = rd<uint32_t>(base + ".nodes"); nodes.resize(nu.size() / 8); memcpy(nodes.data(), nu.data(), nu.size() * 4);
    prim = rd<uint64_t>(base + ".prim"); auto vw = rd<float>(base + ".views");
    build_all(); printf("n4 nodes %zu (bvh2 %zu)\n", n4.size(), nodes.size());
    long ptiles = 0, p_iters = 0, p_trips = 0, pp_visits = 0, pp_trips = 0, pp_splits = 0; long cur_iters = 0, cur_trips = 0, pk_visits = 0, pk_trips = 0, tiles_sh = 0, lane_steps = 0, lnt = 0, ltt = 0, sh_rays = 0;
    for (int f = 0; f < fmax; ++f) { const float* b = &vw[12 * f]; const float* s = &vw[12 * F + 3 * f];
        V3 eye{b[0], b[1], b[2]}, dir{b[3], b[4], b[5]}, iu{b[6], b[7], b[8]}, iv{b[9], b[10], b[11]}, sun{s[0], s[1], s[2]};
        for (int ty = 0; ty < (H + 7) / 8; ++ty) for (int tx = 0; tx < (W + 7) / 8; ++tx) {
            { std::vector<Ray> pr(64); uint64_t pm = 0; std::vector<std::vector<int>> pps(64); int mx = 0;
              for (int l = 0; l < 64; ++l) { int i = tx * 8 + (l & 7), j = ty * 8 + (l >> 3); if (i >= W || j >= H) continue;
                float u = 2 * (i + 0.5f) / W - 1, v = 2 * (j + 0.5f) / H - 1; V3 d = norm(iu * u + iv * v + dir); pr[l] = mk(eye, d);
                if (!box(pr[l], nodes[0].b, FLT_MAX)) continue; pm |= 1ull << l; uint32_t b; float t; prim_lane(pr[l], pps[l], b, t); mx = std::max<int>(mx, pps[l].size()); }
              if (pm) { ptiles++; p_iters += mx; for (int j = 0; j < mx; ++j) { int m = 0; for (int l = 0; l < 64; ++l) if ((pm >> l & 1) && j < (int)pps[l].size()) m = std::max(m, pps[l][j]); p_trips += m; }
                prim_packet(pr, pm, pp_visits, pp_trips, pp_splits); } }
            std::vector<Ray> rays(64); uint64_t mask = 0; std::vector<std::vector<int>> ps(64);
            for (int l = 0; l < 64; ++l) { int i = tx * 8 + (l & 7), j = ty * 8 + (l >> 3); if (i >= W || j >= H) continue;
                float u = 2 * (i + 0.5f) / W - 1, v = 2 * (j + 0.5f) / H - 1; V3 d = norm(iu * u + iv * v + dir);
                Ray r = mk(eye, d); uint32_t hp; float t; if (!closest(r, hp, t)) continue;
                V3 p = eye + d * t; V3 n = norm(tris[hp].n); p = p + n * -0.00001f; V3 sd = norm(sun - p);
                rays[l] = mk(p, sd); mask |= 1ull << l; }
            if (!mask) continue; tiles_sh++;
            int mx = 0; for (int l = 0; l < 64; ++l) if (mask >> l & 1) { anyhit(rays[l], ps[l]); mx = std::max<int>(mx, ps[l].size()); lane_steps += ps[l].size(); sh_rays++; }
            cur_iters += mx; for (int j = 0; j < mx; ++j) { int m = 0; for (int l = 0; l < 64; ++l) if ((mask >> l & 1) && j < (int)ps[l].size()) m = std::max(m, ps[l][j]); cur_trips += m; }
            packet(rays, mask, pk_visits, pk_trips, lnt, ltt); } }
    printf("PRIMARY tiles (root hit) %ld: per-lane iters %.1f/tile trips %.1f/tile | packet visits %.1f/tile trips %.1f/tile splits %.1f/tile\n", ptiles, double(p_iters)/ptiles, double(p_trips)/ptiles, double(pp_visits)/ptiles, double(pp_trips)/ptiles, double(pp_splits)/ptiles);
    printf("tiles with shadow rays %ld, shadow rays %ld (%.1f per tile)\n", tiles_sh, sh_rays, double(sh_rays) / tiles_sh);
    printf("per-lane: wave iterations %ld (%.1f/tile), leaf trips %ld (%.1f/tile), lane steps %.1f per ray\n", cur_iters, double(cur_iters) / tiles_sh, cur_trips, double(cur_trips) / tiles_sh, double(lane_steps) / sh_rays);
    printf("packet:   node visits %ld (%.1f/tile), leaf trips %ld (%.1f/tile); lane node tests %.1f/ray, lane tri tests %.1f/ray\n", pk_visits, double(pk_visits) / tiles_sh, pk_trips, double(pk_trips) / tiles_sh, double(lnt) / sh_rays / 4, double(ltt) / sh_rays);
}
