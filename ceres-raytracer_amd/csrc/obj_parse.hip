// obj_parse.hip -- obj::load_from_stream (obj_norms.hpp:57-118) and rotate_triangles
// (render.hpp:24-44) on gfx950.
//
// Produces the reference loader's exact bits: the same triangles (fan triangulation of each
// face, Triangle(p0, p1, p2) = {p0, p0 - p1, p2 - p0, cross(e1, e2)}, triangle.hpp:30-34) and
// the same per-corner vertex normals -- area-weighted sums accumulated in FACE ORDER
// (obj_norms.hpp:91-94) and normalised (:109-111).  Text rules follow the reference exactly:
// getline into a 1024-byte buffer (a longer line stops reading, the host path's rule), leading
// isspace skipped, '#' and empty lines ignored, trailing isspace trimmed, "v" + isspace ->
// three strtof, "f" + isspace -> read_index loop (i, i/t, i//n, i/t/n, negative = relative to
// the vertices read so far); numbers via glibc-exact strtof/strtol (strtof_exact.hpp).
//
// Pipeline (one thread per byte chunk, then one per line, then one per triangle / vertex):
//   newline positions (per-block counts + scan) -> line classes and triangle counts ->
//   scans (vertex ids, triangle slots) -> vertex parse + face corners -> triangles ->
//   stable radix sort of (vertex, corner) -> per-vertex ordered normal sums -> tri_norms.
// The float sum order per vertex is the reference's (corner index order = face order), so the
// normals are bit-identical, not merely close.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ceres_render.h"
#include "ceres_types.hpp"
#include "dev_scan.hpp"
#include "host_common.hpp"
#include "strtof_exact.hpp"

#pragma clang fp contract(off)

namespace ceres {
namespace objdev {

using namespace txt;
using namespace devscan;

constexpr int kNlChunk = 4096;            // bytes per newline-scan workgroup (256 threads x 16)
constexpr long kMaxLine = 1024;           // istream::getline(line, 1024): at most 1023 characters

struct LineInfo { uint32_t start, end; };  // [start, end) before any NUL cut

__device__ __forceinline__ LineInfo line_of(const uint32_t* nlpos, uint32_t n_nl, uint32_t k, uint32_t len) {
    return {k == 0 ? 0u : nlpos[k - 1] + 1u, k < n_nl ? nlpos[k] : len};
}

// The reference's view of one line: C string from the first non-space character to the
// trimmed end (remove_eol keeps index 0), NUL bytes ending the string like strlen does.
struct LineView {
    Cursor c;          // [ptr, trimmed end)
    bool skip;         // empty or comment
};
__device__ LineView view_line(const char* text, LineInfo li) {
    const char* p = text + li.start;
    const char* e = text + li.end;
    for (const char* q = p; q < e; ++q) if (*q == '\0') { e = q; break; }
    while (p < e && is_space(*p)) ++p;
    LineView v{{p, e}, false};
    if (p == e || *p == '#') { v.skip = true; return v; }
    long i = long(e - p) - 1;
    while (i > 0 && is_space(p[i])) --i;
    v.c.e = p + i + 1;
    return v;
}

// read_index (obj_norms.hpp:30-53): returns false at the end of the list; `pos` advances.
__device__ bool read_index(Cursor line, long& pos, int& index) {
    long b = pos;
    while (is_space(line.at(b))) ++b;
    if (!is_digit(line.at(b)) && line.at(b) != '-') return false;
    long v;
    b += strtol10(Cursor{line.p + b, line.e}, &v);
    while (is_space(line.at(b))) ++b;
    if (line.at(b) == '/') {
        ++b;
        long t;
        if (line.at(b) != '/') b += strtol10(Cursor{line.p + b, line.e}, &t);
        while (is_space(line.at(b))) ++b;
        if (line.at(b) == '/') { ++b; b += strtol10(Cursor{line.p + b, line.e}, &t); }
    }
    pos = b;
    index = int(uint32_t(uint64_t(v)));                      // `int index = std::strtol(...)`
    return true;
}

// j = index < 0 ? vertices.size() + index : index - 1, valid iff j < vertices.size()
__device__ __forceinline__ bool resolve(int index, uint32_t nverts, uint32_t& j) {
    const uint64_t jj = index < 0 ? uint64_t(nverts) + uint64_t(int64_t(index)) : uint64_t(int64_t(index) - 1);
    j = uint32_t(jj);
    return jj < nverts;
}

__global__ void __launch_bounds__(256) k_nl_count(const char* __restrict__ text, uint32_t len, uint32_t* __restrict__ counts) {
    __shared__ uint32_t sh[264];
    const uint32_t base = blockIdx.x * uint32_t(kNlChunk) + threadIdx.x * 16u;
    uint32_t c = 0;
    for (int k = 0; k < 16; ++k) c += (base + k < len && text[base + k] == '\n') ? 1u : 0u;
    uint32_t total;
    (void)block_exclusive_scan_256(c, sh, total);
    if (threadIdx.x == 0) counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(256) k_nl_emit(const char* __restrict__ text, uint32_t len, const uint32_t* __restrict__ offs,
                                                 uint32_t* __restrict__ nlpos) {
    __shared__ uint32_t sh[264];
    const uint32_t base = blockIdx.x * uint32_t(kNlChunk) + threadIdx.x * 16u;
    uint32_t c = 0;
    char b[16];
    for (int k = 0; k < 16; ++k) { b[k] = base + k < len ? text[base + k] : 0; c += b[k] == '\n'; }
    uint32_t total;
    uint32_t o = offs[blockIdx.x] + block_exclusive_scan_256(c, sh, total);
    for (int k = 0; k < 16; ++k) if (b[k] == '\n') nlpos[o++] = base + k;
}

// class of each line: vertex flag, triangles produced; first over-long line; bad face index 0
__global__ void __launch_bounds__(256) k_classify(const char* __restrict__ text, uint32_t len, const uint32_t* __restrict__ nlpos,
                                                  uint32_t n_nl, uint32_t n_lines, uint32_t* __restrict__ vflag,
                                                  uint32_t* __restrict__ tcount, uint32_t* __restrict__ first_long) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n_lines) return;
    const LineInfo li = line_of(nlpos, n_nl, k, len);
    uint32_t vf = 0, tc = 0;
    if (long(li.end) - long(li.start) > kMaxLine - 1) {
        atomicMin(first_long, k);
    } else {
        const LineView v = view_line(text, li);
        if (!v.skip) {
            const char c0 = v.c.at(0), c1 = v.c.at(1);
            if (c0 == 'v' && is_space(c1)) {
                vf = 1;
            } else if (c0 == 'f' && is_space(c1)) {
                long pos = 2;
                int idx;
                uint32_t n = 0;
                while (read_index(v.c, pos, idx)) {
                    ++n;
                    if (idx == 0) break;        // index 0 never resolves (j = -1): the parse pass reports it
                }
                tc = n >= 3 ? n - 2 : 0;
            }
        }
    }
    vflag[k] = vf;
    tcount[k] = tc;
}

// vertices (three strtof, obj_norms.hpp:78-80) and face corners (fan, :84-102)
__global__ void __launch_bounds__(256) k_parse(const char* __restrict__ text, uint32_t len, const uint32_t* __restrict__ nlpos,
                                               uint32_t n_nl, uint32_t n_lines, const uint32_t* __restrict__ vidx,
                                               const uint32_t* __restrict__ tbase, float* __restrict__ verts,
                                               uint32_t* __restrict__ corners, unsigned long long* __restrict__ bad) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n_lines) return;
    const LineInfo li = line_of(nlpos, n_nl, k, len);
    const LineView v = view_line(text, li);
    if (v.skip) return;
    const char c0 = v.c.at(0), c1 = v.c.at(1);
    if (c0 == 'v' && is_space(c1)) {
        const uint32_t id = vidx[k];
        long pos = 1;
        float xyz[3];
        for (int a = 0; a < 3; ++a) pos += strtof_exact(Cursor{v.c.p + pos, v.c.e}, &xyz[a]);
        verts[3 * size_t(id)] = xyz[0]; verts[3 * size_t(id) + 1] = xyz[1]; verts[3 * size_t(id) + 2] = xyz[2];
    } else if (c0 == 'f' && is_space(c1)) {
        const uint32_t nverts = vidx[k];                 // vertices read before this line
        uint32_t t = tbase[k];
        long pos = 2;
        int idx;
        uint32_t first = 0, prev = 0;
        for (uint32_t n = 0; read_index(v.c, pos, idx); ++n) {
            uint32_t j;
            if (!resolve(idx, nverts, j)) {
                // first bad reference in file order: (line << 32) | (index as u32)
                atomicMin(bad, (static_cast<unsigned long long>(k) << 32) | uint32_t(idx));
                return;
            }
            if (n == 0) first = j;
            else if (n == 1) prev = j;
            else {
                corners[3 * size_t(t)] = first; corners[3 * size_t(t) + 1] = prev; corners[3 * size_t(t) + 2] = j;
                ++t;
                prev = j;
            }
        }
    }
}

// Float ops with x86 SSE NaN results (the reference runs on the host): an invalid operation on
// non-NaN operands (0 * inf, inf - inf) yields the default NaN 0xffc00000 (AMD returns
// 0x7fc00000); a NaN operand propagates quieted, the first one first.  Degenerate triangles
// (zero-area normal sums -> 0 * inf) hit this, so the normals stay bit-identical.
__device__ __forceinline__ float x86_nan(float r, float a, float b) {
    if (r == r) return r;
    if (a != a) return __uint_as_float(__float_as_uint(a) | 0x00400000u);
    if (b != b) return __uint_as_float(__float_as_uint(b) | 0x00400000u);
    return __uint_as_float(0xffc00000u);
}
__device__ __forceinline__ float fadd(float a, float b) { return x86_nan(a + b, a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return x86_nan(a - b, a, b); }
__device__ __forceinline__ float fmul(float a, float b) { return x86_nan(a * b, a, b); }
__device__ __forceinline__ float fdiv(float a, float b) { return x86_nan(a / b, a, b); }

// fused a*b + c with the same NaN convention (x86 FMA: the first NaN operand, in a, b, c order --
// the operand order of GCC's vfmadd form is assumed; only NaN/inf OBJ coordinates can reach it)
__device__ __forceinline__ float ffma(float a, float b, float c) {
    const float r = fmaf(a, b, c);
    if (r == r) return r;
    if (a != a) return __uint_as_float(__float_as_uint(a) | 0x00400000u);
    return x86_nan(r, b, c);
}

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return {fsub(a.x, b.x), fsub(a.y, b.y), fsub(a.z, b.z)}; }
// cross (vector.hpp:159-167); G: the reference CMake build's contraction fma(a_j, b_k, -(a_k b_j))
template <bool G>
__device__ __forceinline__ F3 cross(F3 a, F3 b) {
    if (G) return {ffma(a.y, b.z, -fmul(a.z, b.y)), ffma(a.z, b.x, -fmul(a.x, b.z)), ffma(a.x, b.y, -fmul(a.y, b.x))};
    return {fsub(fmul(a.y, b.z), fmul(a.z, b.y)), fsub(fmul(a.z, b.x), fmul(a.x, b.z)), fsub(fmul(a.x, b.y), fmul(a.y, b.x))};
}
__device__ __forceinline__ F3 load3(const float* p) { return {p[0], p[1], p[2]}; }

// Triangle(p0, p1, p2) (triangle.hpp:30-34); corner values for the normal sort
template <bool G>
__global__ void __launch_bounds__(256) k_tris(const float* __restrict__ verts, const uint32_t* __restrict__ corners, uint32_t n_tri,
                                              Tri48* __restrict__ tris, uint32_t* __restrict__ cidx,
                                              uint32_t* __restrict__ vcount) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_tri) return;
    const uint32_t a = corners[3 * size_t(t)], b = corners[3 * size_t(t) + 1], c = corners[3 * size_t(t) + 2];
    const F3 p0 = load3(verts + 3 * size_t(a)), p1 = load3(verts + 3 * size_t(b)), p2 = load3(verts + 3 * size_t(c));
    const F3 e1 = sub(p0, p1), e2 = sub(p2, p0), n = cross<G>(e1, e2);
    tris[t] = Tri48{{p0.x, p0.y, p0.z}, {e1.x, e1.y, e1.z}, {e2.x, e2.y, e2.z}, {n.x, n.y, n.z}};
    for (int k = 0; k < 3; ++k) { cidx[3 * size_t(t) + k] = 3 * t + k; }
    atomicAdd(&vcount[a], 1u); atomicAdd(&vcount[b], 1u); atomicAdd(&vcount[c], 1u);
}

// normals[v] += n in face order, then normalize (obj_norms.hpp:91-94, 109-111); G: the dot of
// normalize contracted as fma(z, z, fma(x, x, y y))
template <bool G>
__global__ void __launch_bounds__(256) k_vnorm(const uint32_t* __restrict__ vstart, const uint32_t* __restrict__ sorted_c,
                                               const Tri48* __restrict__ tris, uint32_t nverts, float* __restrict__ vnorm) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= nverts) return;
    float x = 0.f, y = 0.f, z = 0.f;
    for (uint32_t i = vstart[v]; i < vstart[v + 1]; ++i) {
        const Tri48& t = tris[sorted_c[i] / 3u];
        x = fadd(x, t.n[0]); y = fadd(y, t.n[1]); z = fadd(z, t.n[2]);
    }
    float s;
    if (G) {
        s = ffma(z, z, ffma(x, x, fmul(y, y)));
    } else {
        s = fmul(x, x);
        s = fadd(s, fmul(y, y));
        s = fadd(s, fmul(z, z));
    }
    const float r = sqrtf(s);                              // sqrt of a NaN propagates; s >= 0 otherwise
    const float inv = fdiv(1.0f, x86_nan(r, s, s));
    vnorm[3 * size_t(v)] = fmul(x, inv); vnorm[3 * size_t(v) + 1] = fmul(y, inv); vnorm[3 * size_t(v) + 2] = fmul(z, inv);
}

__global__ void __launch_bounds__(256) k_trinorm(const uint32_t* __restrict__ corners, const float* __restrict__ vnorm, uint32_t n_tri,
                                                 float* __restrict__ norm36) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= n_tri) return;
    for (int k = 0; k < 3; ++k) {
        const uint32_t v = corners[3 * size_t(t) + k];
        for (int a = 0; a < 3; ++a) norm36[9 * size_t(t) + 3 * k + a] = vnorm[3 * size_t(v) + a];
    }
}

// rotate_triangles<Axis> (render.hpp:24-44): rebuild each Triangle from rotated p0, p1(), p2();
// G: each rotated coordinate's first product fused (p1 c - p2 s -> fma(p1, c, -(p2 s)), ...)
template <bool G>
__global__ void __launch_bounds__(256) k_rotate(Tri48* __restrict__ tris, uint32_t n_tri, int axis, float c, float s) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n_tri) return;
    Tri48 t = tris[i];
    const F3 p0 = load3(t.p0), e1 = load3(t.e1), e2 = load3(t.e2);
    const F3 q[3] = {p0, sub(p0, e1), {fadd(p0.x, e2.x), fadd(p0.y, e2.y), fadd(p0.z, e2.z)}};
    F3 r[3];
    for (int k = 0; k < 3; ++k) {
        const F3 p = q[k];
        auto mad = [&](float a, float b, float x, float y, bool minus) {   // a*b -/+ x*y
            if (G) return ffma(a, b, minus ? -fmul(x, y) : fmul(x, y));
            return minus ? fsub(fmul(a, b), fmul(x, y)) : fadd(fmul(a, b), fmul(x, y));
        };
        if (axis == 0) r[k] = {p.x, mad(p.y, c, p.z, s, true), mad(p.y, s, p.z, c, false)};
        else if (axis == 1) r[k] = {mad(p.x, c, p.z, s, false), p.y, mad(-p.x, s, p.z, c, false)};
        else r[k] = {mad(p.x, c, p.y, s, true), mad(p.x, s, p.y, c, false), p.z};
    }
    const F3 ne1 = sub(r[0], r[1]), ne2 = sub(r[2], r[0]), n = cross<G>(ne1, ne2);
    tris[i] = Tri48{{r[0].x, r[0].y, r[0].z}, {ne1.x, ne1.y, ne1.z}, {ne2.x, ne2.y, ne2.z}, {n.x, n.y, n.z}};
}

}  // namespace objdev
}  // namespace ceres

using namespace ceres;
using namespace ceres::objdev;

namespace {

#define OBJ_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) { rc = set_error(CERES_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); goto done; } \
    } while (0)

template <class T>
hipError_t dalloc(T** p, size_t count, hipStream_t s) {
    return hipMallocAsync(reinterpret_cast<void**>(p), std::max<size_t>(count, 1) * sizeof(T), s);
}

}  // namespace

extern "C" {

void ceres_device_free(void* d_ptr) {
    if (d_ptr) (void)hipFree(d_ptr);
}

int ceres_rotate_triangles_device_arith(float* d_tri48, size_t n_tri, int axis, float degrees, void* stream, int arith) {
    if ((!d_tri48 && n_tri) || axis < 0 || axis > 2) return set_error(CERES_EINVAL, "ceres_rotate_triangles_device: bad argument");
    if (arith != CERES_ARITH_EXACT && arith != CERES_ARITH_FMA) return set_error(CERES_EINVAL, "unknown arithmetic %d", arith);
    if (n_tri > 0xffffffffu) return set_error(CERES_EUNSUPPORTED, "too many triangles");
    if (!n_tri) return CERES_OK;
    // the angle's cos/sin on the host, as the reference evaluates them (render.hpp:27-28)
    const float pi = float(3.14159265359);
    const float c = std::cos(degrees * pi / float(180));
    const float s = std::sin(degrees * pi / float(180));
    if (arith == CERES_ARITH_FMA)
        hipLaunchKernelGGL(k_rotate<true>, dim3((n_tri + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                           reinterpret_cast<Tri48*>(d_tri48), uint32_t(n_tri), axis, c, s);
    else
        hipLaunchKernelGGL(k_rotate<false>, dim3((n_tri + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                           reinterpret_cast<Tri48*>(d_tri48), uint32_t(n_tri), axis, c, s);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CERES_OK : set_error(CERES_EHIP, "k_rotate: %s", hipGetErrorString(e));
}

int ceres_rotate_triangles_device(float* d_tri48, size_t n_tri, int axis, float degrees, void* stream) {
    return ceres_rotate_triangles_device_arith(d_tri48, n_tri, axis, degrees, stream, CERES_ARITH_EXACT);
}

// obj::load_from_stream on device text [d_text, d_text + len).  Outputs are hipMalloc'd device
// arrays (free with ceres_device_free); an empty mesh returns n_tri = 0 and NULL arrays.
int ceres_obj_parse_device_arith(const char* d_text, size_t len, float** d_tri48, float** d_norm36, size_t* n_tri,
                                 void* stream_, int arith) {
    if ((!d_text && len) || !d_tri48 || !d_norm36 || !n_tri) return set_error(CERES_EINVAL, "ceres_obj_parse_device: null argument");
    if (arith != CERES_ARITH_EXACT && arith != CERES_ARITH_FMA) return set_error(CERES_EINVAL, "unknown arithmetic %d", arith);
    *d_tri48 = *d_norm36 = nullptr;
    *n_tri = 0;
    if (len >= 0xffffffffu) return set_error(CERES_EUNSUPPORTED, "OBJ text of 4 GiB or more");
    if (len == 0) return CERES_OK;
    hipStream_t stream = static_cast<hipStream_t>(stream_);
    const uint32_t L32 = uint32_t(len);
    const uint32_t nblk = (L32 + kNlChunk - 1) / kNlChunk;
    int rc = CERES_OK;
    uint32_t *counts = nullptr, *offs = nullptr, *part = nullptr, *nlpos = nullptr, *vflag = nullptr, *tcount = nullptr;
    uint32_t *vidx = nullptr, *tbase = nullptr, *first_long = nullptr, *corners = nullptr, *cidx = nullptr, *ckey = nullptr;
    uint32_t *skey = nullptr, *sval = nullptr, *vcount = nullptr, *vstart = nullptr;
    unsigned long long* bad = nullptr;
    float *verts = nullptr, *vnorm = nullptr;
    Tri48* tris = nullptr;
    float* norm36 = nullptr;
    void* sort_tmp = nullptr;
    uint32_t n_nl = 0, n_lines = 0, h_first_long = 0, nverts = 0, ntris = 0;
    unsigned long long h_bad = 0;
    char last = 0;
    OBJ_TRY(dalloc(&counts, nblk, stream));
    OBJ_TRY(dalloc(&offs, nblk + 1, stream));
    OBJ_TRY(dalloc(&part, scan_blocks(std::max(nblk, 1u)) + 2, stream));
    hipLaunchKernelGGL(k_nl_count, dim3(nblk), dim3(256), 0, stream, d_text, L32, counts);
    OBJ_TRY(hipGetLastError());
    OBJ_TRY(exclusive_scan(counts, nblk, offs, part, stream));
    OBJ_TRY(hipMemcpyAsync(&n_nl, offs + nblk, 4, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipMemcpyAsync(&last, d_text + len - 1, 1, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipStreamSynchronize(stream));
    n_lines = n_nl + (last != '\n' ? 1u : 0u);
    OBJ_TRY(dalloc(&nlpos, n_nl, stream));
    hipLaunchKernelGGL(k_nl_emit, dim3(nblk), dim3(256), 0, stream, d_text, L32, offs, nlpos);
    OBJ_TRY(dalloc(&vflag, n_lines, stream));
    OBJ_TRY(dalloc(&tcount, n_lines, stream));
    OBJ_TRY(dalloc(&first_long, 1, stream));
    OBJ_TRY(hipMemsetAsync(first_long, 0xff, 4, stream));
    hipLaunchKernelGGL(k_classify, dim3((n_lines + 255) / 256), dim3(256), 0, stream, d_text, L32, nlpos, n_nl, n_lines,
                       vflag, tcount, first_long);
    OBJ_TRY(hipGetLastError());
    OBJ_TRY(hipMemcpyAsync(&h_first_long, first_long, 4, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipStreamSynchronize(stream));
    n_lines = std::min(n_lines, h_first_long);            // getline fails on an over-long line: reading stops
    OBJ_TRY(dalloc(&vidx, n_lines + 1, stream));
    OBJ_TRY(dalloc(&tbase, n_lines + 1, stream));
    OBJ_TRY(hipFreeAsync(part, stream));
    part = nullptr;
    OBJ_TRY(dalloc(&part, scan_blocks(std::max(n_lines, 1u)) + 2, stream));
    OBJ_TRY(exclusive_scan(vflag, n_lines, vidx, part, stream));
    OBJ_TRY(exclusive_scan(tcount, n_lines, tbase, part, stream));
    OBJ_TRY(hipMemcpyAsync(&nverts, vidx + n_lines, 4, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipMemcpyAsync(&ntris, tbase + n_lines, 4, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipStreamSynchronize(stream));
    OBJ_TRY(dalloc(&verts, 3 * size_t(nverts), stream));
    OBJ_TRY(dalloc(&corners, 3 * size_t(ntris), stream));
    OBJ_TRY(dalloc(&bad, 1, stream));
    OBJ_TRY(hipMemsetAsync(bad, 0xff, 8, stream));
    if (n_lines)
        hipLaunchKernelGGL(k_parse, dim3((n_lines + 255) / 256), dim3(256), 0, stream, d_text, L32, nlpos, n_nl, n_lines,
                           vidx, tbase, verts, corners, bad);
    OBJ_TRY(hipGetLastError());
    OBJ_TRY(hipMemcpyAsync(&h_bad, bad, 8, hipMemcpyDeviceToHost, stream));
    OBJ_TRY(hipStreamSynchronize(stream));
    if (h_bad != ~0ull) {
        rc = set_error(CERES_EIO, "OBJ face references vertex %d (line %llu)", int(uint32_t(h_bad)), (h_bad >> 32) + 1);
        goto done;
    }
    if (ntris) {
        // outputs outlive the call: plain hipMalloc (ceres_device_free = hipFree)
        OBJ_TRY(hipMalloc(&tris, size_t(ntris) * sizeof(Tri48)));
        OBJ_TRY(hipMalloc(&norm36, 36 * size_t(ntris)));
        OBJ_TRY(dalloc(&cidx, 3 * size_t(ntris), stream));
        OBJ_TRY(dalloc(&sval, 3 * size_t(ntris), stream));
        OBJ_TRY(dalloc(&skey, 3 * size_t(ntris), stream));
        OBJ_TRY(dalloc(&vcount, nverts, stream));
        OBJ_TRY(dalloc(&vstart, nverts + 1, stream));
        OBJ_TRY(hipMemsetAsync(vcount, 0, 4 * size_t(nverts), stream));
        if (arith == CERES_ARITH_FMA)
            hipLaunchKernelGGL(k_tris<true>, dim3((ntris + 255) / 256), dim3(256), 0, stream, verts, corners, ntris, tris, cidx, vcount);
        else
            hipLaunchKernelGGL(k_tris<false>, dim3((ntris + 255) / 256), dim3(256), 0, stream, verts, corners, ntris, tris, cidx, vcount);
        OBJ_TRY(hipGetLastError());
        // stable sort of the corners by vertex: each vertex's corners stay in face order
        ckey = corners;
        {
            int end_bit = 1;
            while (end_bit < 32 && (uint64_t(1) << end_bit) < nverts) ++end_bit;
            size_t tmp_bytes = 0;
            OBJ_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, ckey, skey, cidx, sval, size_t(3) * ntris, 0, end_bit, stream));
            OBJ_TRY(hipMallocAsync(&sort_tmp, std::max<size_t>(tmp_bytes, 1), stream));
            OBJ_TRY(rocprim::radix_sort_pairs(sort_tmp, tmp_bytes, ckey, skey, cidx, sval, size_t(3) * ntris, 0, end_bit, stream));
        }
        OBJ_TRY(hipFreeAsync(part, stream));
        part = nullptr;
        OBJ_TRY(dalloc(&part, scan_blocks(std::max(nverts, 1u)) + 2, stream));
        OBJ_TRY(exclusive_scan(vcount, nverts, vstart, part, stream));
        OBJ_TRY(dalloc(&vnorm, 3 * size_t(nverts), stream));
        if (arith == CERES_ARITH_FMA)
            hipLaunchKernelGGL(k_vnorm<true>, dim3((nverts + 255) / 256), dim3(256), 0, stream, vstart, sval, tris, nverts, vnorm);
        else
            hipLaunchKernelGGL(k_vnorm<false>, dim3((nverts + 255) / 256), dim3(256), 0, stream, vstart, sval, tris, nverts, vnorm);
        hipLaunchKernelGGL(k_trinorm, dim3((ntris + 255) / 256), dim3(256), 0, stream, corners, vnorm, ntris, norm36);
        OBJ_TRY(hipGetLastError());
        OBJ_TRY(hipStreamSynchronize(stream));
        *d_tri48 = reinterpret_cast<float*>(tris);
        *d_norm36 = norm36;
        *n_tri = ntris;
        tris = nullptr;
        norm36 = nullptr;
    }
done:
    for (void* p : {(void*)counts, (void*)offs, (void*)part, (void*)nlpos, (void*)vflag, (void*)tcount, (void*)vidx,
                    (void*)tbase, (void*)first_long, (void*)corners, (void*)cidx, (void*)skey, (void*)sval,
                    (void*)vcount, (void*)vstart, (void*)bad, (void*)verts, (void*)vnorm, sort_tmp})
        if (p) (void)hipFreeAsync(p, stream);
    (void)hipStreamSynchronize(stream);
    if (tris) (void)hipFree(tris);                        // only on failure (moved to the caller on success)
    if (norm36) (void)hipFree(norm36);
    return rc;
}

int ceres_obj_parse_device(const char* d_text, size_t len, float** d_tri48, float** d_norm36, size_t* n_tri,
                           void* stream_) {
    return ceres_obj_parse_device_arith(d_text, len, d_tri48, d_norm36, n_tri, stream_, CERES_ARITH_EXACT);
}

// Host-buffer form with ceres_obj_load's contract: the file is read on the host, parsed on
// HIP `device`, and the arrays come back malloc'd (free with ceres_free).
int ceres_obj_load_gpu_arith(const char* path, float** tri48, float** norm36, size_t* n_tri, int device, int arith) {
    if (!path || !tri48 || !norm36 || !n_tri) return set_error(CERES_EINVAL, "ceres_obj_load_gpu: null argument");
    *tri48 = *norm36 = nullptr;
    *n_tri = 0;
    int rc = CERES_OK;
    hipStream_t stream = nullptr;
    char* h_text = nullptr;                                   // pinned: the upload runs at PCIe speed
    char* d_text = nullptr;
    float *d_tri = nullptr, *d_norm = nullptr;
    size_t n = 0, len = 0;
    FILE* f = std::fopen(path, "rb");
    if (!f) return CERES_OK;                                  // unreadable file: empty mesh (obj_norms.hpp:123-126)
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    OBJ_TRY(hipSetDevice(device));
    if (sz > 0) {
        OBJ_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_text), size_t(sz), hipHostMallocDefault));
        len = std::fread(h_text, 1, size_t(sz), f);
    }
    std::fclose(f);
    f = nullptr;
    if (len == 0) goto done;
    OBJ_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    OBJ_TRY(hipMalloc(&d_text, len));
    OBJ_TRY(hipMemcpyAsync(d_text, h_text, len, hipMemcpyHostToDevice, stream));
    if ((rc = ceres_obj_parse_device_arith(d_text, len, &d_tri, &d_norm, &n, stream, arith)) != CERES_OK) goto done;
    if (n) {
        *tri48 = static_cast<float*>(std::malloc(n * 48));
        *norm36 = static_cast<float*>(std::malloc(n * 36));
        if (!*tri48 || !*norm36) { rc = set_error(CERES_ENOMEM, "out of host memory"); goto done; }
        OBJ_TRY(hipMemcpyAsync(*tri48, d_tri, n * 48, hipMemcpyDeviceToHost, stream));
        OBJ_TRY(hipMemcpyAsync(*norm36, d_norm, n * 36, hipMemcpyDeviceToHost, stream));
        OBJ_TRY(hipStreamSynchronize(stream));
        *n_tri = n;
    }
done:
    if (f) std::fclose(f);
    if (rc != CERES_OK) { std::free(*tri48); std::free(*norm36); *tri48 = *norm36 = nullptr; *n_tri = 0; }
    if (d_tri) (void)hipFree(d_tri);
    if (d_norm) (void)hipFree(d_norm);
    if (d_text) (void)hipFree(d_text);
    if (h_text) (void)hipHostFree(h_text);
    if (stream) (void)hipStreamDestroy(stream);
    return rc;
}

int ceres_obj_load_gpu(const char* path, float** tri48, float** norm36, size_t* n_tri, int device) {
    return ceres_obj_load_gpu_arith(path, tri48, norm36, n_tri, device, CERES_ARITH_EXACT);
}

}  // extern "C"
