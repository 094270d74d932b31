// dev_scan.hpp -- exclusive prefix sums of u32 arrays on gfx950 (shared by the BVH builder and
// the OBJ parser).  Three kernels: per-block totals, one workgroup scanning the totals, and the
// per-block down-sweep; x[n] receives the grand total.  Internal linkage (anonymous namespace),
// so every translation unit that includes this gets its own copy of the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ceres {
namespace devscan {
namespace {

constexpr int kScanBlock = 1024;           // elements per block (256 threads x 4)

__device__ uint32_t block_exclusive_scan_256(uint32_t v, uint32_t* sh, uint32_t& total) {
    // sh: 256 + 8 entries
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= uint32_t(off)) x += y;
    }
    if (lane == 63) sh[256 + wave] = x;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t w = 0; w < wave; ++w) wbase += sh[256 + w];
    total = sh[256] + sh[257] + sh[258] + sh[259];
    __syncthreads();
    return wbase + x - v;
}

__global__ void __launch_bounds__(256) k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ partial) {
    __shared__ uint32_t sh[264];
    const uint32_t base = blockIdx.x * uint32_t(kScanBlock) + threadIdx.x * 4u;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) if (base + k < n) v += in[base + k];
    uint32_t total;
    (void)block_exclusive_scan_256(v, sh, total);
    if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// single workgroup: exclusive scan of the block partials in place
__global__ void __launch_bounds__(256) k_scan_partials(uint32_t* partial, uint32_t nb) {
    __shared__ uint32_t sh[264];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nb ? partial[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan_256(v, sh, total);
        if (i < nb) partial[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) partial[nb] = carry;
}

__global__ void __launch_bounds__(256) k_scan_down(const uint32_t* __restrict__ in, uint32_t n, const uint32_t* __restrict__ partial,
                                                   uint32_t* __restrict__ out) {
    __shared__ uint32_t sh[264];
    const uint32_t base = blockIdx.x * uint32_t(kScanBlock) + threadIdx.x * 4u;
    uint32_t v[4], sum = 0;
    for (int k = 0; k < 4; ++k) { v[k] = base + k < n ? in[base + k] : 0u; sum += v[k]; }
    uint32_t total;
    uint32_t x = partial[blockIdx.x] + block_exclusive_scan_256(sum, sh, total);
    for (int k = 0; k < 4; ++k) { if (base + k < n) out[base + k] = x; x += v[k]; }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = partial[gridDim.x];
}

// out[0..n) = exclusive prefix sums of in[0..n), out[n] = total.  partial: scan_partials(n) + 1 u32.
inline uint32_t scan_blocks(uint32_t n) { return (n + kScanBlock - 1) / kScanBlock; }
inline hipError_t exclusive_scan(const uint32_t* in, uint32_t n, uint32_t* out, uint32_t* partial, hipStream_t stream) {
    const uint32_t nb = scan_blocks(n);
    if (nb == 0) return hipMemsetAsync(out, 0, 4, stream);
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(256), 0, stream, in, n, partial);
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, stream, partial, nb);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(256), 0, stream, in, n, partial, out);
    return hipGetLastError();
}

}  // namespace
}  // namespace devscan
}  // namespace ceres
