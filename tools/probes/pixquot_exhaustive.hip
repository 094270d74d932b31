// Exhaustive check of the pixel-coordinate quotient used by primary_dir (render_hip.hip
// pix_quot): for every image size n in [1, 65536] and every pixel index i < n, is
//   q = fma(fma(-n, q0, a), r0, q0),  q0 = a * r0,  r0 = v_rcp_f32(n),  a = 2 * (i + 0.5f)
// the correctly rounded a / n (render.hpp:109-110's `2 * (i + 0.5) / width`, what
// -fhip-fp32-correctly-rounded-divide-sqrt computes with the v_div_scale/fmas/fixup sequence)?
// 2^31 pairs; prints the mismatch count and the first mismatching (n, i).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)

__global__ void check(uint32_t n0, unsigned long long* bad, unsigned long long* first) {
    const uint32_t n = n0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 0 || n > 65536) return;
    const float fn = float(n);
    const float r0 = __builtin_amdgcn_rcpf(fn);
    unsigned long long b = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const float a = 2 * (float(i) + 0.5f);
        const float exact = a / fn;
        const float q0 = a * r0;
        const float q = __builtin_fmaf(__builtin_fmaf(-fn, q0, a), r0, q0);
        if (__float_as_uint(q) != __float_as_uint(exact)) {
            if (!b) atomicCAS(first, 0ull, (unsigned long long)n << 32 | i);
            ++b;
        }
    }
    if (b) atomicAdd(bad, b);
}

int main() {
    unsigned long long *bad, *first;
    hipMalloc(&bad, 8); hipMalloc(&first, 8);
    hipMemset(bad, 0, 8); hipMemset(first, 0, 8);
    hipLaunchKernelGGL(check, dim3(65536 / 64 + 1), dim3(64), 0, 0, 1u, bad, first);
    unsigned long long hb = 0, hf = 0;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 8, hipMemcpyDeviceToHost);
    if (hipDeviceSynchronize() != hipSuccess) { printf("HIP error\n"); return 2; }
    printf("pairs 2147516416 mismatches %llu", hb);
    if (hb) printf(" first n=%llu i=%llu", hf >> 32, hf & 0xffffffffull);
    printf("\n");
    return 0;
}
