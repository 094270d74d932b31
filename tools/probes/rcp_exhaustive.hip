// Exhaustive check (all 2^32 float bit patterns): is r1 = fma(fma(-x, r0, 1), r0, r0) with
// r0 = v_rcp_f32(x) the correctly rounded 1/x (what -fhip-fp32-correctly-rounded-divide-sqrt
// computes with the v_div_scale/fmas/fixup sequence)?  Counts mismatches per input exponent.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang fp contract(off)

__global__ void check(uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const float exact = 1.0f / x;
    const float r0 = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r0, 1.0f);
    const float r1 = __builtin_fmaf(e, r0, r0);
    const uint32_t a = __float_as_uint(exact), b = __float_as_uint(r1);
    const bool nan = (exact != exact) && (r1 != r1);
    if (a != b && !nan) {
        const uint32_t ex = (bits >> 23) & 0xff;
        atomicAdd(&bad[ex], 1ull);
        atomicCAS(&first[ex], 0u, bits);
    }
}

int main() {
    unsigned long long* bad; uint32_t* first;
    hipMalloc(&bad, 256 * 8); hipMalloc(&first, 256 * 4);
    hipMemset(bad, 0, 256 * 8); hipMemset(first, 0, 256 * 4);
    for (uint32_t hi = 0; hi < 256; ++hi) hipLaunchKernelGGL(check, dim3(1 << 16), dim3(256), 0, 0, hi, bad, first);
    unsigned long long hb[256]; uint32_t hf[256];
    hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
    hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    int lo_ok = -1, hi_ok = -1;
    for (int e = 0; e < 256; ++e) {
        tot += hb[e];
        if (hb[e]) printf("exp %3d (2^%d): %llu mismatches, e.g. 0x%08x\n", e, e - 127, hb[e], hf[e]);
    }
    for (int e = 127; e >= 0 && !hb[e]; --e) lo_ok = e;
    for (int e = 127; e < 256 && !hb[e]; ++e) hi_ok = e;
    printf("total mismatches %llu; exact for biased exponents [%d, %d] (2^%d .. 2^%d)\n", tot, lo_ok, hi_ok, lo_ok - 127, hi_ok - 127);
    return 0;
}
