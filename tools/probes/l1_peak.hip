// l1_peak.hip -- calibrates the vector-L1 (TCP) ceiling bench.py prices the render kernel against
// (round 6): how many TCP cache accesses per CU-cycle gfx950 sustains for the
// render kernel's own access shape, measured with rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum on
// this program.  Every lane fetches 64-B records with four 16-B loads (global_load_dwordx4),
// records chosen pseudo-randomly among 128 that stay in the CU's 32-KiB L1 (the divergent shape of
// a BVH2 step, sibling pairs), or (mode 1) one record for the whole wavefront (a uniform step), or
// (mode 2) 16 contiguous bytes per lane (a coalesced stream).  No load depends on an earlier one:
// the loop is throughput-bound, eight waves per SIMD.
//
// usage: l1_peak [mode 0|1|2] [iterations]  -> one JSON line: mode, launches, mean ms, loads
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

constexpr int kRecords = 128;          // 8 KiB of 64-B records per workgroup slice: L1-resident
constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void l1_loads(const float4* __restrict__ recs, int iters, int mode, float4* out) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t st = (blockIdx.x * kBlock + threadIdx.x) * 2654435761u + 12345u;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* base = recs + (blockIdx.x & 7) * kRecords * 4;     // a few slices, all L1/L2-resident
    for (int it = 0; it < iters; ++it) {
        st = st * 1664525u + 1013904223u;
        uint32_t r = (st >> 8) % kRecords;
        if (mode == 1) r = __builtin_amdgcn_readfirstlane(r);
        if (mode == 2) {
            const float4 a = base[(it * 64 + lane) % (kRecords * 4)];
            acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
            continue;
        }
        const float4* q = base + r * 4;
        const float4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc.x += a.x + b.x + c.x + d.x;
        acc.y += a.y + b.y + c.y + d.y;
        acc.z += a.z + b.z + c.z + d.z;
        acc.w += a.w + b.w + c.w + d.w;
    }
    if (acc.x == 1234.5f) out[blockIdx.x * kBlock + threadIdx.x] = acc;   // keeps the loads, never true
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 2048;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 8;                // 8 x 256 threads = 32 waves per CU
    float4 *recs = nullptr, *out = nullptr;
    CHECK(hipMalloc(&recs, 8 * kRecords * 64));
    CHECK(hipMalloc(&out, size_t(blocks) * kBlock * sizeof(float4)));
    CHECK(hipMemset(recs, 0, 8 * kRecords * 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(l1_loads, dim3(blocks), dim3(kBlock), 0, 0, recs, iters, mode, out);   // warm
    CHECK(hipDeviceSynchronize());
    const int launches = 5;
    CHECK(hipEventRecord(e0, 0));
    for (int k = 0; k < launches; ++k) hipLaunchKernelGGL(l1_loads, dim3(blocks), dim3(kBlock), 0, 0, recs, iters, mode, out);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double wave_loads = double(blocks) * (kBlock / 64) * iters * (mode == 2 ? 1 : 4);   // dwordx4 wave-instructions per launch
    std::printf("{\"mode\": %d, \"iters\": %d, \"blocks\": %d, \"cus\": %d, \"launches\": %d, \"mean_ms\": %.5f, "
                "\"wave_load_instructions_per_launch\": %.0f}\n",
                mode, iters, blocks, prop.multiProcessorCount, launches + 1, ms / launches, wave_loads);
    CHECK(hipFree(recs));
    CHECK(hipFree(out));
    return 0;
}
