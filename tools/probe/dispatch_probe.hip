// Workgroup dispatch timeline: every workgroup stamps its entry (100 MHz realtime) and then holds
// its slot for ~10 us, so the spread of entry times is how long the dispatcher takes to place G
// long-lived workgroups of a given footprint (VGPRs, dynamic LDS) when they all fit at once.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

__device__ __forceinline__ void hold(uint64_t t0)
{
    while (__builtin_amdgcn_s_memrealtime() < t0 + 1000) __builtin_amdgcn_s_sleep(2);
}

__global__ void __launch_bounds__(256) k_light(uint64_t *st, uint32_t *sink)
{
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) st[blockIdx.x] = t;
    hold(t);
}

__global__ void __launch_bounds__(256) k_lds(uint64_t *st, uint32_t *sink)
{
    extern __shared__ uint32_t lds[];
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) st[blockIdx.x] = t + (lds[5] == 77u);
    hold(t);
}

// ~96 VGPRs live across the hold
__global__ void __launch_bounds__(256, 5) k_vgpr(uint64_t *st, uint32_t *sink)
{
    extern __shared__ uint32_t lds[];
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    uint32_t r[80];
#pragma unroll
    for (int i = 0; i < 80; ++i) r[i] = threadIdx.x * (i + 3) ^ (uint32_t)t;
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) st[blockIdx.x] = t + (lds[5] == 77u);
    hold(t);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 80; ++i) x = x * 31u + r[i];
    if (x == 0x12345u) sink[threadIdx.x] = x;
}

int main()
{
    uint64_t *st; uint32_t *sink;
    (void)hipMalloc(&st, 16384 * 8);
    (void)hipMalloc(&sink, 4096);
    std::vector<uint64_t> h(16384);
    auto run = [&](const char *name, void (*k)(uint64_t *, uint32_t *), int G, size_t lds) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, 0, st, sink);
            (void)hipDeviceSynchronize();
        }
        (void)hipMemcpy(h.data(), st, G * 8, hipMemcpyDeviceToHost);
        std::vector<uint64_t> v(h.begin(), h.begin() + G);
        std::sort(v.begin(), v.end());
        auto pc = [&](double q) { return (v[(size_t)(q * (G - 1))] - v[0]) / 100.0; };
        printf("%-8s G=%5d lds=%6zu  entry spread us p10 %.2f p50 %.2f p90 %.2f max %.2f\n", name, G, lds,
               pc(0.1), pc(0.5), pc(0.9), pc(1.0));
    };
    run("light", k_light, 1024, 0);
    run("light", k_light, 2048, 0);
    run("vgpr", k_vgpr, 1024, 28160);
    for (size_t l : {15872, 17920, 20480, 28160, 32768, 40000})
        run("lds", k_lds, 1024, l);
    run("lds", k_lds, 512, 40000);
    run("lds", k_lds, 512, 65536);
    return 0;
}
