// Kernel start/drain overhead: rocprofv3 duration of a kernel vs the span of its workgroups
// (first entry .. last exit, chip realtime clock), for busy workgroups with and without 8 MB of
// stores, 1024 workgroups x 256 threads like rx_classify at 1 M frames.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(256) k_busy(uint64_t *st, uint32_t *out, uint32_t iters, int store)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x * 2654435761u;
    for (uint32_t i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
    if (store) {
        for (int k = 0; k < 8; ++k) out[((size_t)blockIdx.x * 8 + k) * 256 + threadIdx.x] = x + k;
    } else if (x == 0x12345678u) {
        out[threadIdx.x] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = t0;
        st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main()
{
    const int G = 1024;
    uint64_t *st; uint32_t *out;
    (void)hipMalloc(&st, G * 16);
    (void)hipMalloc(&out, (size_t)G * 8 * 256 * 4);
    hipStream_t s; (void)hipStreamCreate(&s);
    for (int store = 0; store < 2; ++store) {
        for (uint32_t iters : {1000u, 10000u}) {
            for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_busy, dim3(G), dim3(256), 0, s, st, out, iters, store);
            (void)hipStreamSynchronize(s);
            uint64_t h[2 * G];
            (void)hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
            uint64_t mn = ~0ull, mx = 0;
            for (int i = 0; i < G; ++i) { mn = h[2 * i] < mn ? h[2 * i] : mn; mx = h[2 * i + 1] > mx ? h[2 * i + 1] : mx; }
            printf("store=%d iters=%u: workgroup span %.2f us (compare rocprofv3 k_busy durations)\n",
                   store, iters, (mx - mn) / 100.0);
        }
    }
    return 0;
}
