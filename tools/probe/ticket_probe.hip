// Ticket-latency probe: what does a per-workgroup ticket (one device-scope atomic at kernel
// start) cost a 1024-workgroup launch, against a plain load? Variants: one counter for the grid,
// 8 counters (blockIdx % 8, 128 B apart), one counter per XCD (XCC_ID), and a plain load of a
// per-workgroup word. Prints the mean / max cycles (s_memtime) from entry to the result and the
// kernel time (events, 200 launches). Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int MODE>
__global__ void __launch_bounds__(256) k_ticket(uint32_t *ctr, uint32_t *words, unsigned long long *cyc, uint32_t *sink)
{
    __shared__ uint32_t tk;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        uint32_t v;
        if (MODE == 0) v = atomicAdd(ctr, 1u);
        else if (MODE == 1) v = atomicAdd(ctr + 32 * (blockIdx.x & 7u), 1u);
        else if (MODE == 2) v = atomicAdd(ctr + 32 * (__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 7u), 1u);
        else v = __hip_atomic_load(words + 32 * blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tk = v;
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        cyc[blockIdx.x] = t1 - t0;
        if (tk == 0xFFFFFFFFu) sink[0] = 1;
    }
}

int main()
{
    const int G = 1024;
    uint32_t *ctr, *words, *sink;
    unsigned long long *cyc;
    hipMalloc(&ctr, 4096);
    hipMalloc(&words, G * 128);
    hipMalloc(&sink, 64);
    hipMalloc(&cyc, G * 8);
    hipMemset(words, 0, G * 128);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, void (*k)(uint32_t *, uint32_t *, unsigned long long *, uint32_t *)) {
        hipMemset(ctr, 0, 4096);
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, s, ctr, words, cyc, sink);
        hipEventRecord(e0, s);
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, s, ctr, words, cyc, sink);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> h(G);
        hipMemcpy(h.data(), cyc, G * 8, hipMemcpyDeviceToHost);
        double sum = 0, mx = 0;
        for (auto v : h) { sum += (double)v; mx = (double)v > mx ? (double)v : mx; }
        printf("%-22s cycles mean %8.0f max %8.0f   kernel %.2f us\n", name, sum / G, mx, 1e3 * ms / 200);
    };
    run("one counter", k_ticket<0>);
    run("8 counters (b % 8)", k_ticket<1>);
    run("per-XCD counter", k_ticket<2>);
    run("plain agent load", k_ticket<3>);
    return 0;
}
