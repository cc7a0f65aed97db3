// Launch-overhead probe: how long do kernels of the rx_classify shape take when they do (almost)
// nothing, and what does writing the 8 MB of outputs cost? Timed with HIP events over back-to-back
// launches and by rocprofv3 --kernel-trace.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Big { uint64_t p[24]; uint32_t u[16]; };

__global__ void __launch_bounds__(256) k_empty(Big a) {
    if (threadIdx.x == 0 && a.u[0] == 12345u) ((uint32_t *)a.p[0])[blockIdx.x] = 1;
}
__global__ void __launch_bounds__(256) k_stamp(Big a) {
    // entry realtime per WG -> start skew
    if (threadIdx.x == 0) ((uint64_t *)a.p[1])[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}
// the stamp kernel with rx_classify's footprint: ~120 VGPRs live, dynamic LDS, a ticket atomic
__global__ void __launch_bounds__(256) k_stamp_vgpr(Big a) {
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    float acc[112];
#pragma unroll
    for (int i = 0; i < 112; ++i) acc[i] = (float)(threadIdx.x * i);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 112; ++i) acc[i] = acc[i] * acc[(i + 1) % 112] + 1.0f;
    float s = 0;
#pragma unroll
    for (int i = 0; i < 112; ++i) s += acc[i];
    if (threadIdx.x == 0) ((uint64_t *)a.p[1])[blockIdx.x] = t;
    if (s == 1234.5f) ((float *)a.p[0])[threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k_stamp_lds(Big a) {
    extern __shared__ uint32_t lds[];
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) ((uint64_t *)a.p[1])[blockIdx.x] = t + lds[5] - 5;
}
__global__ void __launch_bounds__(256) k_stamp_ticket(Big a) {
    __shared__ uint32_t tk;
    uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) tk = atomicAdd((uint32_t *)a.p[2], 1u);
    __syncthreads();
    if (threadIdx.x == 0) ((uint64_t *)a.p[1])[blockIdx.x] = t + (tk == 0xFFFFFFFFu);
}
__global__ void __launch_bounds__(256) k_write(Big a) {
    uint32_t *o = (uint32_t *)a.p[0];
    const uint32_t per = a.u[1];
    for (uint32_t i = threadIdx.x; i < per; i += 256) o[(size_t)blockIdx.x * per + i] = i;
}
__global__ void __launch_bounds__(256) k_write_nt(Big a) {
    uint32_t *o = (uint32_t *)a.p[0];
    const uint32_t per = a.u[1];
    for (uint32_t i = threadIdx.x; i < per; i += 256)
        __builtin_nontemporal_store(i, &o[(size_t)blockIdx.x * per + i]);
}

int main() {
    const int G = 512;
    Big a = {};
    uint32_t *o; uint64_t *st;
    hipMalloc(&o, 64u << 20);
    hipMalloc(&st, G * 8);
    uint32_t *tk; hipMalloc(&tk, 64); hipMemset(tk, 0, 64);
    a.p[0] = (uint64_t)o; a.p[1] = (uint64_t)st; a.p[2] = (uint64_t)tk;
    a.u[1] = (8u << 20) / 4 / G;       // 8 MB across the grid
    hipStream_t s; hipStreamCreate(&s);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char *name, void (*k)(Big), int reps) {
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, s, a);
        hipEventRecord(e0, s);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, s, a);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-12s back-to-back avg %.2f us\n", name, 1e3 * ms / reps);
        // single launch bracketed by events
        float tot = 0;
        for (int i = 0; i < reps; ++i) {
            hipEventRecord(e0, s);
            hipLaunchKernelGGL(k, dim3(G), dim3(256), 0, s, a);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1); tot += ms;
        }
        printf("%-12s event-bracketed avg %.2f us\n", name, 1e3 * tot / reps);
    };
    auto spread = [&](const char *name, void (*k)(Big), size_t lds) {
        hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, s, a);
        hipStreamSynchronize(s);
        hipMemset(st, 0, G * 8);
        hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, s, a);
        hipStreamSynchronize(s);
        uint64_t h[G];
        hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
        uint64_t mn = ~0ull, mx = 0;
        for (int i = 0; i < G; ++i) { mn = h[i] < mn ? h[i] : mn; mx = h[i] > mx ? h[i] : mx; }
        printf("%-14s WG entry spread %.2f us\n", name, (mx - mn) / 100.0);
    };
    spread("stamp", k_stamp, 0);
    spread("stamp_vgpr", k_stamp_vgpr, 0);
    spread("stamp_lds4k", k_stamp_lds, 4096);
    spread("stamp_ticket", k_stamp_ticket, 0);
    run("empty", k_empty, 200);
    run("stamp", k_stamp, 200);
    run("write8MB", k_write, 200);
    run("write8MB_nt", k_write_nt, 200);
    return 0;
}
