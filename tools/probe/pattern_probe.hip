// HBM read-pattern probe for the 64 B-frame case: 1 M frames x 64 B (64 MiB) per batch, rotated
// over 10 copies (> the 256 MiB Infinity Cache). Each kernel reads every frame byte once and
// writes one u32 per frame, 1024 workgroups x 256 threads, 4 steps of 64 frames per wave, loads
// of the next step in flight while the current one is summed.
//   lane:      lane = frame, 4 x 16 B per lane at a 64 B stride (rx_classify's window shape)
//   coalesced: the wave reads its 4 KiB step as 4 contiguous 1 KiB wave-loads, then the frame
//              sums are gathered through LDS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int STEPS = 4;

__device__ __forceinline__ uint32_t s4(uint4 v) { return v.x + v.y + v.z + v.w; }

__global__ void __launch_bounds__(256) k_lane(const uint4 *fr, uint32_t *out)
{
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = blockIdx.x * 1024 + w * 64 + lane;       // step s: + s * 256
    uint4 a0 = fr[f0 * 4], a1 = fr[f0 * 4 + 1], a2 = fr[f0 * 4 + 2], a3 = fr[f0 * 4 + 3];
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t f = f0 + s * 256;
        const uint32_t fn = f + (s + 1 < STEPS ? 256 : 0);
        const uint4 b0 = fr[fn * 4], b1 = fr[fn * 4 + 1], b2 = fr[fn * 4 + 2], b3 = fr[fn * 4 + 3];
        out[f] = s4(a0) ^ s4(a1) ^ s4(a2) ^ s4(a3);
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
    }
}

__global__ void __launch_bounds__(256) k_coal(const uint4 *fr, uint32_t *out)
{
    __shared__ uint32_t part[4][256];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t c0 = (blockIdx.x * 1024 + w * 64) * 4;         // chunk index of the wave's step 0
    uint4 a0 = fr[c0 + lane], a1 = fr[c0 + 64 + lane], a2 = fr[c0 + 128 + lane], a3 = fr[c0 + 192 + lane];
    for (int s = 0; s < STEPS; ++s) {
        const uint32_t c = c0 + s * 1024;
        const uint32_t cn = c + (s + 1 < STEPS ? 1024 : 0);
        const uint4 b0 = fr[cn + lane], b1 = fr[cn + 64 + lane], b2 = fr[cn + 128 + lane], b3 = fr[cn + 192 + lane];
        // chunk k of the step belongs to frame k / 4: 4 chunk sums per frame through LDS
        part[w][lane] = s4(a0); part[w][64 + lane] = s4(a1); part[w][128 + lane] = s4(a2); part[w][192 + lane] = s4(a3);
        __builtin_amdgcn_wave_barrier();
        const uint32_t v = part[w][lane * 4] ^ part[w][lane * 4 + 1] ^ part[w][lane * 4 + 2] ^ part[w][lane * 4 + 3];
        __builtin_amdgcn_wave_barrier();
        out[blockIdx.x * 1024 + w * 64 + s * 256 + lane] = v;
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
    }
}

int main()
{
    const size_t N = 1u << 20, COPIES = 10;
    uint4 *fr; uint32_t *out;
    (void)hipMalloc(&fr, N * 64 * COPIES);
    (void)hipMalloc(&out, N * 4);
    (void)hipMemset(fr, 1, N * 64 * COPIES);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int k = 0; k < 2; ++k) {
        auto kern = k == 0 ? k_lane : k_coal;
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(1024), dim3(256), 0, 0, fr + (i % COPIES) * N * 4, out);
        (void)hipEventRecord(e0, 0);
        const int R = 100;
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(kern, dim3(1024), dim3(256), 0, 0, fr + (i % COPIES) * N * 4, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / R;
        printf("%-10s %.2f us per launch, %.2f TB/s (68 MiB read+write)\n", k == 0 ? "lane" : "coalesced", us,
               (N * 68.0) / us / 1e6);
    }
    return 0;
}
