// One-workgroup scan probe: what does rss_base (rx_rss.hip) cost after a grid-wide writer kernel
// filled its histogram, against an empty 1024-thread kernel and a load-only variant? Durations
// from rocprofv3 --kernel-trace --stats.
#include "../../udpdk_amd/csrc/rx_rss.hip"
#include <cstdio>

using namespace udpdk;

__global__ void __launch_bounds__(256) k_writer(uint32_t *hist, uint32_t T, uint32_t S)
{
    // rss_hash's pattern: workgroup t writes entry (q, t) for every q
    for (uint32_t q = threadIdx.x; q < S; q += 256) hist[(size_t)q * T + blockIdx.x] = (blockIdx.x * 7 + q) & 15;
}
__global__ void __launch_bounds__(1024) k_empty1024(uint32_t *p, uint32_t n)
{
    if (threadIdx.x == 0 && n == 12345u) p[0] = 1;
}
__global__ void __launch_bounds__(1024) k_loadonly(uint32_t *hist, uint32_t n, uint32_t *out)
{
    uint32_t s = 0;
    for (uint32_t k = threadIdx.x; k < n; k += 1024) s += hist[k];
    if (s == 0xFFFFFFFFu) out[0] = s;
}
__global__ void __launch_bounds__(1024) k_serial(uint32_t *hist, uint32_t n, uint32_t *out)
{
    // one dependent load chain per thread (latency of a single round trip x rows)
    uint32_t s = 0;
    for (uint32_t k = threadIdx.x; k < n; k += 1024) s += hist[k + (s & 0x80000000u)];
    if (s == 0xFFFFFFFFu) out[0] = s;
}

int main()
{
    const uint32_t S = 8;
    uint32_t *hist, *qo, *tot;
    hipMalloc(&hist, 4 * RSS_BASE_MAX);
    hipMalloc(&qo, 4 * 128);
    hipMalloc(&tot, 4);
    for (uint32_t T : {1024u, 4096u}) {
        for (int r = 0; r < 50; ++r) {
            k_writer<<<T, 256>>>(hist, T, S);
            rss_base<<<1, 1024>>>(hist, T * S, T, qo, tot);
            k_writer<<<T, 256>>>(hist, T, S);
            k_loadonly<<<1, 1024>>>(hist, T * S, tot);
            k_writer<<<T, 256>>>(hist, T, S);
            k_serial<<<1, 1024>>>(hist, T * S, tot);
            k_empty1024<<<1, 1024>>>(hist, T);
            rss_base<<<1, 1024>>>(hist, T * S, T, qo, tot);   // histogram already in this XCD's L2? (no writer)
        }
        hipDeviceSynchronize();
    }
    printf("done %d\n", (int)hipGetLastError());
    return 0;
}
