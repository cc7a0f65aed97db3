// Does a wave's ds_add_rtn_u32 resolve lanes that hit the same LDS word in lane order?
// Every workgroup (8 waves, each with its own counter block) runs many rounds; per round each
// lane picks a key from a seeded hash over K keys and does atomicAdd on counter[wave][key],
// returning the old value. A lane-ordered resolution means: among lanes with equal keys, the
// returned values increase with the lane id. Counts violations over all rounds and grids.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ uint32_t hsh(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__global__ void __launch_bounds__(512) k(uint32_t K, uint32_t rounds, uint32_t inc, unsigned long long *bad,
                                         unsigned long long *tot)
{
    extern __shared__ uint32_t cnt[];                    // [8][K]
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < 8 * K; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    uint32_t nb = 0, nt = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t h = hsh(blockIdx.x * 0x9E3779B9u + r * 0x85EBCA6Bu + lane * 0xC2B2AE35u + w);
        const bool act = (h >> 28) != 0;                 // ~6 % inactive lanes
        const uint32_t key = (h % K);
        uint32_t o = 0;
        if (act) o = atomicAdd(&cnt[w * K + key], inc);
        // check: for every earlier lane with the same key, its return is smaller
        for (uint32_t j = 0; j < 64; ++j) {
            const uint32_t kj = __shfl(key, (int)j, 64);
            const uint32_t oj = __shfl(o, (int)j, 64);
            const bool aj = __shfl((int)act, (int)j, 64) != 0;
            if (act && aj && j < lane && kj == key) { ++nt; if (oj >= o) ++nb; }
        }
    }
    atomicAdd(bad, (unsigned long long)nb);
    atomicAdd(tot, (unsigned long long)nt);
}
int main()
{
    unsigned long long *d; hipMalloc(&d, 16);
    const uint32_t Ks[] = {1, 2, 3, 7, 64, 512, 4096};
    for (uint32_t inc : {1u, 0x10000u})
        for (uint32_t K : Ks) {
            hipMemset(d, 0, 16);
            hipLaunchKernelGGL(k, dim3(2048), dim3(512), 8 * K * 4, 0, K, 256u, inc, d, d + 1);
            unsigned long long h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            printf("K=%5u inc=%#x: same-key lane pairs %llu, out of lane order %llu\n", K, inc, h[1], h[0]);
        }
    return 0;
}
