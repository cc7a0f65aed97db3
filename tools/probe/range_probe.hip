// Buffer-load range check semantics on gfx950: num_records = 20, 16-byte and 4-byte loads at
// several byte offsets near the end; prints which bytes come back non-zero.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint8_t *b, uint32_t nrec, uint32_t *out)
{
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(b), (short)0, (int)nrec, 0x00020000);
    const uint32_t o = threadIdx.x;                 // byte offset 0..31
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0);
    out[o * 5 + 0] = v[0]; out[o * 5 + 1] = v[1]; out[o * 5 + 2] = v[2]; out[o * 5 + 3] = v[3];
    out[o * 5 + 4] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)o, 0, 0);
}
int main()
{
    uint8_t h[64]; for (int i = 0; i < 64; ++i) h[i] = (uint8_t)(0x40 + i);
    uint8_t *b; uint32_t *o; hipMalloc(&b, 64); hipMalloc(&o, 32 * 20);
    hipMemcpy(b, h, 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(32), 0, 0, b, 20u, o);
    uint32_t r[32 * 5]; hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    for (int i = 0; i < 24; ++i)
        printf("off %2d: x4 %08x %08x %08x %08x  x1 %08x\n", i, r[i * 5], r[i * 5 + 1], r[i * 5 + 2], r[i * 5 + 3], r[i * 5 + 4]);
    return 0;
}
