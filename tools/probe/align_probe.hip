// How fast does the vector memory path move 16-byte buffer loads at each alignment? 1 GiB read
// once per launch (more than the 256 MiB Infinity Cache), every wave streaming its own 128 KiB
// span in 4 KiB groups (two groups in flight), one u32 written per lane. Patterns:
//   chunk  lane i reads the 64-byte chunk i of a group as 4 pieces (rx_classify's tail pass)
//   coal   instruction c reads 1 KiB contiguous, lane i at 16 i
// Loaders:
//   b128   byte-addressed 16-byte loads at the shifted address (what the tail pass issues)
//   al     16-byte loads at the aligned-down address (5 per 64-byte chunk for chunk, 17 per
//          1 KiB... coal keeps 4 and adds one) + v_alignbyte funnel to the shifted words
//   b32    four 4-byte loads per piece
// Usage: align_probe [reps]; prints GB/s per (pattern, loader, shift).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 ld128(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint4 ld4x32(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return make_uint4(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0),
                      __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 4, 0, 0),
                      __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 8, 0, 0),
                      __builtin_amdgcn_raw_buffer_load_b32(r, (int)off + 12, 0, 0));
}
__device__ __forceinline__ uint32_t s4(uint4 v) { return v.x + v.y + v.z + v.w; }

// 16 words starting at byte sh (0-15) of the 20 aligned words D
__device__ __forceinline__ uint32_t funnel_sum(const uint32_t (&D)[20], uint32_t sh)
{
    const uint32_t q = sh >> 2, b = (sh & 3u) * 8u;
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t lo = q == 0 ? D[i] : q == 1 ? D[i + 1] : q == 2 ? D[i + 2] : D[i + 3];
        const uint32_t hi = q == 0 ? D[i + 1] : q == 1 ? D[i + 2] : q == 2 ? D[i + 3] : D[i + 4];
        acc += (uint32_t)(((((uint64_t)hi) << 32) | lo) >> b);
    }
    return acc;
}

template <int PAT, int LD>
__global__ void __launch_bounds__(256) k_probe(const uint8_t *buf, uint32_t bytes, uint32_t shift,
                                               uint32_t span, uint32_t *out)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(buf, bytes);
    const uint32_t lane = threadIdx.x & 63, g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t base = g * span + shift;
    uint32_t acc = 0;
#pragma unroll 2
    for (uint32_t k = 0; k < span; k += 4096) {
        const uint32_t o = base + k;
        if (LD == 1) {
            uint32_t D[20];
            if (PAT == 0) {
                const uint32_t a = (o + 64 * lane) & ~15u, sh = (o + 64 * lane) & 15u;
#pragma unroll
                for (int c = 0; c < 5; ++c) {
                    const uint4 v = ld128(r, a + 16 * c);
                    D[4 * c] = v.x; D[4 * c + 1] = v.y; D[4 * c + 2] = v.z; D[4 * c + 3] = v.w;
                }
                acc += funnel_sum(D, sh);
            } else {
                // contiguous: lane i's aligned piece and its right neighbour's first word
                const uint32_t sh = o & 15u;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t a = ((o + 1024 * c) & ~15u) + 16 * lane;
                    const uint4 v = ld128(r, a);
                    const uint32_t nx = __shfl_down(v.x, 1, 64);
                    const uint32_t tail = lane == 63 ? __builtin_amdgcn_raw_buffer_load_b32(r, (int)(a + 16), 0, 0) : nx;
                    const uint32_t w[5] = {v.x, v.y, v.z, v.w, tail};
                    const uint32_t q = sh >> 2, b = (sh & 3u) * 8u;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint32_t lo = q == 0 ? w[i] : q == 1 ? w[min(i + 1, 4)] : q == 2 ? w[min(i + 2, 4)] : w[min(i + 3, 4)];
                        const uint32_t hi = q == 0 ? w[i + 1] : q == 1 ? w[min(i + 2, 4)] : q == 2 ? w[min(i + 3, 4)] : w[4];
                        acc += (uint32_t)(((((uint64_t)hi) << 32) | lo) >> b);
                    }
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t off = PAT == 0 ? o + 64 * lane + 16 * c : o + 1024 * c + 16 * lane;
                acc += s4(LD == 0 ? ld128(r, off) : ld4x32(r, off));
            }
        }
    }
    out[g * 64 + lane] = acc;
}

// copy: wave-contiguous 1 KiB per instruction, source at +rs and destination at +ws bytes
__global__ void __launch_bounds__(256) k_copy(const uint8_t *src, uint8_t *dst, uint32_t bytes,
                                              uint32_t rs, uint32_t ws, uint32_t span)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(src, bytes), w = rsrc(dst, bytes);
    const uint32_t lane = threadIdx.x & 63, g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t base = g * span;
    for (uint32_t k = 0; k < span; k += 4096) {
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = ld128(r, base + k + 1024 * c + 16 * lane + rs);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            __attribute__((ext_vector_type(4))) uint32_t x = {v[c].x, v[c].y, v[c].z, v[c].w};
            __builtin_amdgcn_raw_buffer_store_b128(x, w, (int)(base + k + 1024 * c + 16 * lane + ws), 0, 0);
        }
    }
}

// copy in tasks of `task` bytes (a wave per task, grid-stride over tasks, loads of a task issued
// before its stores), the shape of reasm_emit's per-datagram copies
__global__ void __launch_bounds__(256) k_copy_tasks(const uint8_t *src, uint8_t *dst, uint32_t bytes,
                                                    uint32_t task, uint32_t ntask)
{
    const __amdgpu_buffer_rsrc_t r = rsrc(src, bytes), w = rsrc(dst, bytes);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t t = wv; t < ntask; t += nw) {
        const uint32_t base = t * task;
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t o = 1024 * c + 16 * lane;
            v[c] = ld128(r, o < task ? base + o + 2 : 0x80000000u);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t o = 1024 * c + 16 * lane;
            __attribute__((ext_vector_type(4))) uint32_t x = {v[c].x, v[c].y, v[c].z, v[c].w};
            if (o < task) __builtin_amdgcn_raw_buffer_store_b128(x, w, (int)(base + o + 2), 0, 0);
        }
    }
}

static float run_copy_tasks(const uint8_t *src, uint8_t *dst, uint32_t task, uint32_t ntask,
                            uint32_t blocks, int reps)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t bytes = task * ntask + 64;
    hipLaunchKernelGGL(k_copy_tasks, dim3(blocks), dim3(256), 0, 0, src, dst, bytes, task, ntask);
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_copy_tasks, dim3(blocks), dim3(256), 0, 0, src, dst, bytes, task, ntask);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return (float)(2.0 * task * ntask * reps / (ms * 1e-3) / 1e9);
}

static float run_copy(const uint8_t *src, uint8_t *dst, uint32_t bytes, uint32_t rs, uint32_t ws,
                      uint32_t span, int reps)
{
    const uint32_t blocks = (bytes - 64) / span / 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, src, dst, bytes, rs, ws, span);
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, src, dst, bytes, rs, ws, span);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return (float)(2.0 * blocks * 4 * span * reps / (ms * 1e-3) / 1e9);   // read + written
}

template <int PAT, int LD>
static float run(const uint8_t *buf, uint32_t bytes, uint32_t shift, uint32_t span, uint32_t *out, int reps)
{
    const uint32_t waves = (bytes - 64) / span, blocks = waves / 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_probe<PAT, LD>), dim3(blocks), dim3(256), 0, 0, buf, bytes, shift, span, out);
    CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((k_probe<PAT, LD>), dim3(blocks), dim3(256), 0, 0, buf, bytes, shift, span, out);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return (float)((double)blocks * 4 * span * reps / (ms * 1e-3) / 1e9);
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint32_t span = 128u << 10, bytes = (1u << 30) + 4096;
    uint8_t *buf;
    uint32_t *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 1, bytes));
    CHECK(hipMalloc(&out, (bytes / span + 1) * 64 * 4));
    if (argc > 2) {                      // copy mode: GB/s (read + written) per (src, dst) shift
        uint8_t *dst;
        CHECK(hipMalloc(&dst, bytes));
        // emit-shaped: 256 K tasks of 2992 B (776 MB each way), grids of 2048 / 8192 blocks
        printf("{\"tasks 2992 B x 256K, 2048 blocks\": %.0f, \"tasks 2992 B x 256K, 8192 blocks\": %.0f, "
               "\"tasks 4096 B x 192K, 8192 blocks\": %.0f}\n",
               run_copy_tasks(buf, dst, 2992, 262144, 2048, reps), run_copy_tasks(buf, dst, 2992, 262144, 8192, reps),
               run_copy_tasks(buf, dst, 4096, 196608, 8192, reps));
        const uint32_t cs[][2] = {{0, 0}, {2, 0}, {0, 2}, {2, 2}, {0, 4}, {1, 3}};
        printf("{");
        for (int i = 0; i < 6; ++i)
            printf("%s\"copy src+%u dst+%u\": %.0f", i ? ", " : "", cs[i][0], cs[i][1],
                   run_copy(buf, dst, bytes, cs[i][0], cs[i][1], span, reps));
        printf("}\n");
        CHECK(hipFree(dst));
        return 0;
    }
    const uint32_t shifts[] = {0, 4, 8, 1, 2, 3};
    printf("{");
    const char *sep = "";
    for (uint32_t s : shifts) {
        printf("%s\"chunk b128 +%u\": %.0f", sep, s, run<0, 0>(buf, bytes, s, span, out, reps)); sep = ", ";
        printf(", \"chunk b32 +%u\": %.0f", s, run<0, 2>(buf, bytes, s, span, out, reps));
        printf(", \"chunk al +%u\": %.0f", s, run<0, 1>(buf, bytes, s, span, out, reps));
        printf(", \"coal b128 +%u\": %.0f", s, run<1, 0>(buf, bytes, s, span, out, reps));
        printf(", \"coal al +%u\": %.0f", s, run<1, 1>(buf, bytes, s, span, out, reps));
        fflush(stdout);
    }
    printf("}\n");
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
