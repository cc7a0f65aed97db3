// Access-shape calibration for a line-grid span sweep (round 6).
// Frames of 1500 B or IMIX sizes packed back to back; rx_classify's geometry (workgroup = tile of
// 1024 frames, wave w walks steps w, w + 4, ... of 64 frames). Each step's byte span [o_0, o_63 +
// l_63) is read once in 4 KiB groups from the 64-byte block at or below o_0, two groups in flight:
//   k_span_chunk  lane L of a group takes block L (four 16-byte loads 16 B apart, lanes 64 B apart)
//   k_span_piece  load c of a group covers 1 KiB contiguous (lane L at 1024 c + 16 L)
//   k_span_c128   as k_span_chunk from the 128-byte line at or below o_0
//   k_flat        the whole buffer as one grid-stride stream (the exact case)
// FETCH_SIZE x 2 against the buffer's bytes says which shape reads each line once.
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/sweep_probe tools/probe/sweep_probe.hip
//   sweep_probe [imix]   (under rocprofv3 --pmc FETCH_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t sum4(__attribute__((ext_vector_type(4))) uint32_t v, uint32_t s)
{
    s = __builtin_amdgcn_sad_u16(v[0], 0u, s);
    s = __builtin_amdgcn_sad_u16(v[1], 0u, s);
    s = __builtin_amdgcn_sad_u16(v[2], 0u, s);
    return __builtin_amdgcn_sad_u16(v[3], 0u, s);
}

template <int MODE>
__global__ void __launch_bounds__(256) k_span(const uint8_t *fr, uint32_t bytes, const uint32_t *off,
                                              const uint32_t *len, uint32_t n, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, bytes);
    uint32_t s = 0;
    for (uint32_t st = w; st < 16; st += 4) {
        const uint32_t f0 = blockIdx.x * 1024 + st * 64;
        if (f0 >= n) break;
        const uint32_t fl = min(n, f0 + 64) - 1;
        const uint32_t A = MODE == 2 ? off[f0] & ~127u : off[f0] & ~63u;
        const uint32_t E = off[fl] + len[fl];
        for (uint32_t g = A; g < E; g += 8192) {
            uint32_t b[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t gg = g + 4096u * (c >> 2);
                const uint32_t a = MODE == 1 ? gg + 1024u * (c & 3) + 16u * lane : gg + 64u * lane + 16u * (c & 3);
                b[c] = a < E ? a : 0xFFFFFFF0u;
            }
            __attribute__((ext_vector_type(4))) uint32_t v[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)b[c], 0, 0);
#pragma unroll
            for (int c = 0; c < 8; ++c) s = sum4(v[c], s);
        }
    }
    if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}


// timing variants of the piece-major sweep: IF groups of 4 KiB in flight per wave; JOINT: the 4
// waves of a workgroup sweep the span of its 4 consecutive steps together (wave w takes 1 KiB
// block 4 k + w); XCD: tiles remapped so each XCD streams one contiguous eighth of the batch
template <int IF, int JOINT, int XCD>
__global__ void __launch_bounds__(256) k_var(const uint8_t *fr, uint32_t bytes, const uint32_t *off,
                                             const uint32_t *len, uint32_t n, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, bytes);
    const uint32_t nt = gridDim.x;
    const uint32_t tile = XCD ? (blockIdx.x % 8u) * (nt / 8u) + blockIdx.x / 8u : blockIdx.x;
    uint32_t s = 0;
    if (JOINT) {
        for (uint32_t st = 0; st < 16; st += 4) {
            const uint32_t f0 = tile * 1024 + st * 64;
            const uint32_t fl = min(n, f0 + 256) - 1;
            const uint32_t A = off[f0] & ~127u, E = off[fl] + len[fl];
            for (uint32_t g = A + 1024u * w; g < E; g += 4096u * IF) {
                __attribute__((ext_vector_type(4))) uint32_t v[IF];
#pragma unroll
                for (int c = 0; c < IF; ++c) {
                    const uint32_t a = g + 4096u * c + 16u * lane;
                    v[c] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(a < E ? a : 0xFFFFFFF0u), 0, 0);
                }
#pragma unroll
                for (int c = 0; c < IF; ++c) s = sum4(v[c], s);
            }
        }
    } else {
        for (uint32_t st = w; st < 16; st += 4) {
            const uint32_t f0 = tile * 1024 + st * 64;
            const uint32_t fl = min(n, f0 + 64) - 1;
            const uint32_t A = off[f0] & ~127u, E = off[fl] + len[fl];
            for (uint32_t g = A; g < E; g += 4096u * IF) {
                __attribute__((ext_vector_type(4))) uint32_t v[4 * IF];
#pragma unroll
                for (int c = 0; c < 4 * IF; ++c) {
                    const uint32_t a = g + 1024u * c + 16u * lane;
                    v[c] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(a < E ? a : 0xFFFFFFF0u), 0, 0);
                }
#pragma unroll
                for (int c = 0; c < 4 * IF; ++c) s = sum4(v[c], s);
            }
        }
    }
    if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_flat(const uint4 *p, uint32_t n16, uint32_t *out)
{
    uint32_t s = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) {
        const uint4 v = p[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x9E3779B9u) out[threadIdx.x] = s;
}

int main(int argc, char **argv)
{
    const bool imix = argc > 1 && !strcmp(argv[1], "imix");
    const uint32_t N = 1u << 20;
    std::vector<uint32_t> off(N), len(N);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < N; ++i) {
        uint32_t l = 1500;
        if (imix) {
            const uint32_t r = (i * 2654435761u >> 16) % 12u;
            l = r < 7 ? 64 : r < 11 ? 594 : 1500;
        }
        off[i] = (uint32_t)pos;
        len[i] = l;
        pos += l;
    }
    const uint32_t bytes = (uint32_t)((pos + 255) & ~255ull);
    uint8_t *fr;
    uint32_t *doff, *dlen, *out;
    (void)hipMalloc(&fr, bytes + 256);
    (void)hipMemset(fr, 3, bytes + 256);
    (void)hipMalloc(&doff, N * 4);
    (void)hipMalloc(&dlen, N * 4);
    (void)hipMemcpy(doff, off.data(), N * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dlen, len.data(), N * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 1u << 20);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[3] = {"k_span_chunk", "k_span_piece", "k_span_c128"};
    for (int rep = 0; rep < 5; ++rep) {
        for (int m = 0; m < 3; ++m) {
            (void)hipEventRecord(e0, 0);
            if (m == 0) hipLaunchKernelGGL(k_span<0>, dim3(N / 1024), dim3(256), 0, 0, fr, bytes, doff, dlen, N, out);
            if (m == 1) hipLaunchKernelGGL(k_span<1>, dim3(N / 1024), dim3(256), 0, 0, fr, bytes, doff, dlen, N, out);
            if (m == 2) hipLaunchKernelGGL(k_span<2>, dim3(N / 1024), dim3(256), 0, 0, fr, bytes, doff, dlen, N, out);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep == 4) printf("%s %.1f us\n", names[m], 1e3 * ms);
        }
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_flat, dim3(4096), dim3(256), 0, 0, (const uint4 *)fr, bytes / 16, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep == 4) printf("k_flat %.1f us\n", 1e3 * ms);
    }
    {
        struct V { const char *nm; void (*k)(const uint8_t *, uint32_t, const uint32_t *, const uint32_t *, uint32_t, uint32_t *); };
        const V vs[] = {{"if1", k_var<1, 0, 0>}, {"if2", k_var<2, 0, 0>}, {"if3", k_var<3, 0, 0>},
                        {"if2_xcd", k_var<2, 0, 1>}, {"joint2", k_var<2, 1, 0>}, {"joint4", k_var<4, 1, 0>},
                        {"joint2_xcd", k_var<2, 1, 1>}};
        for (const V &v : vs) {
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipEventRecord(e0, 0);
                hipLaunchKernelGGL(v.k, dim3(N / 1024), dim3(256), 0, 0, fr, bytes, doff, dlen, N, out);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf("k_var %-10s %.1f us (best of 5)\n", v.nm, 1e3 * best);
        }
    }
    (void)hipDeviceSynchronize();
    printf("%s frames %u bytes %.1f MB; FETCH_SIZE (KiB) expected at x2: %.0f\n", imix ? "IMIX" : "1500B", N,
           pos / 1e6, pos / 2048.0);
    return 0;
}
