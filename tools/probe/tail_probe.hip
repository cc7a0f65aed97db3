// FETCH_SIZE calibration in rx_classify's tail-pass access shape (round 5).
// Frames of 1500 B (config 3) or IMIX sizes packed back to back; every frame's bytes [64, len)
// read as 64-byte super-chunks (four 16-byte loads) from the dword at or below offset + 64, the
// shape the tail pass uses. The host computes the exact set of 64-byte blocks and 128-byte lines
// those loads touch, so FETCH_SIZE per dispatch can be compared with a known byte count
// (MI355X_MICROARCH.md: x2 holds for wide coalesced streaming reads, other shapes uncalibrated).
//   kernels: k_tail   lane = chunk of the dispatch's chunk list (the sweep's address set)
//            k_flat   the same bytes as one contiguous coalesced stream (the known x2 case)
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/tail_probe tools/probe/tail_probe.hip
//   tail_probe [imix]      (run under rocprofv3 --pmc FETCH_SIZE, one pass per counter)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

// one 64-byte super-chunk per lane: chunk list entries are dword-aligned buffer offsets
__global__ void __launch_bounds__(256) k_tail(const uint8_t *fr, uint32_t bytes, const uint32_t *chunk, uint32_t n,
                                              uint32_t *out)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, bytes);
    const uint32_t b = i < n ? chunk[i] : 0xFFFFFFF0u;
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(b + 16u * c), 0, 0);
        s += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (s == 0x9E3779B9u) out[i] = s;
}

// the same chunks, piece-major inside each group of 64 chunks: instruction c of a wave covers
// chunks 16 c .. 16 c + 15 of its group, lanes 4 j .. 4 j + 3 the four pieces of chunk 16 c + j
// (consecutive lanes, consecutive 16 bytes: a chunk is one 64-byte request run)
__global__ void __launch_bounds__(256) k_tail_pm(const uint8_t *fr, uint32_t bytes, const uint32_t *chunk,
                                                 uint32_t n, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63u, g = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, bytes);
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t k = g * 64u + 16u * c + (lane >> 2);
        const uint32_t b = k < n ? chunk[k] + 16u * (lane & 3u) : 0xFFFFFFF0u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)b, 0, 0);
        s += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (s == 0x9E3779B9u) out[g] = s;
}

// the chunk-per-lane sweep from 64-byte aligned chunk starts (the block holding each start)
__global__ void __launch_bounds__(256) k_tail_a64(const uint8_t *fr, uint32_t bytes, const uint32_t *chunk,
                                                  uint32_t n, uint32_t *out)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, bytes);
    const uint32_t b = i < n ? chunk[i] & ~63u : 0xFFFFFFF0u;
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(b + 16u * c), 0, 0);
        s += v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (s == 0x9E3779B9u) out[i] = s;
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
    std::vector<uint32_t> chunk;
    std::set<uint64_t> b64, l128;
    uint64_t sweep = 0;
    for (uint32_t i = 0; i < N; ++i) {
        if (len[i] <= 64) continue;
        const uint32_t S = off[i] + 64, E = off[i] + len[i], Sa = S & ~3u;
        for (uint32_t c = Sa; c < E; c += 64) {
            chunk.push_back(c);
            const uint32_t ce = std::min<uint32_t>(c + 64, E);     // bytes of the datagram loaded
            sweep += 64;
            for (uint32_t x = c & ~63u; x < c + 64; x += 64) b64.insert(x);
            for (uint32_t x = c & ~127u; x < c + 64; x += 128) l128.insert(x);
            (void)ce;
        }
    }
    uint8_t *fr;
    uint32_t *dch, *out;
    (void)hipMalloc(&fr, bytes + 256);
    (void)hipMemset(fr, 3, bytes + 256);
    (void)hipMalloc(&dch, chunk.size() * 4);
    (void)hipMemcpy(dch, chunk.data(), chunk.size() * 4, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 1u << 24);
    // the same byte span as one stream: the tail bytes' 64-B blocks, here simply the whole buffer
    const uint32_t n = (uint32_t)chunk.size();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_tail, dim3((n + 255) / 256), dim3(256), 0, 0, fr, bytes, dch, n, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep == 4) printf("k_tail %.1f us\n", 1e3 * ms);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_tail_pm, dim3((n + 255) / 256), dim3(256), 0, 0, fr, bytes, dch, n, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep == 4) printf("k_tail_pm %.1f us\n", 1e3 * ms);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_tail_a64, dim3((n + 255) / 256), dim3(256), 0, 0, fr, bytes, dch, n, out);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep == 4) printf("k_tail_a64 %.1f us\n", 1e3 * ms);
        hipLaunchKernelGGL(k_flat, dim3(4096), dim3(256), 0, 0, (const uint4 *)fr, bytes / 16, out);
    }
    (void)hipDeviceSynchronize();
    printf("%s frames %u chunks %u; loaded (64 B per chunk) %.1f MB; unique 64-B blocks %.1f MB; unique 128-B lines %.1f MB; "
           "k_flat reads %.1f MB\n", imix ? "IMIX" : "1500B", N, n, sweep / 1e6, b64.size() * 64 / 1e6,
           l128.size() * 128 / 1e6, bytes / 1e6);
    printf("FETCH_SIZE (KiB) to expect at x2: tail %.0f (64-B blocks) or %.0f (128-B lines); flat %.0f\n",
           b64.size() * 64 / 2048.0, l128.size() * 128 / 2048.0, bytes / 2048.0);
    return 0;
}
