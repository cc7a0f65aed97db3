// rx_classify's per-wave chain in isolation (round 5): descriptors -> header windows -> step
// arithmetic -> staged verdict words -> tile-end store, over 1 M x 64 B frames (10 rotated device
// copies), back-to-back launches on one stream. Varies the tile (S steps per wave, T = 256 S frames
// per 4-wave workgroup), the windows in flight per wave (K steps ahead, K + 1 register windows
// live) and the arithmetic per step (ALU rounds of the synthetic checksum chain). The question:
// which shape brings the chain to the plain-read floor (tools/probe/stream_probe.hip, ind4 ≈ 14 us).
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/chain_probe tools/probe/chain_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

struct Win {
    uint4 a, b, c;
    uint2 d;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint4 load16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ Win load_win(__amdgpu_buffer_rsrc_t fr, uint32_t o)
{
    const uint32_t b = (o + 12u) & ~3u;
    Win r;
    r.a = load16(fr, b);
    r.b = load16(fr, b + 16u);
    r.c = load16(fr, b + 32u);
    const auto d = __builtin_amdgcn_raw_buffer_load_b64(fr, (int)(b + 48u), 0, 0);
    r.d = make_uint2(d[0], d[1]);
    return r;
}

// the step's arithmetic: funnel to frame-relative words, then ALU rounds of sums over them
// (PRE rounds before the next window is issued, POST after: the real kernel issues it after
// about two thirds of its step work, tools/probe/chain_probe.hip header)
struct Acc {
    uint32_t g[13];
    uint32_t a, b;
};

__device__ __forceinline__ void funnel(Acc &c, const Win &W, uint32_t off, uint32_t len)
{
    const uint32_t D[14] = {W.a.x, W.a.y, W.a.z, W.a.w, W.b.x, W.b.y, W.b.z, W.b.w,
                            W.c.x, W.c.y, W.c.z, W.c.w, W.d.x, W.d.y};
    const uint32_t sh = off & 3u;
#pragma unroll
    for (int i = 0; i < 13; ++i) c.g[i] = __builtin_amdgcn_alignbyte(D[i + 1], D[i], sh);
    c.a = len;
    c.b = off;
#pragma unroll
    for (int i = 0; i < 13; ++i) c.a ^= c.g[i];
}

template <int R0, int R1>
__device__ __forceinline__ void rounds(Acc &c)
{
#pragma unroll
    for (int r = R0; r < R1; ++r) {
        const int i = r % 13;
        c.a = __builtin_amdgcn_sad_u16(c.g[i] ^ (uint32_t)r, 0u, c.a);
        c.b = (c.b & 0xFFFFu) + (c.b >> 16) + (c.g[(i + 5) % 13] & 0xFF00FFu);
    }
}

// S steps per wave (T = 256 S frames per workgroup), K windows ahead, PRE / POST rounds of
// arithmetic before / after the next window's issue (the window of step s + K)
template <int S, int K, int PRE, int POST>
__global__ void __launch_bounds__(256)
k_chain(const uint8_t *fr, uint32_t fbytes, const uint32_t *off, const uint16_t *len, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint32_t stage[256 * S];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = tid & 63u;
    const uint32_t t0 = blockIdx.x * (256u * S);
    const __amdgpu_buffer_rsrc_t r = make_rsrc(fr, fbytes);
    // every step's descriptor (step s of wave w = frames t0 + 64 (4 s + w) + lane)
    uint32_t o[S], l[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const uint32_t p = t0 + 64u * (4u * s + w) + lane;
        o[s] = off[p];
        l[s] = len[p];
    }
    Win W[K + 1];
#pragma unroll
    for (int s = 0; s < K && s < S; ++s) W[s] = load_win(r, o[s]);
    // keep the window loads where they are written: the scheduler otherwise sinks them to their
    // uses (to hold occupancy), which leaves one window in flight whatever K says
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        Acc c;
        funnel(c, W[s % (K + 1)], o[s], l[s]);
        rounds<0, PRE>(c);
        __builtin_amdgcn_sched_barrier(0);
        if (s + K < S) W[(s + K) % (K + 1)] = load_win(r, o[s + K]);
        __builtin_amdgcn_sched_barrier(0);
        rounds<PRE, PRE + POST>(c);
        stage[64u * (4u * s + w) + lane] = c.a ^ c.b;
    }
    __syncthreads();
    const uint4 *s4 = reinterpret_cast<const uint4 *>(stage);
    uint4 *d4 = reinterpret_cast<uint4 *>(out + t0);
#pragma unroll
    for (int i = 0; i < S / 4; ++i) d4[tid + 256 * i] = s4[tid + 256 * i];
}

int main()
{
    const size_t N = 1u << 20, COPIES = 10;
    uint8_t *fr;
    uint32_t *out, *offs;
    uint16_t *lens;
    (void)hipMalloc(&fr, N * 64 * COPIES + 64);
    (void)hipMalloc(&out, N * 4);
    (void)hipMemset(fr, 1, N * 64 * COPIES + 64);
    (void)hipMalloc(&offs, N * 4 * COPIES);
    (void)hipMalloc(&lens, N * 2 * COPIES);
    {
        std::vector<uint32_t> h(N * COPIES);
        std::vector<uint16_t> hl(N * COPIES);
        for (size_t i = 0; i < N * COPIES; ++i) { h[i] = (uint32_t)((i % N) * 64); hl[i] = 64; }
        (void)hipMemcpy(offs, h.data(), N * 4 * COPIES, hipMemcpyHostToDevice);
        (void)hipMemcpy(lens, hl.data(), N * 2 * COPIES, hipMemcpyHostToDevice);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int R = getenv("PROBE_REPS") ? atoi(getenv("PROBE_REPS")) : 200;
    auto run = [&](const char *name, auto kern, int S) {
        const dim3 g((uint32_t)(N / (256u * S)));
        auto launch = [&](int i) {
            const size_t c = (size_t)(i % COPIES);
            hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, fr + c * N * 64, (uint32_t)(N * 64), offs + c * N,
                               lens + c * N, out);
        };
        for (int i = 0; i < 10; ++i) launch(i);
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < R; ++i) launch(i);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / R;
        printf("%-22s %7.2f us per launch, %.2f TB/s (74 MiB)\n", name, us, (N * 74.0) / us / 1e6);
        fflush(stdout);
    };
#define RUN(S, K, P0, P1) run("S" #S " K" #K " pre" #P0 " post" #P1, k_chain<S, K, P0, P1>, S)
    RUN(4, 1, 60, 20);      // the real kernel's shape: next window after 3/4 of the step
    RUN(4, 1, 0, 80);       // next window issued first
    RUN(4, 2, 0, 80);
    RUN(4, 3, 0, 80);
    RUN(4, 1, 0, 0);        // no arithmetic
    RUN(8, 1, 60, 20);
    RUN(8, 1, 0, 80);
    RUN(8, 2, 0, 80);
    RUN(8, 4, 0, 80);
    RUN(16, 2, 0, 80);
    RUN(16, 4, 0, 80);
    RUN(16, 6, 0, 80);
    RUN(4, 1, 120, 40);     // twice the arithmetic
    RUN(4, 1, 0, 160);
    RUN(4, 2, 0, 160);
    RUN(8, 4, 0, 160);
    RUN(16, 4, 0, 160);
    return 0;
}
