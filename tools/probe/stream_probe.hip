// Streaming floor for the 64 B-frame batch: 1 M frames x 64 B (64 MiB) read, one u32 per frame
// written, rotated over 10 device copies (> the 256 MiB Infinity Cache). Variants differ only in
// launch geometry and how many 16-byte loads each lane keeps in flight:
//   lane1   lane = frame, 4 x 16 B per lane, one frame per thread, N/256 workgroups (no loop)
//   laneS   lane = frame, S steps per wave, loads of step s+1 in flight while step s is summed
//   laneA   lane = frame, all S steps' loads issued up front (4 S loads in flight per lane)
//   coal    wave reads 4 contiguous KiB per step; per-frame sums via LDS
//   flat    uint4 grid-stride read of the whole buffer (no per-frame work), one u32 per 16 lanes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint32_t s4(uint4 v) { return v.x + v.y + v.z + v.w; }

__global__ void __launch_bounds__(256) k_lane1(const uint4 *fr, uint32_t *out)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    const uint4 a0 = fr[f * 4], a1 = fr[f * 4 + 1], a2 = fr[f * 4 + 2], a3 = fr[f * 4 + 3];
    out[f] = s4(a0) ^ s4(a1) ^ s4(a2) ^ s4(a3);
}

template <int S>
__global__ void __launch_bounds__(256) k_laneS(const uint4 *fr, uint32_t *out)
{
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = blockIdx.x * (256 * S) + w * 64 + lane;
    uint4 a0 = fr[f0 * 4], a1 = fr[f0 * 4 + 1], a2 = fr[f0 * 4 + 2], a3 = fr[f0 * 4 + 3];
    for (int s = 0; s < S; ++s) {
        const uint32_t f = f0 + s * 256;
        const uint32_t fn = f + (s + 1 < S ? 256 : 0);
        const uint4 b0 = fr[fn * 4], b1 = fr[fn * 4 + 1], b2 = fr[fn * 4 + 2], b3 = fr[fn * 4 + 3];
        out[f] = s4(a0) ^ s4(a1) ^ s4(a2) ^ s4(a3);
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
    }
}

template <int S>
__global__ void __launch_bounds__(256) k_laneA(const uint4 *fr, uint32_t *out)
{
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t f0 = blockIdx.x * (256 * S) + w * 64 + lane;
    uint4 a[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
        for (int c = 0; c < 4; ++c) a[s][c] = fr[(f0 + s * 256) * 4 + c];
#pragma unroll
    for (int s = 0; s < S; ++s) out[f0 + s * 256] = s4(a[s][0]) ^ s4(a[s][1]) ^ s4(a[s][2]) ^ s4(a[s][3]);
}

template <int S>
__global__ void __launch_bounds__(256) k_coal(const uint4 *fr, uint32_t *out)
{
    __shared__ uint32_t part[4][256];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t c0 = (blockIdx.x * (256 * S) + w * 64) * 4;
    uint4 a0 = fr[c0 + lane], a1 = fr[c0 + 64 + lane], a2 = fr[c0 + 128 + lane], a3 = fr[c0 + 192 + lane];
    for (int s = 0; s < S; ++s) {
        const uint32_t c = c0 + s * 1024;
        const uint32_t cn = c + (s + 1 < S ? 1024 : 0);
        const uint4 b0 = fr[cn + lane], b1 = fr[cn + 64 + lane], b2 = fr[cn + 128 + lane], b3 = fr[cn + 192 + lane];
        part[w][lane] = s4(a0); part[w][64 + lane] = s4(a1); part[w][128 + lane] = s4(a2); part[w][192 + lane] = s4(a3);
        __builtin_amdgcn_wave_barrier();
        const uint32_t v = part[w][lane * 4] ^ part[w][lane * 4 + 1] ^ part[w][lane * 4 + 2] ^ part[w][lane * 4 + 3];
        __builtin_amdgcn_wave_barrier();
        out[blockIdx.x * (256 * S) + w * 64 + s * 256 + lane] = v;
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
    }
}


// classify's shape: descriptor indirection (u32 offset + u16 length arrays), window loads one
// step ahead issued from descriptors loaded two steps ahead; LDS=1 stages the verdict words in
// LDS and stores them once per tile
template <int S, int LDS>
__global__ void __launch_bounds__(256) k_ind(const uint8_t *fr, const uint32_t *off, const uint16_t *len, uint32_t *out)
{
    __shared__ uint32_t stage[256 * S];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t0 = blockIdx.x * (256 * S);
    auto ld = [&](int s, uint32_t &o, uint32_t &l) { const uint32_t i = t0 + (s < S ? s : S - 1) * 256 + w * 64 + lane; o = off[i]; l = len[i]; };
    auto win = [&](uint32_t o, uint4 (&a)[4]) { const uint4 *p = (const uint4 *)(fr + o); a[0] = p[0]; a[1] = p[1]; a[2] = p[2]; a[3] = p[3]; };
    uint32_t co, cl, no, nl;
    ld(0, co, cl);
    uint4 A[4];
    win(co, A);
    ld(1, no, nl);
    for (int s = 0; s < S; ++s) {
        uint4 B[4];
        win(no, B);
        uint32_t nno, nnl;
        ld(s + 2, nno, nnl);
        const uint32_t v = (s4(A[0]) ^ s4(A[1]) ^ s4(A[2]) ^ s4(A[3])) + cl;
        if (LDS) stage[s * 256 + w * 64 + lane] = v; else out[t0 + s * 256 + w * 64 + lane] = v;
        A[0] = B[0]; A[1] = B[1]; A[2] = B[2]; A[3] = B[3];
        co = no; cl = nl; no = nno; nl = nnl;
    }
    if (LDS) {
        __syncthreads();
        uint4 *d4 = (uint4 *)(out + t0);
        for (uint32_t i = threadIdx.x; i < 64 * S; i += 256) d4[i] = ((const uint4 *)stage)[i];
    }
}

// all of the wave's descriptors loaded up front, windows two steps ahead
template <int S>
__global__ void __launch_bounds__(256) k_ind2(const uint8_t *fr, const uint32_t *off, const uint16_t *len, uint32_t *out)
{
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t0 = blockIdx.x * (256 * S);
    uint32_t o[S], l[S];
#pragma unroll
    for (int s = 0; s < S; ++s) { o[s] = off[t0 + s * 256 + w * 64 + lane]; l[s] = len[t0 + s * 256 + w * 64 + lane]; }
    uint4 A[S][4];
#pragma unroll
    for (int s = 0; s < S; ++s) { const uint4 *p = (const uint4 *)(fr + o[s]); A[s][0] = p[0]; A[s][1] = p[1]; A[s][2] = p[2]; A[s][3] = p[3]; }
#pragma unroll
    for (int s = 0; s < S; ++s) out[t0 + s * 256 + w * 64 + lane] = (s4(A[s][0]) ^ s4(A[s][1]) ^ s4(A[s][2]) ^ s4(A[s][3])) + l[s];
}


// k_ind<4,1> with rx_classify's extra features switched on one at a time (F bits):
//   1 buffer loads (range-checked resource) instead of global loads
//   2 the fifth-dword OOB buffer load per lane
//   4 XCD-aware tile remap
//   8 funnel shift (ballots, lane selects, alignbyte) of the window
//  16 tile-end counter reduction (DPP scans) + per-tile row stores
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb)
{
    if (nb < 16) return b;
    const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}
__device__ __forceinline__ uint32_t scan_dpp(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}
__device__ __forceinline__ uint32_t lane_select(unsigned long long m, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
template <int F>
__global__ void __launch_bounds__(256, 5) k_feat(const uint8_t *fr, const uint32_t *off, const uint16_t *len, uint32_t *out, uint32_t nbytes, uint32_t *rows)
{
    constexpr int S = 4;
    __shared__ uint32_t stage[256 * S];
    __shared__ uint32_t cnt[4][16];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t tile = (F & 4) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t t0 = tile * (256 * S);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(fr), (short)0, (int)nbytes, 0x00020000);
    auto ld = [&](int s, uint32_t &o, uint32_t &l) { const uint32_t i = t0 + (s < S ? s : S - 1) * 256 + w * 64 + lane; o = off[i]; l = len[i]; };
    auto win = [&](uint32_t o, uint4 (&a)[4], uint32_t &c4) {
        if (F & 1) {
            const uint32_t ab = (o + 12u) & ~15u;
#pragma unroll
            for (int c = 0; c < 4; ++c) { const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(ab + 16 * c), 0, 0); a[c] = make_uint4(v[0], v[1], v[2], v[3]); }
        } else {
            const uint4 *p = (const uint4 *)(fr + o); a[0] = p[0]; a[1] = p[1]; a[2] = p[2]; a[3] = p[3];
        }
        c4 = 0;
        if (F & 2) { const uint32_t o4 = ((o + 12u) & 15u) > 12u ? ((o + 12u) & ~15u) + 64u : nbytes; c4 = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)o4, 0, 0); }
    };
    uint32_t acc0 = 0, acc1 = 0, acc2 = 0;
    uint32_t co, cl, no, nl, c4a, c4b;
    extern __shared__ uint32_t dyn[];
    if (F & 64) {
        for (uint32_t i = threadIdx.x; i < 1024; i += 256) dyn[4096 + i] = 0;
        __syncthreads();
    }
    if (F & 32) {
        uint32_t o_[4], l_[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { o_[i] = off[t0 + i * 256 + threadIdx.x]; l_[i] = len[t0 + i * 256 + threadIdx.x]; }
#pragma unroll
        for (int i = 0; i < 4; ++i) { dyn[i * 256 + threadIdx.x] = o_[i]; dyn[1024 + i * 256 + threadIdx.x] = l_[i]; }
        __syncthreads();
        auto rd = [&](int s_, uint32_t &o, uint32_t &l) { const uint32_t i = (s_ < S ? s_ : S - 1) * 256 + w * 64 + lane; o = dyn[i]; l = dyn[1024 + i]; };
        rd(0, co, cl);
        rd(1, no, nl);
    } else {
        ld(0, co, cl);
        ld(1, no, nl);
    }
    uint4 A[4];
    win(co, A, c4a);
    for (int s = 0; s < S; ++s) {
        uint4 B[4];
        win(no, B, c4b);
        uint32_t nno, nnl;
        if (F & 32) { const uint32_t i = (s + 2 < S ? s + 2 : S - 1) * 256 + w * 64 + lane; nno = dyn[i]; nnl = dyn[1024 + i]; }
        else ld(s + 2, nno, nnl);
        uint32_t v;
        if (F & 8) {
            uint32_t wd[17], w1[16], w2[14], g[13];
            const uint32_t sh = (co + 12u) & 15u, s3 = sh & 3u;
#pragma unroll
            for (int i = 0; i < 4; ++i) { wd[4 * i] = A[i].x; wd[4 * i + 1] = A[i].y; wd[4 * i + 2] = A[i].z; wd[4 * i + 3] = A[i].w; }
            wd[16] = c4a;
            const unsigned long long m4 = __ballot((sh & 4u) != 0u), m8 = __ballot((sh & 8u) != 0u);
#pragma unroll
            for (int i = 0; i < 16; ++i) w1[i] = lane_select(m4, wd[i], wd[i + 1]);
#pragma unroll
            for (int i = 0; i < 14; ++i) w2[i] = lane_select(m8, w1[i], w1[i + 2]);
#pragma unroll
            for (int i = 0; i < 13; ++i) g[i] = __builtin_amdgcn_alignbyte(w2[i + 1], w2[i], s3);
            v = 0;
#pragma unroll
            for (int i = 0; i < 13; ++i) v ^= g[i];
        } else {
            v = (s4(A[0]) ^ s4(A[1]) ^ s4(A[2]) ^ s4(A[3])) + c4a;
        }
        v += cl;
        acc0 += v & 0xFF; acc1 += (v >> 8) & 0xFF; acc2 += cl;
        stage[s * 256 + w * 64 + lane] = v;
        A[0] = B[0]; A[1] = B[1]; A[2] = B[2]; A[3] = B[3]; c4a = c4b;
        co = no; cl = nl; no = nno; nl = nnl;
    }
    if (F & 16) {
        const uint32_t x0 = __builtin_amdgcn_readlane((int)scan_dpp(acc0), 63);
        const uint32_t x1 = __builtin_amdgcn_readlane((int)scan_dpp(acc1), 63);
        const uint32_t x2 = __builtin_amdgcn_readlane((int)scan_dpp(acc2), 63);
        if (lane < 3) cnt[w][lane] = lane == 0 ? x0 : lane == 1 ? x1 : x2;
    }
    __syncthreads();
    uint4 *d4 = (uint4 *)(out + t0);
    for (uint32_t i = threadIdx.x; i < 64 * S; i += 256) d4[i] = ((const uint4 *)stage)[i];
    if ((F & 16) && threadIdx.x < 16) rows[tile * 16 + threadIdx.x] = cnt[0][threadIdx.x & 3] + cnt[1][threadIdx.x & 3];
}


// S steps per wave, P windows in flight ahead (descriptors for all S steps loaded up front into
// LDS by the wave itself, no barrier)
template <int S, int P, int C = 0>
__global__ void __launch_bounds__(256) k_indp(const uint8_t *fr, const uint32_t *off, const uint16_t *len, uint32_t *out)
{
    __shared__ uint32_t d[4][S * 64];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t0 = blockIdx.x * (256 * S);
    // wave w: steps st = w + 4 j, j < S
    uint32_t o0 = off[t0 + w * 64 + lane];
    uint32_t l0 = len[t0 + w * 64 + lane];
    uint32_t ot[S], lt[S];
#pragma unroll
    for (int j = 1; j < S; ++j) { ot[j] = off[t0 + (w + 4 * j) * 64 + lane]; lt[j] = len[t0 + (w + 4 * j) * 64 + lane]; }
    uint4 A[P + 1][4];
    {
        const uint4 *p = (const uint4 *)(fr + o0); A[0][0] = p[0]; A[0][1] = p[1]; A[0][2] = p[2]; A[0][3] = p[3];
    }
#pragma unroll
    for (int j = 1; j < S; ++j) { d[w][j * 64 + lane] = ot[j]; d[w][S * 64 - 64 + lane] = d[w][S * 64 - 64 + lane]; }
    // lengths kept in regs (only step use)
#pragma unroll
    for (int j = 1; j <= P && j < S; ++j) {
        const uint4 *p = (const uint4 *)(fr + ot[j]); A[j][0] = p[0]; A[j][1] = p[1]; A[j][2] = p[2]; A[j][3] = p[3];
    }
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const int b = j % (P + 1);
        if (j + P + 1 < S) {
            // issue before consuming (the buffer being consumed is b; the new one goes to (j+P+1)%(P+1) == b)
        }
        uint32_t v = (s4(A[b][0]) ^ s4(A[b][1]) ^ s4(A[b][2]) ^ s4(A[b][3])) + (j ? lt[j] : l0);
        // C full-rate VALU ops (4 independent chains) emulating the per-frame parse work
        uint32_t c0 = v, c1 = A[b][1].y, c2 = A[b][2].z, c3 = A[b][3].w;
#pragma unroll
        for (int k = 0; k < C / 4; ++k) {
            c0 = __builtin_amdgcn_alignbyte(c0, c1, k & 3);
            c1 = c1 ^ c2;
            c2 = __builtin_amdgcn_alignbyte(c2, c3, (k + 1) & 3);
            c3 = c3 + c0;
        }
        v += c0 ^ c1 ^ c2 ^ c3;
        out[t0 + (w + 4 * j) * 64 + lane] = v;
        if (j + P + 1 < S) {
            const uint4 *p = (const uint4 *)(fr + d[w][(j + P + 1) * 64 + lane]); A[b][0] = p[0]; A[b][1] = p[1]; A[b][2] = p[2]; A[b][3] = p[3];
        }
    }
}


// window loaded straight from frame byte 12 (unaligned: 3 x 16 B + 4 B = bytes 12..63) with
// buffer loads, U=1; aligned 4 x 16 B from (o + 12) & ~15, U=0
template <int U>
__global__ void __launch_bounds__(256) k_unal(const uint8_t *fr, const uint32_t *off, const uint16_t *len, uint32_t *out, uint32_t nbytes)
{
    constexpr int S = 4;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t0 = blockIdx.x * (256 * S);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(fr), (short)0, (int)nbytes, 0x00020000);
    uint32_t o[S], l[S];
#pragma unroll
    for (int s = 0; s < S; ++s) { o[s] = off[t0 + s * 256 + w * 64 + lane]; l[s] = len[t0 + s * 256 + w * 64 + lane]; }
    uint32_t acc = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
        uint32_t x = 0;
        if (U) {
            const uint32_t b = o[s] + 12u;
#pragma unroll
            for (int c = 0; c < 3; ++c) { const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(b + 16 * c), 0, 0); x ^= v[0] + v[1] + v[2] + v[3]; }
            x ^= __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(b + 48), 0, 0);
        } else {
            const uint32_t b = (o[s] + 12u) & ~15u;
#pragma unroll
            for (int c = 0; c < 4; ++c) { const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(b + 16 * c), 0, 0); x ^= v[0] + v[1] + v[2] + v[3]; }
        }
        out[t0 + s * 256 + w * 64 + lane] = x + l[s];
    }
    (void)acc;
}

__global__ void __launch_bounds__(256) k_flat(const uint4 *fr, uint32_t *out, uint32_t n16)
{
    const uint32_t stride = gridDim.x * 256;
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) acc ^= s4(fr[i]);
    // 4 MiB of output like the per-frame kernels: one u32 per 16 input bytes / 4
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t < n16 / 4) out[t] = acc;
}

int main()
{
    const size_t N = getenv("PROBE_N") ? (size_t)atol(getenv("PROBE_N")) : (1u << 20), COPIES = 10;
    uint4 *fr; uint32_t *out;
    (void)hipMalloc(&fr, N * 64 * COPIES);
    (void)hipMalloc(&out, N * 4);
    (void)hipMemset(fr, 1, N * 64 * COPIES);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    auto time = [&](const char *name, auto launch) {
        for (int i = 0; i < 10; ++i) launch(fr + (i % COPIES) * N * 4);
        (void)hipEventRecord(e0, 0);
        const int R = getenv("PROBE_REPS") ? atoi(getenv("PROBE_REPS")) : 200;
        for (int i = 0; i < R; ++i) launch(fr + (i % COPIES) * N * 4);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / R;
        printf("%-14s %7.2f us per launch, %.2f TB/s (68 MiB)\n", name, us, (N * 68.0) / us / 1e6);
    };
    time("lane1", [&](const uint4 *f) { hipLaunchKernelGGL(k_lane1, dim3(N / 256), dim3(256), 0, 0, f, out); });
    time("laneS2", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneS<2>, dim3(N / 512), dim3(256), 0, 0, f, out); });
    time("laneS4", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneS<4>, dim3(N / 1024), dim3(256), 0, 0, f, out); });
    time("laneS8", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneS<8>, dim3(N / 2048), dim3(256), 0, 0, f, out); });
    time("laneA2", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneA<2>, dim3(N / 512), dim3(256), 0, 0, f, out); });
    time("laneA4", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneA<4>, dim3(N / 1024), dim3(256), 0, 0, f, out); });
    time("coal1", [&](const uint4 *f) { hipLaunchKernelGGL(k_coal<1>, dim3(N / 256), dim3(256), 0, 0, f, out); });
    time("coal4", [&](const uint4 *f) { hipLaunchKernelGGL(k_coal<4>, dim3(N / 1024), dim3(256), 0, 0, f, out); });
    time("laneS16", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneS<16>, dim3(N / 4096), dim3(256), 0, 0, f, out); });
    time("laneS32", [&](const uint4 *f) { hipLaunchKernelGGL(k_laneS<32>, dim3(N / 8192), dim3(256), 0, 0, f, out); });
    time("coal16", [&](const uint4 *f) { hipLaunchKernelGGL(k_coal<16>, dim3(N / 4096), dim3(256), 0, 0, f, out); });
    time("coal32", [&](const uint4 *f) { hipLaunchKernelGGL(k_coal<32>, dim3(N / 8192), dim3(256), 0, 0, f, out); });
    for (int g : {1024, 2048, 4096, 8192, 16384})
        time(g == 1024 ? "flat1024" : g == 2048 ? "flat2048" : g == 4096 ? "flat4096" : g == 8192 ? "flat8192" : "flat16384",
             [&](const uint4 *f) { hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, 0, f, out, (uint32_t)(N * 4)); });

    uint32_t *offs; uint16_t *lens;
    (void)hipMalloc(&offs, N * 4 * COPIES);
    (void)hipMalloc(&lens, N * 2 * COPIES);
    {
        uint32_t *h = (uint32_t *)malloc(N * 4 * COPIES); uint16_t *hl = (uint16_t *)malloc(N * 2 * COPIES);
        for (size_t i = 0; i < N * COPIES; ++i) { h[i] = (uint32_t)((i % N) * 64); hl[i] = 64; }
        (void)hipMemcpy(offs, h, N * 4 * COPIES, hipMemcpyHostToDevice);
        (void)hipMemcpy(lens, hl, N * 2 * COPIES, hipMemcpyHostToDevice);
    }
    auto timei = [&](const char *name, auto launch) {
        for (int i = 0; i < 10; ++i) launch((const uint8_t *)(fr + (i % COPIES) * N * 4), offs + (i % COPIES) * N, lens + (i % COPIES) * N);
        (void)hipEventRecord(e0, 0);
        const int R = getenv("PROBE_REPS") ? atoi(getenv("PROBE_REPS")) : 200;
        for (int i = 0; i < R; ++i) launch((const uint8_t *)(fr + (i % COPIES) * N * 4), offs + (i % COPIES) * N, lens + (i % COPIES) * N);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / R;
        printf("%-14s %7.2f us per launch, %.2f TB/s (74 MiB)\n", name, us, (N * 74.0) / us / 1e6);
    };
    timei("ind1", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind<1, 0>), dim3(N / 256), dim3(256), 0, 0, f, o, l, out); });
    timei("ind2", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind<2, 0>), dim3(N / 512), dim3(256), 0, 0, f, o, l, out); });
    timei("ind4", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind<4, 0>), dim3(N / 1024), dim3(256), 0, 0, f, o, l, out); });
    timei("ind4lds", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind<4, 1>), dim3(N / 1024), dim3(256), 0, 0, f, o, l, out); });
    timei("ind2lds", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind<2, 1>), dim3(N / 512), dim3(256), 0, 0, f, o, l, out); });
    timei("ind2all", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind2<2>), dim3(N / 512), dim3(256), 0, 0, f, o, l, out); });
    timei("ind4all", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind2<4>), dim3(N / 1024), dim3(256), 0, 0, f, o, l, out); });
    timei("ind1all", [&](const uint8_t *f, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_ind2<1>), dim3(N / 256), dim3(256), 0, 0, f, o, l, out); });

    uint32_t *rows; (void)hipMalloc(&rows, 4096 * 64);
#define FEAT(f) timei("feat" #f, [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_feat<f>), dim3(N / 1024), dim3(256), 17920, 0, f_, o, l, out, (uint32_t)(N * 64), rows); })
    FEAT(121);

#define INDP(S_, P_, C_) timei("indp" #S_ "_" #P_ "_c" #C_, [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_indp<S_, P_, C_>), dim3(N / (256 * S_)), dim3(256), 0, 0, f_, o, l, out); })
    INDP(4, 1, 0);
    timei("unal0", [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_unal<0>), dim3(N / 1024), dim3(256), 0, 0, f_, o, l, out, (uint32_t)(N * 64)); });
    timei("unal1", [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_unal<1>), dim3(N / 1024), dim3(256), 0, 0, f_, o, l, out, (uint32_t)(N * 64)); });
    timei("unal0", [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_unal<0>), dim3(N / 1024), dim3(256), 0, 0, f_, o, l, out, (uint32_t)(N * 64)); });
    timei("unal1", [&](const uint8_t *f_, const uint32_t *o, const uint16_t *l) { hipLaunchKernelGGL((k_unal<1>), dim3(N / 1024), dim3(256), 0, 0, f_, o, l, out, (uint32_t)(N * 64)); });
    return 0;
}
