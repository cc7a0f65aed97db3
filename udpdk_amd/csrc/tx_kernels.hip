// tx_kernels.hip — gfx950 TX header build (udpdk_syscall.c:314-356) for a batch of datagrams.
//
// Per datagram: Ethernet (config MACs, type 0x0800), IPv4 (0x45, tos 0, total length, id 0,
// frag 0, ttl 64, proto 17, rte_ipv4_cksum, src = bound slot IP unless ANY else config IP,
// dst), UDP (raw src/dst ports, length, checksum 0), then the payload. The 42 header bytes of a
// wave's 64 datagrams are built by one lane each into an LDS window laid out with the output
// frame's 16-byte alignment; the output is then written as 16-byte chunks swept across lanes
// (whole chunks as one 16 B store, frame-boundary chunks byte-masked), the payload read with two
// aligned 16 B loads and a funnel shift. Bytes per datagram: len read + (len + 42) written +
// 4 x 4 B + 2 x 2 B descriptors.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

namespace {

__device__ __forceinline__ void wave_sync_tx()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t excl_scan64(uint32_t v, uint32_t *total)
{
    const uint32_t lane = __lane_id();
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ uint32_t win_mask(int a, int e, int i)
{
    int la = min(max(a - 4 * i, 0), 4);
    int le = min(max(e - 4 * i, 0), 4);
    uint32_t hm = le >= 4 ? 0xFFFFFFFFu : ((1u << (8 * le)) - 1u);
    uint32_t lm = la >= 4 ? 0xFFFFFFFFu : ((1u << (8 * la)) - 1u);
    return hm & ~lm;
}

__device__ __forceinline__ uint32_t sel4(uint32_t d, uint32_t a0, uint32_t a1, uint32_t a2,
                                         uint32_t a3)
{
    return d == 0 ? a0 : (d == 1 ? a1 : (d == 2 ? a2 : a3));
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// rte_raw_cksum + rte_ipv4_cksum of DPDK 20.05 over the 20-byte header built below
// (cksum field zero): raw == 0xffff is returned unchanged.
__device__ __forceinline__ uint32_t ipv4_cksum(uint32_t tl, uint32_t src, uint32_t dst)
{
    uint32_t s = 0x0045u + bswap16(tl) + 0x1140u + (src & 0xFFFFu) + (src >> 16) +
                 (dst & 0xFFFFu) + (dst >> 16);
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    s &= 0xFFFFu;
    return s == 0xFFFFu ? s : (~s & 0xFFFFu);
}

constexpr int TX_WIN = 64;  // bytes of header window per datagram (16 dwords)

} // namespace

__global__ void __launch_bounds__(TX_BLOCK)
tx_build(TxArgs a)
{
    __shared__ __attribute__((aligned(16))) uint32_t win[TX_BLOCK / 64][64][TX_WIN / 4];
    __shared__ uint32_t l_cs[TX_BLOCK / 64][64], l_fo[TX_BLOCK / 64][64],
        l_len[TX_BLOCK / 64][64], l_po[TX_BLOCK / 64][64];
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.payload), (short)0, (int)a.payload_rsrc, 0x00020000);
    const uint32_t waves_total = gridDim.x * (TX_BLOCK / 64);

    for (uint32_t g = blockIdx.x * (TX_BLOCK / 64) + w; g * 64 < a.n; g += waves_total) {
        const uint32_t i = g * 64 + lane;
        const bool valid = i < a.n;
        uint32_t fo = 0, L = 0, po = 0, nch = 0;
        if (valid) {
            fo = a.frame_off[i];
            L = a.payload_len[i];
            po = a.payload_off[i];
            const int32_t sock = a.sockfd[i];
            const bool ok = (uint64_t)fo + L + 42u <= a.frames_bytes &&
                            (uint64_t)po + L <= a.payload_bytes && sock >= 0 &&
                            (uint32_t)sock < a.n_slots;
            if (ok) {
                nch = ((fo & 15u) + L + 42u + 15u) >> 4;
                const uint4 sl = a.slots[sock];
                const uint32_t src = (sl.z && sl.x != 0u) ? sl.x : a.src_ip;   // :329-334
                const uint32_t dst = a.dst_ip[i];                               // :335
                const uint32_t tl = L + 28u;                                    // :336
                const uint32_t ul = L + 8u;                                     // :344
                const uint32_t ck = ipv4_cksum(tl, src, dst);                   // :337
                uint32_t h[12];
                h[0] = a.mac_lo[0]; h[1] = a.mac_lo[1]; h[2] = a.mac_lo[2];      // :315-317
                h[3] = 0x00450008u;                                 // type 0x0800, 0x45, tos 0
                h[4] = bswap16(tl);                                 // total length, id 0
                h[5] = 0x11400000u;                                 // frag 0, ttl 64, proto 17
                h[6] = ck | ((src & 0xFFFFu) << 16);
                h[7] = (src >> 16) | ((dst & 0xFFFFu) << 16);
                h[8] = (dst >> 16) | ((sl.y & 0xFFFFu) << 16);      // src port raw, :341
                h[9] = ((uint32_t)a.dst_port[i] & 0xFFFFu) | (bswap16(ul) << 16); // :342, :344
                h[10] = 0u;                                         // UDP checksum 0, :343
                h[11] = 0u;
                // shift into the frame's 16-byte alignment: byte r of the header lands at
                // window byte (fo & 15) + r
                const uint32_t sh = fo & 15u, s3 = sh & 3u, d0 = sh >> 2;
                uint32_t *wq = win[w][lane];
#pragma unroll
                for (int k = 0; k < 16; ++k) wq[k] = 0u;
#pragma unroll
                for (int k = 0; k < 12; ++k) {
                    const uint32_t prev = k ? h[k - 1] : 0u;
                    const uint32_t gk = s3 ? ((h[k] << (8u * s3)) | (prev >> (32u - 8u * s3))) : h[k];
                    wq[d0 + k] = gk;
                }
                if (s3) wq[d0 + 12] = h[11] >> (32u - 8u * s3);
            }
        }
        uint32_t total;
        const uint32_t cs = excl_scan64(nch, &total);
        l_cs[w][lane] = cs;
        l_fo[w][lane] = fo;
        l_len[w][lane] = L;
        l_po[w][lane] = po;
        wave_sync_tx();

        for (uint32_t k = lane; k < total; k += 64) {
            uint32_t q = 0;
#pragma unroll
            for (int sft = 32; sft >= 1; sft >>= 1)
                if (l_cs[w][q + sft] <= k) q += sft;
            const uint32_t j = k - l_cs[w][q];
            const uint32_t fq = l_fo[w][q], Lq = l_len[w][q], pq = l_po[w][q];
            const uint32_t abase = (fq & ~15u) + 16u * j;
            const int r0 = (int)(abase - fq);
            // header part
            uint32_t H[4] = {0u, 0u, 0u, 0u};
            if (j < 4) {
                const uint4 hv = *reinterpret_cast<const uint4 *>(&win[w][q][4 * j]);
                H[0] = hv.x; H[1] = hv.y; H[2] = hv.z; H[3] = hv.w;
            }
            // payload part: bytes at payload offset pq + r0 - 42 + b
            uint32_t P[4] = {0u, 0u, 0u, 0u};
            if (r0 + 16 > 42) {
                const int64_t src0 = (int64_t)pq + r0 - 42;
                const int64_t sa = src0 & ~(int64_t)15;
                const uint32_t sft = (uint32_t)(src0 - sa);       // 0..15
                const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)(uint32_t)sa, 0, 0);
                const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)(uint32_t)(sa + 16), 0, 0);
                const uint32_t wv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
                const uint32_t d = sft >> 2, s = sft & 3u;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t lo = sel4(d, wv[t], wv[t + 1], wv[t + 2], wv[t + 3]);
                    const uint32_t hi = sel4(d, wv[t + 1], wv[t + 2], wv[t + 3], wv[t + 4]);
                    P[t] = __builtin_amdgcn_alignbyte(hi, lo, s);
                }
            }
            uint32_t o[4], own[4];
            bool full = true;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t hm = win_mask(-r0, 42 - r0, t);
                const uint32_t pm = win_mask(42 - r0, 42 + (int)Lq - r0, t);
                o[t] = (H[t] & hm) | (P[t] & pm);
                own[t] = hm | pm;
                full = full && own[t] == 0xFFFFFFFFu;
            }
            uint8_t *dst = a.frames + abase;
            if (full) {
                *reinterpret_cast<uint4 *>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (own[t] == 0xFFFFFFFFu) {
                        *reinterpret_cast<uint32_t *>(dst + 4 * t) = o[t];
                    } else if (own[t]) {
                        for (int b = 0; b < 4; ++b)
                            if ((own[t] >> (8 * b)) & 0xFFu) dst[4 * t + b] = (uint8_t)(o[t] >> (8 * b));
                    }
                }
            }
        }
        wave_sync_tx();
    }
}

} // namespace udpdk
