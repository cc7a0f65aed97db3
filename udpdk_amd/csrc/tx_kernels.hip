// tx_kernels.hip — gfx950 TX header build (udpdk_syscall.c:314-356) for a batch of datagrams,
// with the poller's IPv4 fragmentation (udpdk_poller.c:461-501) when an MTU is given.
//
// Per datagram: Ethernet (config MACs, type 0x0800), IPv4 (0x45, tos 0, total length, id 0,
// frag 0, ttl 64, proto 17, rte_ipv4_cksum, src = bound slot IP unless ANY else config IP,
// dst), UDP (raw src/dst ports, length, checksum 0), then the payload.
//
// Fragmentation (mtu != 0 and len + 42 > mtu, the poller's pkt_len > IPV4_MTU_DEFAULT test):
// the IPv4 packet is cut the way DPDK 20.05 rte_ipv4_fragment_packet does (restated in
// oracle/udpdk_oracle.c): every fragment carries mtu - 20 bytes of the IP payload (UDP header +
// data), the last the remainder; each fragment repeats the Ethernet header and the IPv4 header
// with total length = 20 + its payload, fragment offset in 8-byte units and MF on all but the
// last. DPDK leaves the fragment header checksum 0 with PKT_TX_IP_CKSUM set, so the NIC fills
// it: here it is filled as the NIC would (~fold of the RFC 1071 sum). A datagram's frames are
// contiguous from frame_off[i]: fragment k at + k * (mtu + 14), so its span is
// (len + 8) + 34 * n_frames (len + 42 unfragmented).
//
// A wave takes 64 datagrams, expands them into output frames (one per datagram unless it is
// fragmented) and handles 64 frames per round: one lane builds a frame's 42 (or 34) header
// bytes into an LDS window laid out with the output frame's 16-byte alignment; the frames are
// then written as 16-byte chunks swept across lanes (whole chunks as one 16 B store,
// frame-boundary chunks byte-masked), the payload read with two aligned 16 B loads and a funnel
// shift. Bytes per datagram: len read + span written + 4 x 4 B + 2 x 2 B descriptors.
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

// Sum of the 20-byte IPv4 header built below (checksum field zero) as LE 16-bit words:
// version/IHL 0x45, tos 0, total length tl, id 0, fragment field ff (host order), ttl 64,
// proto 17, src, dst (raw).
__device__ __forceinline__ uint32_t ipv4_raw(uint32_t tl, uint32_t ff, uint32_t src, uint32_t dst)
{
    uint32_t s = 0x0045u + bswap16(tl) + bswap16(ff) + 0x1140u + (src & 0xFFFFu) + (src >> 16) +
                 (dst & 0xFFFFu) + (dst >> 16);
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    return s & 0xFFFFu;
}

// rte_ipv4_cksum of DPDK 20.05: raw == 0xffff is returned unchanged.
__device__ __forceinline__ uint32_t ipv4_cksum(uint32_t raw) { return raw == 0xFFFFu ? raw : (~raw & 0xFFFFu); }

// The checksum a NIC computes for PKT_TX_IP_CKSUM (fragments, rte_ipv4_fragment_packet leaves 0).
__device__ __forceinline__ uint32_t ipv4_cksum_nic(uint32_t raw) { return ~raw & 0xFFFFu; }

constexpr int TX_WIN = 64;  // bytes of header window per frame (16 dwords)
constexpr int TXW = TX_BLOCK / 64;

constexpr uint32_t TX_SMALL_SPAN = 80;       // frames up to this size take tx_small
constexpr uint32_t TX_SMALL_LOADS = (TX_SMALL_SPAN - 42u + 15u) / 16u;

// The frame of datagram i built in this lane's registers and stored as 16-byte pieces: for waves
// whose frames are all <= TX_SMALL_SPAN bytes and unfragmented. The payload loads go out with
// the slot lookup (byte-aligned 16-byte buffer loads; pieces past the payload are addressed out
// of range, so they cost no memory access and read as 0), so a wave's frames take one round
// trip after the descriptors instead of one per 64-chunk sweep step.
__device__ __forceinline__ void tx_small(const TxArgs &a, uint32_t i, uint32_t fo, uint32_t L,
                                         uint32_t po, int32_t sock)
{
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.payload), (short)0, (int)a.payload_rsrc, 0x00020000);
    const __amdgpu_buffer_rsrc_t fw = __builtin_amdgcn_make_buffer_rsrc(
        a.frames, (short)0, (int)a.frames_bytes, 0x00020000);
    const uint32_t span = L + 42u;
    const bool ok = i < a.n && (uint64_t)fo + span <= a.frames_bytes &&
                    (uint64_t)po + L <= a.payload_bytes && sock >= 0 && (uint32_t)sock < a.n_slots;
    uint32_t P[4 * TX_SMALL_LOADS + 1];
#pragma unroll
    for (uint32_t m = 0; m < TX_SMALL_LOADS; ++m) {
        // (a piece no lane needs is not issued: its lanes would still cost address-unit cycles)
        const bool need = ok && 16u * m < L;
        P[4 * m] = P[4 * m + 1] = P[4 * m + 2] = P[4 * m + 3] = 0u;
        if (__ballot(need)) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(pr, (int)(need ? po + 16u * m : 0x80000000u), 0, 0);
            P[4 * m] = v[0]; P[4 * m + 1] = v[1]; P[4 * m + 2] = v[2]; P[4 * m + 3] = v[3];
        }
    }
    P[4 * TX_SMALL_LOADS] = 0u;
    if (!ok) return;
    const uint4 sl = a.slots[sock];
    const uint32_t sq = (sl.z && sl.x != 0u) ? sl.x : a.src_ip;                    // :329-334
    const uint32_t dq = a.dst_ip[i];                                               // :335
    const uint32_t ptq = (sl.y & 0xFFFFu) | ((uint32_t)a.dst_port[i] << 16);        // :341-342
    const uint32_t tl = L + 28u, ul = L + 8u;                                      // :336, :344
    uint32_t H[10];
    H[0] = a.mac_lo[0]; H[1] = a.mac_lo[1]; H[2] = a.mac_lo[2];                    // :315-317
    H[3] = 0x00450008u;
    H[4] = bswap16(tl);
    H[5] = 0x11400000u;
    H[6] = ipv4_cksum(ipv4_raw(tl, 0u, sq, dq)) | ((sq & 0xFFFFu) << 16);          // :337
    H[7] = (sq >> 16) | ((dq & 0xFFFFu) << 16);
    H[8] = (dq >> 16) | ((ptq & 0xFFFFu) << 16);
    H[9] = (ptq >> 16) | (bswap16(ul) << 16);
    // frame dword d: the header for d < 10; then frame byte 42 + t = payload byte t, so dword
    // d >= 10 = payload bytes [4d - 42, 4d - 38) (bytes 40-41: UDP checksum 0)
    auto F = [&](uint32_t d) -> uint32_t {
        return d < 10u ? H[d] : (d == 10u ? P[0] << 16 : __builtin_amdgcn_alignbyte(P[d - 10u], P[d - 11u], 2));
    };
    // whole 16-byte pieces, then the frame's last 0-15 bytes as dword / byte stores
#pragma unroll
    for (uint32_t c = 0; c < TX_SMALL_SPAN / 16; ++c) {
        if (16u * c + 16u <= span) {
            const __attribute__((ext_vector_type(4))) uint32_t v = {F(4 * c), F(4 * c + 1), F(4 * c + 2), F(4 * c + 3)};
            __builtin_amdgcn_raw_buffer_store_b128(v, fw, (int)(fo + 16u * c), 0, 0);
        } else if (16u * c < span) {
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t b = 16u * c + 4u * t;
                if (b + 4u <= span) {
                    __builtin_amdgcn_raw_buffer_store_b32(F(4 * c + t), fw, (int)(fo + b), 0, 0);
                } else if (b < span) {
                    for (uint32_t k = 0; b + k < span; ++k)
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(F(4 * c + t) >> (8 * k)), fw, (int)(fo + b + k), 0, 0);
                }
            }
        }
    }
}

} // namespace

__global__ void __launch_bounds__(TX_BLOCK) __attribute__((amdgpu_waves_per_eu(6, 8)))
tx_build(TxArgs a)
{
    __shared__ __attribute__((aligned(16))) uint32_t win[TXW][64][TX_WIN / 4];
    // per output frame of the current round
    // (l_len bit 31: 34-byte header, a fragment after the first)
    __shared__ uint32_t l_cs[TXW][64], l_fo[TXW][64], l_len[TXW][64], l_po[TXW][64];
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.payload), (short)0, (int)a.payload_rsrc, 0x00020000);
    const uint32_t waves_total = gridDim.x * TXW;
    const uint32_t fpl = a.mtu ? a.mtu - 20u : 0u;      // IP payload bytes per full fragment

    // a.parts waves share each group of 64 datagrams: every one builds the group's headers and
    // takes every a.parts-th 64 chunks of its sweep (few large datagrams, e.g. 256 K datagrams
    // of 2952 B, are 4096 groups: one wave per group left 4 waves per SIMD, each a long sweep)
    const uint32_t groups = (a.n + 63u) / 64u;
    for (uint32_t gp = blockIdx.x * TXW + w; gp < groups * a.parts; gp += waves_total) {
        const uint32_t g = gp / a.parts, part = gp % a.parts;
        const uint32_t i = g * 64 + lane;
        uint32_t nf = 0, fo = 0, L = 0, po = 0, src = 0, dst = 0, pt = 0;
        int32_t sock = -1;
        if (i < a.n) {
            fo = a.frame_off[i];
            L = a.payload_len[i];
            po = a.payload_off[i];
            sock = a.sockfd[i];
        }
        // a wave of small unfragmented frames: one lane builds and stores its own frame
        if (!__ballot(i < a.n && (L + 42u > TX_SMALL_SPAN || (a.mtu && L + 42u > a.mtu)))) {
            if (part == 0u) tx_small(a, i, fo, L, po, sock);
            continue;
        }
        if (i < a.n) {
            const bool frag = a.mtu && L + 42u > a.mtu;                    // poller.c:466
            const uint32_t n_fr = frag ? (L + 8u + fpl - 1u) / fpl : 1u;
            const uint32_t span = frag ? L + 8u + 34u * n_fr : L + 42u;
            const bool ok = (uint64_t)fo + span <= a.frames_bytes &&
                            (uint64_t)po + L <= a.payload_bytes && sock >= 0 &&
                            (uint32_t)sock < a.n_slots;
            if (ok) {
                nf = n_fr;
                const uint4 sl = a.slots[sock];
                src = (sl.z && sl.x != 0u) ? sl.x : a.src_ip;                   // :329-334
                dst = a.dst_ip[i];                                               // :335
                pt = (sl.y & 0xFFFFu) | ((uint32_t)a.dst_port[i] << 16);          // :341-342
            }
        }
        // per datagram, kept in its lane's registers and read across lanes with shuffles:
        // first frame, frame offset, length | n_frames << 16 (fragmented), payload offset, src
        // ip, dst ip, src port | dst port << 16
        uint32_t n_frames;
        const uint32_t fs = excl_scan64(nf, &n_frames);
        const uint32_t ln = L | ((a.mtu && L + 42u > a.mtu) ? nf << 16 : 0u);

        // no fragmented datagram in the wave: frame = datagram = lane, no shuffles
        const bool direct = !__ballot(nf && (ln >> 16));
        for (uint32_t r0 = 0; r0 < (direct ? 1u : n_frames); r0 += 64) {
            const uint32_t f = r0 + lane;
            uint32_t nch = 0, ffo = 0, plen = 0, ppo = 0, hl = 0;
            uint32_t k = 0, lnq = ln, sq = src, dq = dst, ptq = pt, foq = fo, poq = po;
            bool act = nf != 0;
            if (!direct) {
                // the datagram of frame f: the last q with fs[q] <= f (datagrams without frames
                // share their successor's first index); shuffles run with every lane active
                const uint32_t fc = min(f, n_frames - 1u);
                uint32_t q = 0;
#pragma unroll
                for (int sft = 32; sft >= 1; sft >>= 1) {
                    const uint32_t v = __shfl(fs, (int)(q + sft), 64);
                    if (v <= fc) q += sft;
                }
                k = fc - __shfl(fs, (int)q, 64);
                lnq = __shfl(ln, (int)q, 64);
                sq = __shfl(src, (int)q, 64);
                dq = __shfl(dst, (int)q, 64);
                ptq = __shfl(pt, (int)q, 64);
                foq = __shfl(fo, (int)q, 64);
                poq = __shfl(po, (int)q, 64);
                act = f < n_frames;
            }
            const uint32_t Lq = lnq & 0xFFFFu, nfq = lnq >> 16;
            if (act) {
                uint32_t tl, ff, ck;
                if (!nfq) {                       // unfragmented: udpdk_sendto's frame as built
                    tl = Lq + 28u;                                               // :336
                    ff = 0u;
                    ck = ipv4_cksum(ipv4_raw(tl, 0u, sq, dq));                   // :337
                    hl = 42u;
                    ffo = foq;
                    ppo = poq;
                    plen = Lq;
                } else {                          // fragment k of nfq (rte_ipv4_fragment_packet)
                    const uint32_t ofs = k * fpl;
                    const bool last = k + 1u == nfq;
                    const uint32_t ipp = last ? Lq + 8u - ofs : fpl;
                    tl = 20u + ipp;
                    ff = (ofs >> 3) | (last ? 0u : 0x2000u);
                    ck = ipv4_cksum_nic(ipv4_raw(tl, ff, sq, dq));
                    hl = k ? 34u : 42u;
                    ffo = foq + k * (a.mtu + 14u);
                    ppo = poq + (k ? ofs - 8u : 0u);
                    plen = k ? ipp : ipp - 8u;
                }
                const uint32_t ul = Lq + 8u;                                     // :344
                uint32_t h[12];
                h[0] = a.mac_lo[0]; h[1] = a.mac_lo[1]; h[2] = a.mac_lo[2];      // :315-317
                h[3] = 0x00450008u;                                 // type 0x0800, 0x45, tos 0
                h[4] = bswap16(tl);                                 // total length, id 0
                h[5] = bswap16(ff) | 0x11400000u;                   // fragment field, ttl 64, 17
                h[6] = ck | ((sq & 0xFFFFu) << 16);
                h[7] = (sq >> 16) | ((dq & 0xFFFFu) << 16);
                h[8] = (dq >> 16) | ((ptq & 0xFFFFu) << 16);        // src port raw, :341
                h[9] = (ptq >> 16) | (bswap16(ul) << 16);           // dst port raw, :342, :344
                h[10] = 0u;                                         // UDP checksum 0, :343
                h[11] = 0u;
                // shift into the frame's 16-byte alignment: byte r of the header lands at
                // window byte (ffo & 15) + r
                const uint32_t sh = ffo & 15u, s3 = sh & 3u, d0 = sh >> 2;
                uint32_t *wq = win[w][lane];
#pragma unroll
                for (int t = 0; t < 16; ++t) wq[t] = 0u;
#pragma unroll
                for (int t = 0; t < 12; ++t) {
                    const uint32_t prev = t ? h[t - 1] : 0u;
                    const uint32_t gk = s3 ? ((h[t] << (8u * s3)) | (prev >> (32u - 8u * s3))) : h[t];
                    wq[d0 + t] = gk;
                }
                if (s3) wq[d0 + 12] = h[11] >> (32u - 8u * s3);
                nch = ((ffo & 15u) + hl + plen + 15u) >> 4;
            }
            uint32_t total;
            const uint32_t cs = excl_scan64(nch, &total);
            l_cs[w][lane] = cs;
            l_fo[w][lane] = ffo;
            l_len[w][lane] = plen | (hl == 34u ? 0x80000000u : 0u);
            l_po[w][lane] = ppo;
            wave_sync_tx();

            for (uint32_t k = lane + 64u * part; k < total; k += 64u * a.parts) {
                uint32_t q = 0;
#pragma unroll
                for (int sft = 32; sft >= 1; sft >>= 1)
                    if (l_cs[w][q + sft] <= k) q += sft;
                const uint32_t j = k - l_cs[w][q];
                const uint32_t fq = l_fo[w][q], lw = l_len[w][q], pq = l_po[w][q];
                const uint32_t Lq = lw & 0x7FFFFFFFu;
                const int hq = (lw >> 31) ? 34 : 42;
                const uint32_t abase = (fq & ~15u) + 16u * j;
                const int r0c = (int)(abase - fq);
                // header part
                uint32_t H[4] = {0u, 0u, 0u, 0u};
                if (j < 4) {
                    const uint4 hv = *reinterpret_cast<const uint4 *>(&win[w][q][4 * j]);
                    H[0] = hv.x; H[1] = hv.y; H[2] = hv.z; H[3] = hv.w;
                }
                // payload part: bytes at payload offset pq + r0c - hq + b
                uint32_t P[4] = {0u, 0u, 0u, 0u};
                if (r0c + 16 > hq) {
                    const int64_t src0 = (int64_t)pq + r0c - hq;
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
                    const uint32_t hm = win_mask(-r0c, hq - r0c, t);
                    const uint32_t pm = win_mask(hq - r0c, hq + (int)Lq - r0c, t);
                    o[t] = (H[t] & hm) | (P[t] & pm);
                    own[t] = hm | pm;
                    full = full && own[t] == 0xFFFFFFFFu;
                }
                uint8_t *dstp = a.frames + abase;
                if (full) {
                    *reinterpret_cast<uint4 *>(dstp) = make_uint4(o[0], o[1], o[2], o[3]);
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (own[t] == 0xFFFFFFFFu) {
                            *reinterpret_cast<uint32_t *>(dstp + 4 * t) = o[t];
                        } else if (own[t]) {
                            for (int b = 0; b < 4; ++b)
                                if ((own[t] >> (8 * b)) & 0xFFu) dstp[4 * t + b] = (uint8_t)(o[t] >> (8 * b));
                        }
                    }
                }
            }
            wave_sync_tx();
        }
    }
}

} // namespace udpdk
