// rx_gather.hip — gfx950 payload delivery: the batch form of udpdk_recvfrom
// (udpdk_syscall.c:401-488) over a range of lane entries produced by the RX pipeline.
//
// Lane entry k (frame i = lane_pkt[first + k]): payload = frame bytes
// [42, 42 + min(data_len - 42, dgram_len - 8)) (Ethernet padding trimmed, :459-466), truncated
// to slot_bytes (recvfrom's len, :467-472), copied to payload + k * slot_bytes (packed slots, as
// the poll uses them: payload + slot_off[k], slot_off[k + 1] - slot_off[k] bytes); len[k] = bytes
// copied (recvfrom's return, :487); src_ip[k] / src_port[k] = ip_hdr->src_addr /
// udp_hdr->src_port, raw (:446-447).
//
// One lane per entry: one byte-aligned 16-byte load of frame bytes [26, 42) gives the source
// address, source port and dgram_len. Payloads move in 16-byte pieces stored as aligned 16-byte
// slot writes (the slot tail past len is scratch): a wave whose payloads are all short copies
// one per lane; otherwise the wave copies its entries two at a time with every wave-load a
// contiguous KiB of one payload (coalesced reads and writes). HBM-bound:
// bytes per entry = payload read + payload written + 16 (header) + 4 (lane entry) + 6
// (descriptor) + 10 (len, src_ip, src_port).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

__global__ void __launch_bounds__(GATHER_BLOCK) rx_gather(GatherArgs a)
{
    const __amdgpu_buffer_rsrc_t fr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.frames), (short)0, (int)a.rsrc_bytes, 0x00020000);
    const uint32_t lane = __lane_id();
    for (uint32_t k = blockIdx.x * GATHER_BLOCK + threadIdx.x; k - threadIdx.x < a.count;
         k += gridDim.x * GATHER_BLOCK) {
        const bool valid = k < a.count;
        const uint32_t i = valid ? min(a.lane_pkt[a.first + k], a.n - 1u) : 0u;
        const uint32_t o = a.offset[i];
        const uint32_t len = a.length[i];
        // Frame bytes [26, 42) (source address and port, dgram_len) and, for a short frame, its
        // first 64 payload bytes [42, 106), as up to six dword-aligned 16-byte loads from the
        // dword at or below offset + 26, funnelled by offset & 3 (byte-aligned 16-byte loads run
        // the vector memory path ~25 % slower, tools/probe/align_probe.hip). The frame length
        // bounds the payload part; pieces past it are addressed out of range (no memory access).
        const uint32_t fseg = len >= 42u ? len - 42u : 0u;
        const uint32_t X = o + 26u, sh = X & 3u;
        const uint32_t need = 16u + (valid && fseg <= 64u ? fseg : 0u) + sh;
        uint32_t D[24];
#pragma unroll
        for (uint32_t u = 0; u < 6; ++u) {
            const uint32_t off = 16u * u < need ? (X & ~3u) + 16u * u : 0x80000000u;
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(fr, (int)off, 0, 0);
            D[4 * u] = x[0]; D[4 * u + 1] = x[1]; D[4 * u + 2] = x[2]; D[4 * u + 3] = x[3];
        }
        uint32_t W[20];                                          // W[m] = frame bytes 26 + 4m ..
#pragma unroll
        for (int m = 0; m < 20; ++m) W[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], sh);
        const uint32_t h[4] = {W[0], W[1], W[2], W[3]};
        uint4 v0[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) v0[u] = make_uint4(W[4 + 4 * u], W[5 + 4 * u], W[6 + 4 * u], W[7 + 4 * u]);
        const uint32_t dlr = h[3] & 0xFFFFu;                                           // dgram_len, BE
        const uint32_t dl = ((dlr & 0xFFu) << 8) | (dlr >> 8);
        const uint32_t pl = (dl - 8u) & 0xFFFFu;                 // uint16_t dgram_payl_len (:436)
        const uint32_t seg = len >= 42u ? len - 42u : 0u;        // data_len - offset_payload (:458)
        const uint32_t so32 = valid && a.slot_off ? a.slot_off[k] : 0u;
        const uint64_t so = !valid ? 0ull : a.slot_off ? (uint64_t)so32 : (uint64_t)k * a.slot_bytes;
        const uint32_t cap = !valid ? 0u : a.slot_off ? a.slot_off[k + 1] - so32 : a.slot_bytes;
        const uint32_t n = valid ? min(min(seg, pl), cap) : 0u;
        if (valid) {
            a.len_out[k] = n;
            a.src_ip[k] = h[0];
            a.src_port[k] = (uint16_t)(h[2] & 0xFFFFu);
        }
        const uint32_t kw = k - lane;                            // the wave's first entry
        if (!__ballot(n > 128u)) {
            // short payloads: each lane copies its own, 16-byte pieces, four loads in flight
            uint8_t *dst = a.payload + so;
            for (uint32_t c = 0; c < n; c += 64u) {
                uint4 v[4];
                if (c == 0u && fseg <= 64u) {
#pragma unroll
                    for (uint32_t u = 0; u < 4; ++u) v[u] = v0[u];
                } else {
#pragma unroll
                    for (uint32_t u = 0; u < 4; ++u) {
                        const auto x = __builtin_amdgcn_raw_buffer_load_b128(fr, (int)(o + 42u + c + 16u * u), 0, 0);
                        v[u] = make_uint4(x[0], x[1], x[2], x[3]);
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < 4; ++u)
                    if (c + 16u * u < n) *reinterpret_cast<uint4 *>(dst + c + 16u * u) = v[u];
            }
        } else {
            // long payloads: the wave copies its entries one pair at a time, every wave-load a
            // contiguous KiB of one payload (lane i: bytes 16 i .. 16 i + 15 of each KiB)
            for (uint32_t j = 0; j < 64u; j += 2u) {
                uint32_t nj[2], oj[2];
                uint64_t dj[2];
#pragma unroll
                for (uint32_t u = 0; u < 2; ++u) {
                    nj[u] = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)(j + u));
                    oj[u] = (uint32_t)__builtin_amdgcn_readlane((int)o, (int)(j + u));
                    dj[u] = a.slot_off ? (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)so32, (int)(j + u))
                                       : (uint64_t)(kw + j + u) * a.slot_bytes;
                }
                const uint32_t m = max(nj[0], nj[1]);
                // Sources are read from the dword-aligned offset at or below each piece (byte-
                // aligned 16-byte loads run the vector memory path ~15-25 % slower,
                // tools/probe/align_probe.hip) and funnelled by the payload's offset & 3 with the
                // next lane's first dword; lane 63 loads its own next dword. Shift 0: identity.
                uint32_t sh[2];
#pragma unroll
                for (uint32_t u = 0; u < 2; ++u) sh[u] = (oj[u] + 42u) & 3u;
                for (uint32_t c = 0; c < m; c += 2048u) {
                    uint4 v[2][2];
                    uint32_t e[2][2];
#pragma unroll
                    for (uint32_t u = 0; u < 2; ++u)
#pragma unroll
                        for (uint32_t h2 = 0; h2 < 2; ++h2) {
                            const uint32_t b = c + 1024u * h2 + 16u * lane;
                            const uint32_t sa = (oj[u] + 42u + b) & ~3u;
                            // (a piece just past the payload still loads when the piece before
                            // it needs its first dword)
                            const auto x = __builtin_amdgcn_raw_buffer_load_b128(
                                fr, (int)(b < nj[u] + (sh[u] != 0u ? 16u : 0u) ? sa : 0x80000000u), 0, 0);
                            v[u][h2] = make_uint4(x[0], x[1], x[2], x[3]);
                            e[u][h2] = __builtin_amdgcn_raw_buffer_load_b32(
                                fr, (int)(lane == 63u && sh[u] != 0u && b < nj[u] ? sa + 16u : 0x80000000u), 0, 0);
                        }
#pragma unroll
                    for (uint32_t u = 0; u < 2; ++u)
#pragma unroll
                        for (uint32_t h2 = 0; h2 < 2; ++h2) {
                            const uint32_t b = c + 1024u * h2 + 16u * lane;
                            const uint4 x = v[u][h2];
                            const uint32_t nx = __shfl_down(x.x, 1, 64);
                            const uint32_t hi = lane == 63u ? e[u][h2] : nx;
                            const uint4 y = make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, sh[u]),
                                                       __builtin_amdgcn_alignbyte(x.z, x.y, sh[u]),
                                                       __builtin_amdgcn_alignbyte(x.w, x.z, sh[u]),
                                                       __builtin_amdgcn_alignbyte(hi, x.w, sh[u]));
                            if (b < nj[u])
                                *reinterpret_cast<uint4 *>(a.payload + dj[u] + b) = y;
                        }
                }
            }
        }
    }
}

} // namespace udpdk
