// rx_kernels.hip — gfx950 RX datapath: parse + validate + checksums + port demux + lanes.
//
// Replaces, for a batch of N frames, N calls of reassemble() (udpdk_poller.c:316-413) from the
// burst loop (udpdk_poller.c:516-545) plus the per-socket rx_buffer appends and ring flushes
// (udpdk_poller.c:274-298). Three stages, all integer/byte work bound by HBM:
//
//   rx_classify  one workgroup per tile of T frames. Frames are read once, as 16-byte chunks
//                assigned to lanes so that a wave-instruction reads 1 KiB of consecutive bytes
//                whatever the frame sizes. The first 64 B window of every frame is staged in
//                LDS and parsed by the frame's lane; the RFC 1071 sums of the IPv4 header and
//                the whole UDP datagram are accumulated per frame in LDS. Demux walks the
//                flattened bind snapshot. Writes one verdict word per frame and the tile's
//                per-lane delivery histogram (lane-major: hist[lane][tile]).
//   rx_scan      exclusive scan of the lane-major histogram: hist[lane][tile] becomes the
//                position of the tile's first delivery in that lane; lane_off falls out as
//                hist[lane][0]. One launch when small, reduce/top/down-sweep otherwise.
//   rx_scatter   one wave per tile walks its frames in order and writes each delivery at its
//                stable position (wave multi-split by ballots, LDS running cursor per lane).
//
// Bytes per frame: frame_len (every byte is summed) + 6 (offset u32 + length u16) + 4 (verdict)
// in rx_classify; + 4 (verdict re-read) + 4 per delivery in rx_scatter.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

// ------------------------------------------------------------------------------------------
// wave helpers (wave64)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Exclusive prefix sum across the wave; *total = sum over all 64 lanes.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total)
{
    const uint32_t lane = lane_id();
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Bytes [a, e) of a 16-byte chunk as four dword masks (a, e clamped to [0, 16]).
__device__ __forceinline__ uint32_t dword_window(int a, int e, int i)
{
    int la = min(max(a - 4 * i, 0), 4);
    int le = min(max(e - 4 * i, 0), 4);
    uint32_t hm = le >= 4 ? 0xFFFFFFFFu : ((1u << (8 * le)) - 1u);
    uint32_t lm = la >= 4 ? 0xFFFFFFFFu : ((1u << (8 * la)) - 1u);
    return hm & ~lm;
}

// Sum of the 16-bit halves of the masked dwords: <= 8 * 0xFFFF per chunk.
__device__ __forceinline__ uint32_t masked_sum16(const uint32_t d[4], int a, int e)
{
    if (e <= a) return 0;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t v = d[i] & dword_window(a, e, i);
        s += (v & 0xFFFFu) + (v >> 16);
    }
    return s;
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// consecutive tiles land on one XCD so their lane-major histogram stores share L2 lines.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb)
{
    if (nb < 16) return b;
    const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                             0x00020000);
}

// ------------------------------------------------------------------------------------------
// rx_classify
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(RX_BLOCK)
rx_classify(RxArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);

    uint8_t  *hdr  = smem + w * 64 * HDR_STRIDE;
    uint32_t *arr  = reinterpret_cast<uint32_t *>(smem + HDR_BYTES) + w * WAVE_ARRAYS * 64;
    uint32_t *l_cs = arr, *l_off = arr + 64, *l_len = arr + 128, *l_ip = arr + 192,
             *l_udp = arr + 256;
    uint32_t *cnt  = reinterpret_cast<uint32_t *>(smem + CNT_OFF);
    uint32_t *hist = reinterpret_cast<uint32_t *>(smem + HIST_OFF);

    for (uint32_t s = tid; s < a.n_lanes; s += RX_BLOCK) hist[s] = 0;
    if (tid < UDPDK_N_COUNTERS) cnt[tid] = 0;
    __syncthreads();

    const __amdgpu_buffer_rsrc_t fr = make_rsrc(a.frames, a.rsrc_bytes);
    const uint32_t t0 = tile * a.tile_frames;
    const uint32_t t1 = min(a.n, t0 + a.tile_frames);
    const uint32_t steps = a.tile_frames / 64;

    for (uint32_t st = w; st < steps; st += RX_WAVES) {
        const uint32_t p = t0 + st * 64 + lane;
        const bool valid = p < t1;
        const uint32_t off = valid ? a.offset[p] : 0u;
        const uint32_t len = valid ? (uint32_t)a.length[p] : 0u;
        const bool bad_desc = valid && ((uint64_t)off + len > (uint64_t)a.frames_bytes);
        const uint32_t nch = (valid && !bad_desc && len) ? (((off & 15u) + len + 15u) >> 4) : 0u;
        uint32_t total;
        const uint32_t cs = wave_excl_scan(nch, &total);
        l_cs[lane] = cs;
        l_off[lane] = off;
        l_len[lane] = len;
        l_ip[lane] = 0;
        l_udp[lane] = 0;
        wave_sync();

        // ---- chunk sweep: lane k of the sweep reads the k-th 16-byte chunk of this step ----
        for (uint32_t k0 = 0; k0 < total; k0 += 64 * RX_UNROLL) {
            uint32_t d[RX_UNROLL][4];
            uint32_t q[RX_UNROLL], j[RX_UNROLL];
            int rel[RX_UNROLL];
#pragma unroll
            for (int u = 0; u < RX_UNROLL; ++u) {
                const uint32_t k = k0 + u * 64 + lane;
                // last frame whose first chunk index is <= k (frames with no chunk are skipped)
                uint32_t qq = 0;
#pragma unroll
                for (int sft = 32; sft >= 1; sft >>= 1)
                    if (l_cs[qq + sft] <= k) qq += sft;
                q[u] = qq;
                j[u] = k - l_cs[qq];
                const uint32_t fo = l_off[qq];
                const uint32_t base = (fo & ~15u) + 16u * j[u];
                rel[u] = (int)(base - fo);
                if (k < total) {
                    auto v = __builtin_amdgcn_raw_buffer_load_b128(fr, (int)base, 0, 0);
                    d[u][0] = v[0]; d[u][1] = v[1]; d[u][2] = v[2]; d[u][3] = v[3];
                } else {
                    d[u][0] = d[u][1] = d[u][2] = d[u][3] = 0u;
                }
            }
#pragma unroll
            for (int u = 0; u < RX_UNROLL; ++u) {
                const uint32_t k = k0 + u * 64 + lane;
                if (k >= total) continue;
                const uint32_t qq = q[u];
                if (j[u] < 4) {
                    uint32_t *hw = reinterpret_cast<uint32_t *>(hdr + qq * HDR_STRIDE + 16 * j[u]);
                    *reinterpret_cast<uint4 *>(hw) = make_uint4(d[u][0], d[u][1], d[u][2], d[u][3]);
                }
                const int r = rel[u];
                const int flen = (int)l_len[qq];
                const uint32_t ip = masked_sum16(d[u], 14 - r, 34 - r);
                const uint32_t ud = masked_sum16(d[u], 34 - r, flen - r);
                if (ip) atomicAdd(&l_ip[qq], ip);
                if (ud) atomicAdd(&l_udp[qq], ud);
            }
        }
        wave_sync();

        // ---- per-frame parse (lane = frame) from the staged 64-byte window ----
        uint32_t word = 0, verdict = UDPDK_V_BAD_DESC, fan = 0, first = 0;
        bool ip_bad = false, udp_ok = false, udp_bad = false, udp_none = false, len_bad = false,
             ihl_ne5 = false;
        if (valid && !bad_desc) {
            const uint32_t sh = off & 15u;
            const uint32_t *hw = reinterpret_cast<const uint32_t *>(hdr + lane * HDR_STRIDE +
                                                                   (sh & ~3u));
            uint32_t raw[12], h[11];
#pragma unroll
            for (int i = 0; i < 12; ++i) raw[i] = hw[i];
#pragma unroll
            for (int i = 0; i < 11; ++i) h[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh & 3u);
            // h[i] = frame bytes 4i .. 4i+3 (little-endian)
            uint32_t pt;
            if (a.ptype) pt = a.ptype[p];
            else pt = len >= 14 ? (((h[3] & 0xFFFFu) == 0x0008u) ? 0x211u : 0x1u) : 0u;
            if (!(pt & 0x10u)) {
                verdict = UDPDK_V_NOT_IPV4;               // udpdk_poller.c:334, :362-366
            } else if (len < 42) {
                verdict = UDPDK_V_TRUNC;
            } else {
                const uint32_t ipsum = l_ip[lane];
                const bool ip_ok = ipsum != 0u && (ipsum % 65535u) == 0u;
                ip_bad = !ip_ok;
                ihl_ne5 = ((h[3] >> 16) & 0x0Fu) != 5u;
                word |= (ip_ok ? 1u : 0u) << 4 | (ihl_ne5 ? 1u : 0u) << 8;
                const uint32_t frag = ((h[5] & 0xFFu) << 8) | ((h[5] >> 8) & 0xFFu);
                if ((frag & 0x2000u) || (frag & 0x1FFFu)) {
                    verdict = UDPDK_V_FRAG;               // udpdk_poller.c:338
                } else if ((h[5] >> 24) != 17u) {
                    verdict = UDPDK_V_NOT_UDP;            // udpdk_poller.c:368-371
                } else {
                    const uint32_t src = (h[6] >> 16) | (h[7] << 16);
                    const uint32_t dip = (h[7] >> 16) | (h[8] << 16);   // poller.c:373
                    const uint32_t dport = h[9] & 0xFFFFu;               // poller.c:372
                    const uint32_t ulen_raw = h[9] >> 16;
                    const uint32_t ulen = ((ulen_raw & 0xFFu) << 8) | (ulen_raw >> 8);
                    const uint32_t ucks = h[10] & 0xFFFFu;
                    len_bad = ulen < 8u || 34u + ulen > len;
                    uint32_t state;
                    if (ucks == 0u) {
                        state = UDPDK_UDP_CSUM_NONE;
                    } else if (len_bad) {
                        state = UDPDK_UDP_CSUM_BAD;
                    } else {
                        uint32_t s = l_udp[lane] % 65535u;
                        if (34u + ulen < len) {            // Ethernet padding after the datagram
                            uint32_t pad = 0;
                            for (uint32_t b = off + 34u + ulen; b < off + len; ++b)
                                pad += (uint32_t)a.frames[b] << (8u * (b & 1u));
                            s = (s + 65535u - pad % 65535u) % 65535u;
                        }
                        if (off & 1u) s = (s * 256u) % 65535u;           // odd start: swap bytes
                        const uint32_t pseudo = (src & 0xFFFFu) + (src >> 16) + (dip & 0xFFFFu) +
                                                (dip >> 16) + 0x1100u + ulen_raw;
                        state = ((s + pseudo) % 65535u) == 0u ? UDPDK_UDP_CSUM_OK
                                                             : UDPDK_UDP_CSUM_BAD;
                    }
                    udp_ok = state == UDPDK_UDP_CSUM_OK;
                    udp_bad = state == UDPDK_UDP_CSUM_BAD;
                    udp_none = state == UDPDK_UDP_CSUM_NONE;
                    word |= state << 5 | (len_bad ? 1u : 0u) << 7;

                    // ---- demux: btable_get_bindings + list walk, udpdk_poller.c:376-405 ----
                    const uint32_t e = a.port_tab[dport];
                    const uint32_t nb = e & 0xFFFu;
                    if (nb == 0u) {
                        verdict = UDPDK_V_NO_BIND;
                    } else {
                        const uint32_t b0 = e >> 12;
                        for (uint32_t i = 0; i < nb; ++i) {
                            const uint2 b = a.binds[b0 + i];
                            if (dip == b.x || b.x == 0u) {                // poller.c:391
                                const uint32_t sock = b.y & 0x7FFFFFFFu;
                                atomicAdd(&hist[sock & a.lane_mask], 1u);   // poller.c:393
                                if (fan == 0) first = sock;
                                ++fan;
                                if (!(b.y >> 31)) break;                 // poller.c:396-403
                            }
                        }
                        verdict = fan ? UDPDK_V_DELIVERED : UDPDK_V_NO_MATCH;
                    }
                }
            }
        }
        word |= verdict | (min(fan, 127u) << 9) | ((first & 0xFFFFu) << 16);
        if (valid) a.meta[p] = word;

        // ---- per-tile counters via ballots (no per-frame logging, cf. poller.c:363-410) ----
        uint32_t cv[UDPDK_N_COUNTERS];
#pragma unroll
        for (int v = 0; v < UDPDK_N_VERDICTS; ++v)
            cv[v] = (uint32_t)__popcll(__ballot(valid && verdict == (uint32_t)v));
        cv[UDPDK_C_DELIVERIES] = wave_sum(valid ? fan : 0u);
        cv[UDPDK_C_IP_BAD] = (uint32_t)__popcll(__ballot(valid && ip_bad));
        cv[UDPDK_C_UDP_OK] = (uint32_t)__popcll(__ballot(valid && udp_ok));
        cv[UDPDK_C_UDP_BAD] = (uint32_t)__popcll(__ballot(valid && udp_bad));
        cv[UDPDK_C_UDP_NONE] = (uint32_t)__popcll(__ballot(valid && udp_none));
        cv[UDPDK_C_LEN_BAD] = (uint32_t)__popcll(__ballot(valid && len_bad));
        cv[UDPDK_C_IHL_NE5] = (uint32_t)__popcll(__ballot(valid && ihl_ne5));
        cv[UDPDK_C_BYTES] = wave_sum(valid && !bad_desc ? len : 0u);
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < UDPDK_N_COUNTERS; ++c)
                if (cv[c]) atomicAdd(&cnt[c], cv[c]);
        }
        wave_sync();
    }
    __syncthreads();
    for (uint32_t s = tid; s < a.n_lanes; s += RX_BLOCK) a.hist[(size_t)s * a.n_tiles + tile] = hist[s];
    if (tid < UDPDK_N_COUNTERS) a.tile_cnt[(size_t)tile * UDPDK_N_COUNTERS + tid] = cnt[tid];
}

// ------------------------------------------------------------------------------------------
// rx_scan: exclusive scan of hist[E] (lane-major) in place; lane_off; counter reduction
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds16, uint32_t *total)
{
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t wt;
    const uint32_t x = wave_excl_scan(v, &wt);
    if (lane == 0) lds16[w] = wt;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t t = lds16[i];
        if (i < w) pre += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return pre + x;
}

// Counter reduction over tiles: counters[c] = sum_t tile_cnt[t][c] (64-bit).
__device__ void reduce_counters(const uint32_t *tile_cnt, uint32_t n_tiles,
                                unsigned long long *counters, unsigned long long *lds)
{
    const uint32_t tid = threadIdx.x;
    if (tid < UDPDK_N_COUNTERS) lds[tid] = 0;
    __syncthreads();
    const uint32_t c = tid % UDPDK_N_COUNTERS;
    unsigned long long s = 0;
    for (uint32_t t = tid / UDPDK_N_COUNTERS; t < n_tiles; t += blockDim.x / UDPDK_N_COUNTERS)
        s += tile_cnt[(size_t)t * UDPDK_N_COUNTERS + c];
    atomicAdd(&lds[c], s);
    __syncthreads();
    if (tid < UDPDK_N_COUNTERS) counters[tid] = lds[tid];
}

// Small case: one workgroup of SCAN_BLOCK threads, E <= SCAN_BLOCK * SCAN_SMALL_PER.
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_small(ScanArgs a)
{
    __shared__ uint32_t lds16[SCAN_BLOCK / 64];
    __shared__ unsigned long long lcnt[UDPDK_N_COUNTERS];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (a.n_elems + SCAN_BLOCK - 1) / SCAN_BLOCK;
    const uint32_t i0 = tid * per, i1 = min(a.n_elems, i0 + per);
    uint32_t s = 0;
    for (uint32_t i = i0; i < i1; ++i) s += a.hist[i];
    uint32_t total;
    uint32_t run = block_excl_scan(s, lds16, &total);
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t v = a.hist[i];
        a.hist[i] = run;
        if (i % a.n_tiles == 0) a.lane_off[i / a.n_tiles] = run;
        run += v;
    }
    if (tid == 0) { a.lane_off[a.n_lanes] = total; *a.total = total; }
    reduce_counters(a.tile_cnt, a.n_tiles, a.counters, lcnt);
}

// Large case, pass 1: partial[b] = sum of chunk b (SCAN_CHUNK elements).
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_reduce(ScanArgs a)
{
    __shared__ uint32_t lds16[SCAN_BLOCK / 64];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t base = b * SCAN_CHUNK;
    uint32_t s = 0;
#pragma unroll 4
    for (uint32_t i = tid; i < SCAN_CHUNK; i += SCAN_BLOCK)
        if (base + i < a.n_elems) s += a.hist[base + i];
    s = wave_sum(s);
    if (lane_id() == 0) lds16[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (uint32_t i = 0; i < SCAN_BLOCK / 64; ++i) t += lds16[i];
        a.partial[b] = t;
    }
}

// Large case, pass 2: exclusive scan of partial[] (one workgroup) + counters.
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_top(ScanArgs a, uint32_t n_part)
{
    __shared__ uint32_t lds16[SCAN_BLOCK / 64];
    __shared__ unsigned long long lcnt[UDPDK_N_COUNTERS];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (n_part + SCAN_BLOCK - 1) / SCAN_BLOCK;
    const uint32_t i0 = tid * per, i1 = min(n_part, i0 + per);
    uint32_t s = 0;
    for (uint32_t i = i0; i < i1; ++i) s += a.partial[i];
    uint32_t total;
    uint32_t run = block_excl_scan(s, lds16, &total);
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t v = a.partial[i];
        a.partial[i] = run;
        run += v;
    }
    if (tid == 0) { a.lane_off[a.n_lanes] = total; *a.total = total; }
    reduce_counters(a.tile_cnt, a.n_tiles, a.counters, lcnt);
}

// Large case, pass 3: rescan each chunk from its partial offset; write lane_off entries.
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_down(ScanArgs a)
{
    __shared__ uint32_t lds16[SCAN_BLOCK / 64];
    constexpr uint32_t PER = SCAN_CHUNK / SCAN_BLOCK;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t i0 = b * SCAN_CHUNK + tid * PER;
    uint32_t v[PER];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
        v[k] = (i0 + k < a.n_elems) ? a.hist[i0 + k] : 0u;
        s += v[k];
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, lds16, &total) + a.partial[b];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
        const uint32_t i = i0 + k;
        if (i < a.n_elems) {
            a.hist[i] = run;
            if (i % a.n_tiles == 0) a.lane_off[i / a.n_tiles] = run;
        }
        run += v[k];
    }
}

// ------------------------------------------------------------------------------------------
// rx_scatter: stable per-lane compaction, one wave per tile
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_cursor(uint32_t *cur, const ScatterArgs &a, uint32_t key,
                                                uint32_t tile)
{
    uint32_t c = cur[key];
    if (c == 0xFFFFFFFFu) c = a.base[(size_t)key * a.n_tiles + tile];
    return c;
}

__global__ void __launch_bounds__(64)
rx_scatter(ScatterArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *cur = reinterpret_cast<uint32_t *>(smem);   // running position per lane
    const uint32_t lane = lane_id();
    const uint32_t tile = blockIdx.x;
    for (uint32_t s = lane; s < a.n_lanes; s += 64) cur[s] = 0xFFFFFFFFu;
    wave_sync();
    const uint32_t t0 = tile * a.tile_frames;
    const uint32_t t1 = min(a.n, t0 + a.tile_frames);
    const uint64_t lt_mask = (1ull << lane) - 1ull;

    for (uint32_t f0 = t0; f0 < t1; f0 += 64) {
        const uint32_t p = f0 + lane;
        const bool valid = p < t1;
        const uint32_t m = valid ? a.meta[p] : 0u;
        const bool deliver = valid && UDPDK_META_VERDICT(m) == UDPDK_V_DELIVERED;
        const uint32_t fan = UDPDK_META_FANOUT(m);
        const uint64_t multi = __ballot(deliver && fan > 1u);
        if (multi == 0ull) {
            // fast path: one delivery per frame. Wave multi-split on the lane key.
            const uint32_t key = UDPDK_META_SOCKFD(m) & a.lane_mask;
            uint64_t peers = __ballot(deliver);
            for (uint32_t bit = 0; bit < a.key_bits; ++bit) {
                const bool kb = (key >> bit) & 1u;
                const uint64_t bal = __ballot(kb);
                peers &= kb ? bal : ~bal;
            }
            const uint32_t leader = deliver ? (uint32_t)__ffsll((long long)peers) - 1u : 64u;
            uint32_t c = 0;
            if (deliver && lane == leader) {
                c = lane_cursor(cur, a, key, tile);
                cur[key] = c + (uint32_t)__popcll(peers);
            }
            c = __shfl(c, deliver ? (int)leader : 0, 64);
            const uint32_t pos = c + (uint32_t)__popcll(peers & lt_mask);
            if (deliver && pos < a.lane_cap) a.lane_pkt[pos] = p;
        } else {
            // fan-out path (SO_REUSEADDR/SO_REUSEPORT clones, poller.c:396-399): deliveries in
            // frame order, then list order, re-derived from the frame header. Serial in lane 0.
            if (lane == 0) {
                for (uint32_t i = 0; i < 64 && f0 + i < t1; ++i) {
                    const uint32_t mi = a.meta[f0 + i];
                    if (UDPDK_META_VERDICT(mi) != UDPDK_V_DELIVERED) continue;
                    const uint32_t fp = f0 + i;
                    const uint8_t *f = a.frames + a.offset[fp];
                    const uint32_t dport = (uint32_t)f[36] | ((uint32_t)f[37] << 8);
                    const uint32_t dip = (uint32_t)f[30] | ((uint32_t)f[31] << 8) |
                                         ((uint32_t)f[32] << 16) | ((uint32_t)f[33] << 24);
                    const uint32_t e = a.port_tab[dport];
                    const uint32_t nb = e & 0xFFFu, b0 = e >> 12;
                    for (uint32_t k = 0; k < nb; ++k) {
                        const uint2 b = a.binds[b0 + k];
                        if (dip == b.x || b.x == 0u) {
                            const uint32_t key = (b.y & 0x7FFFFFFFu) & a.lane_mask;
                            const uint32_t c = lane_cursor(cur, a, key, tile);
                            cur[key] = c + 1u;
                            if (c < a.lane_cap) a.lane_pkt[c] = fp;
                            if (!(b.y >> 31)) break;
                        }
                    }
                }
            }
        }
        wave_sync();
    }
}

} // namespace udpdk
