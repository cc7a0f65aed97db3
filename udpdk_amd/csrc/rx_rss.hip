// rx_rss.hip — gfx950 receive-side scaling: the per-frame Toeplitz hash a
// NIC computes for ETH_MQ_RX_RSS (the mode udpdk_init.c:137 asks for, with one RX ring and a
// "TODO add RSS support" at :112) and the redirection-table lookup that picks the frame's RX
// queue, then stable per-queue lists: queue q's frames in arrival order, the input for one
// GPU (or poller) per queue.
//
// Hash input (rss_hf = IPv4 | non-fragmented IPv4 UDP): frame bytes [26, 38) = source address,
// destination address, source port, destination port for an unfragmented UDP frame, bytes
// [26, 34) for other IPv4 frames (fragments, other protocols), nothing (hash 0) for frames the
// IPv4 gate rejects (the same ptype rule as rx_classify, fixed offsets as the reference parses).
// Queue = reta[hash & (reta_size - 1)].
//
// Kernels: rss_hash (one workgroup per 1024-frame tile: a 12 x 256 table of key windows, built
// once on the host and staged into LDS, turns the bit-serial Toeplitz product into 12 lookups
// per frame; hash and queue per frame; the
// tile's queue histogram by wave multi-split), the tile-major scan shared with rx (rx_scan_*),
// rss_scatter (per tile, each wave's contiguous quarter placed after the earlier quarters).
// Bytes per frame: 26 header bytes read (one or two 32 B sectors) + 8 descriptor + 4 hash + 1
// queue id written, then 1 + 4 (queue id read, list entry written) in the scatter.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

namespace {

// Orders a wave's LDS accesses across lanes (its DS instructions execute in order).
__device__ __forceinline__ void wsync()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Lanes of the wave holding the same key (key < 2^bits), from one ballot per key bit.
// Inclusive wave64 prefix sum on the DPP network (every lane active): six VALU ops where the
// __shfl_up chain made six ds_bpermute round trips
__device__ __forceinline__ uint32_t rss_scan_dpp(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

__device__ __forceinline__ unsigned long long peers_of(uint32_t key, uint32_t bits, bool active)
{
    unsigned long long peers = __ballot(active);
    for (uint32_t b = 0; b < bits; ++b) {
        const bool kb = (key >> b) & 1u;
        const unsigned long long bal = __ballot(kb);
        peers &= kb ? bal : ~bal;
    }
    return peers;
}

// The fused form of rss_base, run by the last rss_hash workgroup (RssArgs::fuse): the same
// exclusive scan of the queue-major histogram as one array, in passes of 32 entries per thread
// (8 x 16-byte sc1 loads, written through by the other workgroups), a running carry between
// passes; queue_off[q] = the scanned value at q * T, queue_off[Q] = total.
__device__ void rss_scan_last(uint32_t *hist, uint32_t n, uint32_t T, uint32_t *queue_off, uint32_t *total)
{
    __shared__ uint32_t wsum[RSS_BLOCK / 64];
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(hist, (short)0, (int)(4u * n), 0x00020000);
    constexpr uint32_t PER = 32;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += PER * RSS_BLOCK) {
        const uint32_t k0 = b0 + PER * tid;
        uint32_t v[PER];
#pragma unroll
        for (uint32_t i = 0; i < PER / 4u; ++i) {
            const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(hr, (int)(4u * k0 + 16u * i), 0, 16));
            v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
        }
        uint32_t sum = 0;
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) sum += v[i];
        uint32_t incl = sum;
        incl = rss_scan_dpp(incl);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t run = carry + incl - sum, grand = 0;
#pragma unroll
        for (uint32_t i = 0; i < RSS_BLOCK / 64; ++i) {
            run += i < w ? wsum[i] : 0u;
            grand += wsum[i];
        }
        uint32_t next = k0 < n ? ((k0 + T - 1u) / T) * T : 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i) {
            if (k0 + i == next) {
                queue_off[next / T] = run;
                next += T;
            }
            const uint32_t x = v[i];
            v[i] = run;
            run += x;
        }
#pragma unroll
        for (uint32_t i = 0; i < PER / 4u; ++i)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3])),
                hr, (int)(4u * k0 + 16u * i), 0, 0);
        carry += grand;
        __syncthreads();                                   // wsum read by every wave
    }
    if (tid == 0) {
        queue_off[n / T] = carry;
        *total = carry;
    }
}

} // namespace

__global__ void __launch_bounds__(RSS_BLOCK) rss_hash(RssArgs a)
{
    __shared__ __attribute__((aligned(16))) uint32_t tab[12][256];
    __shared__ uint16_t reta[RSS_RETA_MAX];
    __shared__ uint32_t hist[RSS_MAX_QUEUES];
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.frames), (short)0, (int)a.rsrc_bytes, 0x00020000);
    const uint32_t tile = blockIdx.x;
    const uint32_t t0 = tile * RSS_TILE, t1 = min(a.n, t0 + RSS_TILE);
    constexpr uint32_t STEPS = RSS_TILE / RSS_BLOCK;
    // all of the thread's frames' loads first (descriptors, then header words), then the work
    uint32_t o[STEPS], len[STEPS];
    uint4 h0[STEPS], h1[STEPS];        // frame bytes [12, 38) from the dword at or below offset + 12
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const uint32_t i = t0 + s * RSS_BLOCK + (tid & ~63u) + lane;
        o[s] = i < t1 ? a.offset[i] : 0u;
        len[s] = i < t1 ? a.length[i] : 0u;
    }
    // the key-window table (udpdk_gpu_rss_config builds it: tab[p][v] = XOR of the key windows
    // key bits [8p + j, 8p + j + 32) over the set bits j, MSB first, of byte value v at input
    // position p): its 16-byte loads go out while the descriptors are in flight, the LDS stores
    // after the header loads are issued
    constexpr uint32_t KV = 12u * 256u / 4u / RSS_BLOCK;
    uint4 kv[KV];
    const uint4 *ksrc = reinterpret_cast<const uint4 *>(a.ktab);
#pragma unroll
    for (uint32_t e = 0; e < KV; ++e) kv[e] = ksrc[e * RSS_BLOCK + tid];
    // two dword-aligned 16-byte loads per frame instead of five 4-byte loads, three of them at
    // byte offsets (26, 30, 34: byte-aligned loads run the vector memory path ~25 % slower,
    // tools/probe/align_probe.hip); the words are funnelled by offset & 3 below
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const bool ok = (uint64_t)o[s] + len[s] <= a.frames_bytes && len[s] >= 34u;
        const uint32_t A = ok ? (o[s] + 12u) & ~3u : 0u;
        h0[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(fr, (int)A, 0, 0));
        h1[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(fr, (int)(A + 16u), 0, 0));
    }
    {
        uint4 *dst = reinterpret_cast<uint4 *>(&tab[0][0]);
#pragma unroll
        for (uint32_t e = 0; e < KV; ++e) dst[e * RSS_BLOCK + tid] = kv[e];
    }
    for (uint32_t e = tid; e < a.reta_size; e += RSS_BLOCK) reta[e] = a.reta[e];
    for (uint32_t q = tid; q < a.n_queues; q += RSS_BLOCK) hist[q] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const uint32_t i = t0 + s * RSS_BLOCK + (tid & ~63u) + lane;
        const bool in = i < t1;
        uint32_t hash = 0;
        const bool ok = in && (uint64_t)o[s] + len[s] <= a.frames_bytes && len[s] >= 34u;
        // frame-relative words g[i] = frame bytes [12 + 4 i, 16 + 4 i)
        const uint32_t D[8] = {h0[s].x, h0[s].y, h0[s].z, h0[s].w, h1[s].x, h1[s].y, h1[s].z, h1[s].w};
        const uint32_t sh = o[s] & 3u;
        uint32_t g[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) g[k] = __builtin_amdgcn_alignbyte(D[k + 1], D[k], sh);
        const uint32_t w12 = g[0], w20 = g[2];
        const uint32_t src = (g[3] >> 16) | (g[4] << 16), dst = (g[4] >> 16) | (g[5] << 16);
        const uint32_t ports = (g[5] >> 16) | (g[6] << 16);       // used only when len >= 38
        const uint32_t pt = ok ? (a.ptype ? a.ptype[i] : ((w12 & 0xFFFFu) == 0x0008u ? 0x211u : 0x1u)) : 0u;
        if (ok && (pt & 0x10u)) {
            const uint32_t ff = ((w20 & 0xFFu) << 8) | ((w20 >> 8) & 0xFFu);
            const bool frag = (ff & 0x3FFFu) != 0u;
            const bool udp4 = !frag && ((w20 >> 24) & 0xFFu) == 17u && len[s] >= 38u && (a.hash_types & 2u);
            if (udp4 || (a.hash_types & 1u)) {
                const uint32_t sa = src, da = dst, pp = ports;
                hash = tab[0][sa & 255u] ^ tab[1][(sa >> 8) & 255u] ^ tab[2][(sa >> 16) & 255u] ^
                       tab[3][sa >> 24] ^ tab[4][da & 255u] ^ tab[5][(da >> 8) & 255u] ^
                       tab[6][(da >> 16) & 255u] ^ tab[7][da >> 24];
                if (udp4)
                    hash ^= tab[8][pp & 255u] ^ tab[9][(pp >> 8) & 255u] ^ tab[10][(pp >> 16) & 255u] ^
                            tab[11][pp >> 24];
            }
        }
        const uint32_t q = reta[hash & (a.reta_size - 1u)];
        if (in) {
            a.hash[i] = hash;
            a.qid[i] = (uint8_t)q;
        }
        const unsigned long long peers = peers_of(q, a.q_bits, in);
        if (in && lane == (uint32_t)__ffsll((long long)peers) - 1u)
            atomicAdd(&hist[q], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    if (!a.fuse) {
        for (uint32_t q = tid; q < a.n_queues; q += RSS_BLOCK)
            a.hist[a.qmajor ? (size_t)q * a.n_tiles + tile : (size_t)tile * a.n_queues + q] = hist[q];
        return;
    }
    // fused queue bases (queue-major histogram): the row written through and drained, then the
    // launch's last workgroup scans the histogram (rss_base's work, no third launch)
    __shared__ uint32_t last;
    for (uint32_t q = tid; q < a.n_queues; q += RSS_BLOCK)
        __hip_atomic_store(&a.hist[(size_t)q * a.n_tiles + tile], hist[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        unsigned long long fin;
        last = fanin_arrive(a.fuse, tile, a.n_tiles, 0ull, &fin) ? 1u : 0u;
    }
    __syncthreads();
    if (!last) return;
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    rss_scan_last(a.hist, a.n_queues * a.n_tiles, a.n_tiles, a.queue_off, a.total);
}

// The scan between rss_hash and rss_scatter for up to RSS_BASE_MAX histogram entries, in one
// workgroup: rss_hash wrote the histogram queue-major ([n_queues][T]), so an exclusive scan of it
// as one array turns entry (q, t) into queue q's list start plus the earlier tiles' counts for q,
// and queue_off[q] is the value at q * T. Thread tid owns entries [32 tid, 32 tid + 32) (eight
// 16-byte loads, all in flight at once), sums them serially, and one wave scan plus one scan of
// the 16 wave sums gives its start. (Row-per-wave ownership with a wave scan per row measured
// 13-16 us: 32 dependent shuffle chains per wave; this form has one.)
__global__ void __launch_bounds__(1024)
rss_base(uint32_t *hist, uint32_t n, uint32_t T, uint32_t *queue_off, uint32_t *total)
{
    constexpr uint32_t PER = RSS_BASE_MAX / 1024u;
    __shared__ uint32_t wsum[16];
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    // range-checked per dword: entries past n read as 0 and are never written
    const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(hist, (short)0, (int)(4u * n), 0x00020000);
    const uint32_t k0 = PER * tid;
    uint32_t v[PER];
#pragma unroll
    for (uint32_t i = 0; i < PER / 4u; ++i) {
        const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(hr, (int)(4u * k0 + 16u * i), 0, 0));
        v[4 * i] = q.x; v[4 * i + 1] = q.y; v[4 * i + 2] = q.z; v[4 * i + 3] = q.w;
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) sum += v[i];
    uint32_t incl = sum;
    incl = rss_scan_dpp(incl);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum, grand = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        run += i < w ? wsum[i] : 0u;
        grand += wsum[i];
    }
    // queue starts: the multiples of T inside this thread's range
    uint32_t next = k0 < n ? ((k0 + T - 1u) / T) * T : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
        if (k0 + i == next) {
            queue_off[next / T] = run;
            next += T;
        }
        const uint32_t x = v[i];
        v[i] = run;
        run += x;
    }
#pragma unroll
    for (uint32_t i = 0; i < PER / 4u; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3])),
            hr, (int)(4u * k0 + 16u * i), 0, 0);
    if (tid == 0) {
        queue_off[n / T] = grand;
        *total = grand;
    }
}

// Per tile: wave w owns frames [t0 + 256 w, t0 + 256 w + 256); its base for queue q is the
// tile's scanned start for q plus the earlier waves' counts.
__global__ void __launch_bounds__(RSS_BLOCK) rss_scatter(RssArgs a)
{
    __shared__ uint32_t cnt[RSS_BLOCK / 64][RSS_MAX_QUEUES], run[RSS_BLOCK / 64][RSS_MAX_QUEUES];
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    const uint32_t t0 = blockIdx.x * RSS_TILE, t1 = min(a.n, t0 + RSS_TILE);
    const uint32_t wb = t0 + w * (RSS_TILE / (RSS_BLOCK / 64));
    constexpr uint32_t STEPS = RSS_TILE / RSS_BLOCK;
    for (uint32_t q = lane; q < a.n_queues; q += 64) cnt[w][q] = 0;
    uint32_t qv[STEPS];
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const uint32_t i = wb + 64u * s + lane;
        qv[s] = i < t1 ? a.qid[i] : 0u;
    }
    wsync();
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const uint32_t i = wb + 64u * s + lane;
        const unsigned long long peers = peers_of(qv[s], a.q_bits, i < t1);
        if (i < t1 && lane == (uint32_t)__ffsll((long long)peers) - 1u) cnt[w][qv[s]] += (uint32_t)__popcll(peers);
        wsync();
    }
    __syncthreads();
    // running position per queue for this wave (row w of run[] is wave w's alone)
    for (uint32_t q = lane; q < a.n_queues; q += 64) {
        uint32_t b = a.hist[a.qmajor ? (size_t)q * a.n_tiles + blockIdx.x : (size_t)blockIdx.x * a.n_queues + q];
        for (uint32_t v = 0; v < w; ++v) b += cnt[v][q];
        run[w][q] = b;
    }
    wsync();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t s = 0; s < STEPS; ++s) {
        const uint32_t i = wb + 64u * s + lane;
        const bool in = i < t1;
        const uint32_t q = qv[s];
        const unsigned long long peers = peers_of(q, a.q_bits, in);
        const uint32_t base = in ? run[w][q] : 0u;
        wsync();
        if (in) {
            const uint32_t pos = base + (uint32_t)__popcll(peers & lt);
            a.queue_pkt[pos] = i;
            if (lane == (uint32_t)__ffsll((long long)peers) - 1u) run[w][q] = base + (uint32_t)__popcll(peers);
        }
        wsync();
    }
}

} // namespace udpdk
