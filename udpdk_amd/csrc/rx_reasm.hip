// rx_reasm.hip — gfx950 RX reassembly of IPv4 fragments: the poller's
// rte_ipv4_frag_reassemble_packet step (udpdk_poller.c:338-361) over a whole batch, against a
// device-resident flow table with the geometry of the poller's rte_ip_frag_table_create
// (udpdk_poller.c:130: NUM_FLOWS_DEF buckets x IP_FRAG_TBL_BUCKET_ENTRIES, frag_cycles TTL).
//
// Semantics: oracle/udpdk_oracle_frag.c restates DPDK 20.05's table (ip_frag_lookup/find/process,
// ipv4_frag_reassemble) and is the parity checker; this file follows it fragment for fragment.
// The reference handles one fragment at a time in arrival order; here the batch's fragments are
// grouped by flow key (two stable radix sorts: (id, index) then src|dst) and each flow's fragments
// are processed in arrival order by one wavefront, flows in parallel. The result equals the
// sequential one whenever the flows of a batch do not compete for the last free slot of a
// bucket pair (then which flow gets it depends on timing, as it would on arrival order).
//
// Launch sequence (udpdk_gpu_rx_reassemble, synchronous):
//   reasm_collect   FRAG verdicts -> fragment list + (id << 32 | index) sort keys
//   radix sort 1    by (id, index); reasm_keys: src|dst keys in that order; radix sort 2 (stable)
//   reasm_process   one wave per flow segment: table find (2 x assoc slots scanned by the lanes,
//                   entry locks), ip_frag_process on lane 0, completion records, store jobs
//   radix sort 3    completions by origin (the arrival index of the completing fragment: where
//                   the reference delivers the datagram) + exclusive scan of frame sizes
//   reasm_emit      one wave per datagram: first fragment's header (total length, DF only, IPv4
//                   checksum) + every fragment's data at its offset, from the batch or the table
//   reasm_store     one wave per fragment left pending: its data (and header, for offset 0) into
//                   the flow's entry buffer, after every read of the table buffers
//
// Table memory: entries x 80 B of state + entries x stride bytes of fragment data (stride =
// 34 + max_dgram rounded to 256). All cross-wave state is accessed with agent-scope atomics (the
// per-XCD L2s are not coherent for plain accesses); entry locks are acquire/release.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>

#include <algorithm>
#include <cerrno>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

namespace {

constexpr uint32_t RS_BLOCK = 256;
constexpr uint32_t RS_WAVES = RS_BLOCK / 64;
constexpr uint32_t RS_HELD = 0xFFFFFFFFu;       // fragment data lives in the entry buffer
constexpr uint32_t RS_NONE = 0xFFFFFFFFu;
constexpr uint32_t RS_MAX_FRAG = 4;             // RTE_LIBRTE_IP_FRAG_MAX_FRAG
constexpr uint32_t RS_SPIN = 1u << 20;          // bound on lock spins / find retries

struct FragEntry {            // one table entry (struct ip_frag_pkt)
    uint32_t lock;            // 0 free, else holder tag
    uint32_t valid;           // key_len != 0
    uint32_t src, dst, id;
    uint32_t frag_size, total_size, last_idx;
    unsigned long long start;
    uint32_t fr[RS_MAX_FRAG];     // ofs | len << 16, 0 = empty slot (len > 0 when present)
    uint32_t where[RS_MAX_FRAG];  // frame index in the current call, or RS_HELD
};

struct ReasmDone {            // one reassembled datagram
    uint32_t origin, total, n, entry;
    uint32_t fr[RS_MAX_FRAG], where[RS_MAX_FRAG];
};

struct ReasmJob { uint32_t frame, entry, fr, pad; };

struct ReasmArgs {
    const uint8_t *frames;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *meta;
    uint32_t n, rsrc_bytes;
    uint32_t *frag_list;               // [F] (unordered)
    unsigned long long *k1;            // [F] id << 32 | index
    const uint32_t *v1s;               // [F] frame indices sorted by (id, index)
    unsigned long long *k2;            // [F] src | dst << 32 in v1s order
    const uint32_t *order;             // [F] frame indices sorted by (src, dst, id, index)
    uint32_t *counts;                  // [0] F, [1] completions, [2] store jobs
    unsigned long long *stats;         // [UDPDK_RS_N]
    unsigned long long *out_bytes;
    FragEntry *tab;
    uint8_t *ebuf;
    uint32_t mask, assoc, max_dgram, stride;
    unsigned long long max_cycles, tms;
    ReasmDone *done;
    ReasmJob *jobs;
    uint32_t tag_base;
};

template <typename T>
__device__ __forceinline__ T ld_a(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_a(T *p, T v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint32_t ld32(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

__device__ __forceinline__ uint32_t crc32c_u32(uint32_t crc, uint32_t v)
{
    crc ^= v;
#pragma unroll
    for (int i = 0; i < 32; ++i) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    return crc;
}

// Fragment header fields of frame i.
struct FragHdr {
    uint32_t src, dst, id, tl, ff, flen;
};

__device__ __forceinline__ FragHdr frag_hdr(const ReasmArgs &a, __amdgpu_buffer_rsrc_t fr, uint32_t i)
{
    const uint32_t o = a.offset[i];
    FragHdr h;
    const uint32_t w16 = ld32(fr, o + 16);   // total length | id
    const uint32_t w20 = ld32(fr, o + 20);   // fragment field | ttl | proto
    h.tl = bswap16(w16 & 0xFFFFu);
    h.id = w16 >> 16;
    h.ff = bswap16(w20 & 0xFFFFu);
    h.src = ld32(fr, o + 26);
    h.dst = ld32(fr, o + 30);
    h.flen = a.length[i];
    return h;
}

// Wave copy of len bytes from (r, src_off) to dst: dword stores where the destination is
// dword-aligned, byte stores at both ends (neighbouring regions may share those dwords).
__device__ void wave_copy(uint8_t *dst, __amdgpu_buffer_rsrc_t r, uint32_t src_off, uint32_t len)
{
    const uint32_t lane = __lane_id();
    const uint32_t head = std::min<uint32_t>((4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u, len);
    if (lane < head) dst[lane] = (uint8_t)ld32(r, src_off + lane);
    const uint32_t body = (len - head) >> 2;
    uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + head);
    for (uint32_t k = lane; k < body; k += 64) d32[k] = ld32(r, src_off + head + 4u * k);
    const uint32_t tail = len - head - 4u * body;
    if (lane < tail) dst[head + 4u * body + lane] = (uint8_t)ld32(r, src_off + head + 4u * body + lane);
}

} // namespace

// FRAG verdicts -> fragment list and sort keys (order within the list does not matter: the
// keys carry the arrival index).
__global__ void __launch_bounds__(RS_BLOCK) reasm_collect(ReasmArgs a)
{
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    const uint32_t lane = __lane_id();
    for (uint32_t i0 = (blockIdx.x * RS_BLOCK + threadIdx.x) & ~63u; i0 < a.n; i0 += gridDim.x * RS_BLOCK) {
        const uint32_t i = i0 + lane;
        const bool f = i < a.n && (a.meta[i] & 0xFu) == UDPDK_V_FRAG;
        const unsigned long long m = __ballot(f);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == 0) {
            base = atomicAdd(&a.counts[0], (uint32_t)__popcll(m));
            atomicAdd(&a.stats[UDPDK_RS_FRAGS], (unsigned long long)__popcll(m));
        }
        base = __shfl(base, 0, 64);
        if (f) {
            const uint32_t j = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            const uint32_t id = ld32(fr, a.offset[i] + 16) >> 16;
            a.frag_list[j] = i;
            a.k1[j] = ((unsigned long long)id << 32) | i;
        }
    }
}

// src | dst << 32 of the fragments in (id, index) order (the second, stable, sort key).
__global__ void __launch_bounds__(RS_BLOCK) reasm_keys(ReasmArgs a, uint32_t F)
{
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    for (uint32_t p = blockIdx.x * RS_BLOCK + threadIdx.x; p < F; p += gridDim.x * RS_BLOCK) {
        const uint32_t o = a.offset[a.v1s[p]];
        a.k2[p] = (unsigned long long)ld32(fr, o + 26) | ((unsigned long long)ld32(fr, o + 30) << 32);
    }
}

namespace {

struct WaveState {                // lane 0's copy of the held entry (LDS, one per wave)
    uint32_t frag_size, total_size, last_idx;
    uint32_t fr[RS_MAX_FRAG], where[RS_MAX_FRAG];
};

// ip_frag_find: returns the locked entry for the key, or RS_NONE (no space). Wave-uniform.
__device__ uint32_t table_find(const ReasmArgs &a, uint32_t src, uint32_t dst, uint32_t id,
                               uint32_t tag, WaveState &ws)
{
    const uint32_t lane = __lane_id();
    uint32_t v = crc32c_u32(0xeaad8405u, src);
    v = crc32c_u32(v, dst);
    v = crc32c_u32(v, id);
    const uint32_t p1 = v & a.mask, p2 = ((v << 7) + (v >> 14)) & a.mask;
    for (uint32_t tries = 0; tries < RS_SPIN; ++tries) {
        // lanes scan p1[0], p2[0], p1[1], p2[1], ... (ip_frag_lookup's order)
        const bool in = lane < 2u * a.assoc;
        const uint32_t slot = (lane & 1u ? p2 : p1) + (lane >> 1);
        bool match = false, empty = false, stale = false;
        if (in) {
            const FragEntry *e = a.tab + slot;
            const uint32_t val = ld_a(&e->valid);
            if (val) {
                match = ld_a(&e->src) == src && ld_a(&e->dst) == dst && ld_a(&e->id) == id;
                stale = !match && a.max_cycles + ld_a(&e->start) < a.tms;
            } else {
                empty = true;
            }
        }
        const unsigned long long mm = __ballot(match), ms = __ballot(stale), me = __ballot(empty);
        uint32_t cand;
        int kind;                                  // 0 match, 1 stale, 2 empty
        if (mm) { cand = __shfl(slot, __ffsll((long long)mm) - 1, 64); kind = 0; }
        else if (ms) { cand = __shfl(slot, __ffsll((long long)ms) - 1, 64); kind = 1; }
        else if (me) { cand = __shfl(slot, __ffsll((long long)me) - 1, 64); kind = 2; }
        else return RS_NONE;
        uint32_t ok = 0;
        if (lane == 0) {
            FragEntry *e = a.tab + cand;
            uint32_t exp = 0;
            bool got = __hip_atomic_compare_exchange_strong(&e->lock, &exp, tag, __ATOMIC_ACQUIRE,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // a matching entry can only be held briefly by a wave testing it as a candidate
            for (uint32_t s = 0; !got && kind == 0 && s < RS_SPIN; ++s) {
                __builtin_amdgcn_s_sleep(2);
                exp = 0;
                got = __hip_atomic_compare_exchange_strong(&e->lock, &exp, tag, __ATOMIC_ACQUIRE,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (got) {
                const uint32_t val = ld_a(&e->valid);
                const bool same = val && ld_a(&e->src) == src && ld_a(&e->dst) == dst && ld_a(&e->id) == id;
                const bool expired = val && a.max_cycles + ld_a(&e->start) < a.tms;
                bool fresh = false;
                if (kind == 0 && same) {
                    ok = 1;
                    if (expired) {                                   // ip_frag_tbl_reuse
                        atomicAdd(&a.stats[UDPDK_RS_EXPIRED], 1ull);
                        fresh = true;
                    }
                } else if (kind == 1 && val && !same && expired) {   // ip_frag_tbl_del + add
                    atomicAdd(&a.stats[UDPDK_RS_EXPIRED], 1ull);
                    ok = 1;
                    fresh = true;
                } else if (kind == 2 && !val) {                      // ip_frag_tbl_add
                    ok = 1;
                    fresh = true;
                }
                if (ok && fresh) {
                    st_a(&e->src, src);
                    st_a(&e->dst, dst);
                    st_a(&e->id, id);
                    st_a(&e->start, a.tms);
                    st_a(&e->valid, 1u);
                    ws.frag_size = 0;
                    ws.total_size = 0xFFFFFFFFu;
                    ws.last_idx = 2;
                    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) { ws.fr[k] = 0; ws.where[k] = RS_HELD; }
                } else if (ok) {
                    ws.frag_size = ld_a(&e->frag_size);
                    ws.total_size = ld_a(&e->total_size);
                    ws.last_idx = ld_a(&e->last_idx);
                    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
                        ws.fr[k] = ld_a(&e->fr[k]);
                        ws.where[k] = ld_a(&e->where[k]);
                    }
                } else {
                    __hip_atomic_store(&e->lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        ok = __shfl(ok, 0, 64);
        if (ok) return cand;
    }
    return RS_NONE;
}

// Write the held entry's state back and release it (lane 0).
__device__ void table_release(const ReasmArgs &a, uint32_t cur, const WaveState &ws, bool invalidate)
{
    FragEntry *e = a.tab + cur;
    if (invalidate) {
        st_a(&e->valid, 0u);
    } else {
        st_a(&e->frag_size, ws.frag_size);
        st_a(&e->total_size, ws.total_size);
        st_a(&e->last_idx, ws.last_idx);
        for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
            st_a(&e->fr[k], ws.fr[k]);
            st_a(&e->where[k], ws.where[k]);
        }
    }
    __hip_atomic_store(&e->lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ipv4_frag_reassemble's backward chain walk over the held fragments.
__device__ bool chain_ok(const WaveState &ws)
{
    const uint32_t first_len = ws.fr[0] >> 16;
    const uint32_t n = ws.last_idx - 1u;
    uint32_t ofs = ws.fr[1] & 0xFFFFu, curr = 1;
    for (uint32_t guard = 0; ofs != first_len && guard < 8; ++guard) {
        const uint32_t prev = curr;
        for (uint32_t i = n; i != 0 && ofs != first_len; i--) {
            if ((ws.fr[i] & 0xFFFFu) + (ws.fr[i] >> 16) == ofs) {
                curr = i;
                ofs = ws.fr[i] & 0xFFFFu;
            }
        }
        if (curr == prev) return false;
    }
    return ofs == first_len;
}

} // namespace

// One wave per flow segment of the sorted fragment list.
__global__ void __launch_bounds__(RS_BLOCK) reasm_process(ReasmArgs a, uint32_t F)
{
    __shared__ WaveState s_ws[RS_WAVES];
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    WaveState &ws = s_ws[w];
    const uint32_t gw = blockIdx.x * RS_WAVES + w, nw = gridDim.x * RS_WAVES;
    const uint32_t tag = a.tag_base + gw + 1u;
    for (uint32_t base = gw * 64u; base < F; base += nw * 64u) {
        const uint32_t p = base + lane;
        bool start = false;
        if (p < F) {
            const FragHdr h = frag_hdr(a, fr, a.order[p]);
            if (p == 0) {
                start = true;
            } else {
                const FragHdr g = frag_hdr(a, fr, a.order[p - 1]);
                start = g.src != h.src || g.dst != h.dst || g.id != h.id;
            }
        }
        unsigned long long starts = __ballot(start);
        while (starts) {
            const uint32_t s = base + (uint32_t)(__ffsll((long long)starts) - 1);
            starts &= starts - 1ull;
            const FragHdr k0 = frag_hdr(a, fr, a.order[s]);
            uint32_t cur = RS_NONE;
            for (uint32_t q = s; q < F; ++q) {
                const uint32_t i = a.order[q];
                const FragHdr h = frag_hdr(a, fr, i);
                if (q != s && (h.src != k0.src || h.dst != k0.dst || h.id != k0.id)) break;
                const int32_t ip_len = (int32_t)h.tl - 20;                // l3_len = 20
                if (ip_len <= 0) {
                    if (lane == 0) atomicAdd(&a.stats[UDPDK_RS_DROP_LEN], 1ull);
                    continue;
                }
                const uint32_t len = (uint32_t)ip_len;
                const uint32_t ofs = (h.ff & 0x1FFFu) * 8u, mf = h.ff & 0x2000u;
                if (34u + len > h.flen || ofs + len > a.max_dgram) {
                    if (lane == 0) atomicAdd(&a.stats[UDPDK_RS_DROP_SHORT], 1ull);
                    continue;
                }
                if (cur == RS_NONE) {
                    cur = table_find(a, k0.src, k0.dst, k0.id, tag, ws);
                    if (cur == RS_NONE) {
                        if (lane == 0) atomicAdd(&a.stats[UDPDK_RS_NO_SPACE], 1ull);
                        continue;
                    }
                }
                // ip_frag_process (lane 0 owns the state; the outcome is broadcast)
                uint32_t keep = 1;
                if (lane == 0) {
                    uint32_t idx;
                    ws.frag_size += len;
                    if (ofs == 0) {
                        idx = ws.fr[0] == 0 ? 0u : RS_NONE;
                    } else if (!mf) {
                        ws.total_size = ofs + len;
                        idx = ws.fr[1] == 0 ? 1u : RS_NONE;
                    } else {
                        idx = ws.last_idx;
                        if (idx < RS_MAX_FRAG) ws.last_idx++;
                    }
                    if (idx >= RS_MAX_FRAG) {
                        atomicAdd(&a.stats[UDPDK_RS_ERRORS], 1ull);
                        table_release(a, cur, ws, true);
                        keep = 0;
                    } else {
                        ws.fr[idx] = ofs | (len << 16);
                        ws.where[idx] = i;
                        if (ws.frag_size >= ws.total_size) {
                            const bool sized = ws.frag_size == ws.total_size && ws.fr[0] != 0;
                            if (sized && chain_ok(ws)) {
                                const uint32_t d = atomicAdd(&a.counts[1], 1u);
                                ReasmDone r;
                                r.origin = i;
                                r.total = ws.total_size;
                                r.n = ws.last_idx;
                                r.entry = cur;
                                for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) { r.fr[k] = ws.fr[k]; r.where[k] = ws.where[k]; }
                                a.done[d] = r;
                                atomicAdd(a.out_bytes, (unsigned long long)((34u + ws.total_size + 15u) & ~15u));
                                atomicAdd(&a.stats[UDPDK_RS_DONE], 1ull);
                            } else {
                                atomicAdd(&a.stats[sized ? UDPDK_RS_HOLES : UDPDK_RS_ERRORS], 1ull);
                            }
                            table_release(a, cur, ws, true);
                            keep = 0;
                        }
                    }
                }
                if (!__shfl(keep, 0, 64)) cur = RS_NONE;
            }
            if (cur != RS_NONE && lane == 0) {
                // still pending: this call's fragments move into the entry buffer (reasm_store)
                for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
                    if (ws.fr[k] && ws.where[k] != RS_HELD) {
                        const uint32_t j = atomicAdd(&a.counts[2], 1u);
                        ReasmJob jb;
                        jb.frame = ws.where[k];
                        jb.entry = cur;
                        jb.fr = ws.fr[k];
                        jb.pad = 0;
                        a.jobs[j] = jb;
                        ws.where[k] = RS_HELD;
                        atomicAdd(&a.stats[UDPDK_RS_STORED], 1ull);
                    }
                }
                table_release(a, cur, ws, false);
            }
        }
    }
}

// Sort keys of the completions: the arrival index of the completing fragment.
__global__ void __launch_bounds__(RS_BLOCK) reasm_origin_keys(const ReasmDone *done, unsigned long long *k,
                                                             uint32_t *v, uint32_t C)
{
    for (uint32_t j = blockIdx.x * RS_BLOCK + threadIdx.x; j < C; j += gridDim.x * RS_BLOCK) {
        k[j] = done[j].origin;
        v[j] = j;
    }
}

// Frame sizes of the completions in origin order (for the offset scan).
__global__ void __launch_bounds__(RS_BLOCK) reasm_sizes(const ReasmDone *done, const uint32_t *perm,
                                                       uint32_t *sizes, uint32_t C)
{
    for (uint32_t k = blockIdx.x * RS_BLOCK + threadIdx.x; k < C; k += gridDim.x * RS_BLOCK)
        sizes[k] = (34u + done[perm[k]].total + 15u) & ~15u;
}

struct EmitArgs {
    const uint8_t *frames;
    const uint32_t *offset;
    uint32_t rsrc_bytes;
    const uint8_t *ebuf;
    uint32_t stride;
    const ReasmDone *done;
    const uint32_t *perm;
    const uint32_t *out_off_in;   // scan of the sizes
    uint8_t *out;
    uint32_t *out_off;
    uint16_t *out_len;
    uint32_t *out_ptype;
    uint32_t *out_origin;
    uint32_t C;
};

__global__ void __launch_bounds__(RS_BLOCK) reasm_emit(EmitArgs a)
{
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    for (uint32_t k = blockIdx.x * RS_WAVES + w; k < a.C; k += gridDim.x * RS_WAVES) {
        const ReasmDone r = a.done[a.perm[k]];
        const uint32_t oo = a.out_off_in[k];
        uint8_t *o = a.out + oo;
        const uint8_t *eb = a.ebuf + (size_t)r.entry * a.stride;
        const __amdgpu_buffer_rsrc_t er = rsrc(eb, a.stride);
        // header: the first fragment's 34 bytes (ipv4_frag_reassemble keeps the first mbuf's)
        const bool hh = r.where[0] == RS_HELD;
        const __amdgpu_buffer_rsrc_t hr = hh ? er : fr;
        const uint32_t hb = hh ? 0u : a.offset[r.where[0]];
        uint32_t hw = 0;
        if (lane < 9) hw = ld32(hr, hb + 4u * lane);      // bytes 0..35 (34, 35 dropped)
        // dword 4: bytes 16-17 total length, 18-19 id; dword 5: 20-21 fragment field, 22-23;
        // dword 6: 24-25 checksum, 26-27 src
        const uint32_t tl = r.total + 20u;
        if (lane == 4) hw = (hw & 0xFFFF0000u) | bswap16(tl);
        if (lane == 5) hw = (hw & 0xFFFF0000u) | (hw & 0x40u);                  // DF only
        if (lane == 6) hw &= 0xFFFF0000u;
        // RFC 1071 sum over IPv4 header bytes 14..33 (dwords 3..8, minus bytes 12-13, 34-35)
        uint32_t part = 0;
        if (lane >= 3 && lane < 9) {
            uint32_t x = hw;
            if (lane == 3) x &= 0xFFFF0000u;
            if (lane == 8) x &= 0x0000FFFFu;
            part = (x & 0xFFFFu) + (x >> 16);
        }
        // bytes 14.. are the odd halves: dword 3 holds bytes 12-15 -> 14-15 in its high half; the
        // 16-bit words of the header are (14,15), (16,17), ... i.e. high half of dword 3, then
        // both halves of dwords 4..7, then the low half of dword 8: all 16-bit aligned
        for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d, 64);
        uint32_t s = part;
        s = (s >> 16) + (s & 0xFFFFu);
        s = (s >> 16) + (s & 0xFFFFu);
        const uint32_t ck = ~s & 0xFFFFu;
        if (lane == 6) hw |= ck;
        if (lane < 8) reinterpret_cast<uint32_t *>(o)[lane] = hw;      // o is 16-byte aligned
        if (lane == 8) { o[32] = (uint8_t)hw; o[33] = (uint8_t)(hw >> 8); }
        for (uint32_t q = 0; q < r.n && q < RS_MAX_FRAG; ++q) {
            if (!r.fr[q]) continue;
            const uint32_t ofs = r.fr[q] & 0xFFFFu, len = r.fr[q] >> 16;
            if (r.where[q] == RS_HELD) wave_copy(o + 34 + ofs, er, 34u + ofs, len);
            else wave_copy(o + 34 + ofs, fr, a.offset[r.where[q]] + 34u, len);
        }
        if (lane == 0) {
            a.out_off[k] = oo;
            a.out_len[k] = (uint16_t)(34u + r.total);
            a.out_ptype[k] = 0x211u;              // L2_ETHER | L3_IPV4 | L4_UDP
            a.out_origin[k] = r.origin;
        }
    }
}

struct StoreArgs {
    const uint8_t *frames;
    const uint32_t *offset;
    uint32_t rsrc_bytes;
    uint8_t *ebuf;
    uint32_t stride;
    const ReasmJob *jobs;
    uint32_t J;
};

__global__ void __launch_bounds__(RS_BLOCK) reasm_store(StoreArgs a)
{
    const uint32_t w = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    for (uint32_t k = blockIdx.x * RS_WAVES + w; k < a.J; k += gridDim.x * RS_WAVES) {
        const ReasmJob jb = a.jobs[k];
        uint8_t *eb = a.ebuf + (size_t)jb.entry * a.stride;
        const uint32_t ofs = jb.fr & 0xFFFFu, len = jb.fr >> 16, fo = a.offset[jb.frame];
        if (ofs == 0) wave_copy(eb, fr, fo, 34u);
        wave_copy(eb + 34 + ofs, fr, fo + 34u, len);
    }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct Reasm {
    int device = 0;
    FragEntry *tab = nullptr;
    uint8_t *ebuf = nullptr;
    uint32_t entries = 0, assoc = 0, mask = 0, max_dgram = 0, stride = 0;
    uint64_t max_cycles = 0;
    uint32_t cap = 0;                        // fragments per call (= context max_frames)
    uint32_t *frag_list = nullptr, *v1 = nullptr, *v1s = nullptr, *v2s = nullptr;
    unsigned long long *k1 = nullptr, *k1s = nullptr, *k2 = nullptr, *k2s = nullptr;
    uint32_t *counts = nullptr;              // device [4]
    unsigned long long *stats = nullptr;     // device [UDPDK_RS_N]
    unsigned long long *out_bytes = nullptr;
    ReasmDone *done = nullptr;
    ReasmJob *jobs = nullptr;
    unsigned long long *dk = nullptr, *dks = nullptr;
    uint32_t *dv = nullptr, *perm = nullptr, *sizes = nullptr, *offs = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    uint32_t *host = nullptr;                // pinned readback: counts + out_bytes + stats
    uint8_t *out = nullptr;
    uint64_t out_cap = 0;
    uint32_t *out_off = nullptr, *out_ptype = nullptr, *out_origin = nullptr;
    uint16_t *out_len = nullptr;
    uint32_t calls = 0;
};

namespace {

template <typename T>
hipError_t dalloc(T **p, size_t count)
{
    return hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T));
}

} // namespace

#define RS_HIP(expr)                                                         \
    do {                                                                     \
        hipError_t e_ = (expr);                                              \
        if (e_ != hipSuccess) { *hip_err = (int)e_; return -EIO; }           \
    } while (0)

void reasm_destroy(Reasm *r)
{
    if (!r) return;
    void *dev[] = {r->tab, r->ebuf, r->frag_list, r->v1, r->v1s, r->v2s, r->k1, r->k1s, r->k2,
                   r->k2s, r->counts, r->stats, r->out_bytes, r->done, r->jobs, r->dk, r->dks,
                   r->dv, r->perm, r->sizes, r->offs, r->tmp, r->out, r->out_off, r->out_ptype,
                   r->out_origin, r->out_len};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (r->host) (void)hipHostFree(r->host);
    delete r;
}

int reasm_create(Reasm **out, int device, uint32_t max_frames, const udpdk_frag_table_cfg_t *cfg,
                 int *hip_err)
{
    const uint64_t want = (uint64_t)cfg->bucket_num * cfg->bucket_entries;
    if (!cfg->bucket_num || !cfg->bucket_entries || (cfg->bucket_entries & (cfg->bucket_entries - 1)) ||
        cfg->bucket_entries > 32 || want > (1u << 22) || !cfg->max_dgram || cfg->max_dgram > 65515u)
        return -EINVAL;
    uint64_t entries = 1;
    while (entries < want) entries <<= 1;
    Reasm *r = new (std::nothrow) Reasm;
    if (!r) return -ENOMEM;
    r->device = device;
    r->entries = (uint32_t)entries;
    r->assoc = cfg->bucket_entries;
    r->mask = (r->entries - 1u) & ~(r->assoc - 1u);
    r->max_cycles = cfg->max_cycles;
    r->max_dgram = cfg->max_dgram;
    r->stride = (34u + cfg->max_dgram + 4u + 255u) & ~255u;   // + 4: dword loads of the last bytes
    r->cap = std::max<uint32_t>(max_frames, 1);
    int rc = 0;
    auto fail = [&](hipError_t e) { *hip_err = (int)e; rc = e == hipErrorOutOfMemory ? -ENOMEM : -EIO; };
    hipError_t e = hipSuccess;
    const size_t C = r->cap;
    if ((e = dalloc(&r->tab, r->entries)) != hipSuccess ||
        (e = hipMemset(r->tab, 0, (size_t)r->entries * sizeof(FragEntry))) != hipSuccess ||
        (e = hipMalloc((void **)&r->ebuf, (size_t)r->entries * r->stride)) != hipSuccess ||
        (e = dalloc(&r->frag_list, C)) != hipSuccess || (e = dalloc(&r->v1s, C)) != hipSuccess ||
        (e = dalloc(&r->v2s, C)) != hipSuccess || (e = dalloc(&r->k1, C)) != hipSuccess ||
        (e = dalloc(&r->k1s, C)) != hipSuccess || (e = dalloc(&r->k2, C)) != hipSuccess ||
        (e = dalloc(&r->k2s, C)) != hipSuccess || (e = dalloc(&r->counts, 4)) != hipSuccess ||
        (e = dalloc(&r->stats, UDPDK_RS_N)) != hipSuccess || (e = dalloc(&r->out_bytes, 1)) != hipSuccess ||
        (e = dalloc(&r->done, C)) != hipSuccess || (e = dalloc(&r->jobs, C)) != hipSuccess ||
        (e = dalloc(&r->dk, C)) != hipSuccess || (e = dalloc(&r->dks, C)) != hipSuccess ||
        (e = dalloc(&r->dv, C)) != hipSuccess || (e = dalloc(&r->perm, C)) != hipSuccess ||
        (e = dalloc(&r->sizes, C)) != hipSuccess || (e = dalloc(&r->offs, C)) != hipSuccess ||
        (e = dalloc(&r->out_off, C)) != hipSuccess || (e = dalloc(&r->out_len, C)) != hipSuccess ||
        (e = dalloc(&r->out_ptype, C)) != hipSuccess || (e = dalloc(&r->out_origin, C)) != hipSuccess ||
        (e = hipHostMalloc((void **)&r->host, 4096)) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    // rocPRIM temporary storage for the largest call (sorts of u64 keys / u32 values, u32 scan)
    size_t t1 = 0, t2 = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, t1, r->k1, r->k1s, r->v1s, r->v2s, (size_t)C, 0, 64)) != hipSuccess ||
        (e = rocprim::exclusive_scan(nullptr, t2, r->sizes, r->offs, 0u, (size_t)C, rocprim::plus<uint32_t>())) != hipSuccess ||
        (e = hipMalloc(&r->tmp, std::max<size_t>(std::max(t1, t2), 256))) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    r->tmp_bytes = std::max<size_t>(std::max(t1, t2), 256);
    *out = r;
    return 0;
}

int reasm_run(Reasm *r, hipStream_t st, const udpdk_rx_batch_t *bt, const uint32_t *meta_dev,
              uint64_t tms, udpdk_reasm_out_t *o, int *hip_err)
{
    if (bt->n > r->cap) return -EINVAL;
    const uint32_t n = bt->n;
    ReasmArgs a;
    a.frames = bt->frames_dev;
    a.offset = bt->offset_dev;
    a.length = bt->length_dev;
    a.meta = meta_dev;
    a.n = n;
    a.rsrc_bytes = (uint32_t)std::min<uint64_t>((bt->frames_bytes + 3 + 3) & ~3ull, 0xFFFFFFFCull);
    a.frag_list = r->frag_list;
    a.k1 = r->k1;
    a.v1s = r->v1s;
    a.k2 = r->k2;
    a.order = r->v2s;
    a.counts = r->counts;
    a.stats = r->stats;
    a.out_bytes = r->out_bytes;
    a.tab = r->tab;
    a.ebuf = r->ebuf;
    a.mask = r->mask;
    a.assoc = r->assoc;
    a.max_dgram = r->max_dgram;
    a.stride = r->stride;
    a.max_cycles = r->max_cycles;
    a.tms = tms;
    a.done = r->done;
    a.jobs = r->jobs;
    a.tag_base = 0;
    RS_HIP(hipMemsetAsync(r->counts, 0, 4 * sizeof(uint32_t), st));
    RS_HIP(hipMemsetAsync(r->stats, 0, UDPDK_RS_N * sizeof(unsigned long long), st));
    RS_HIP(hipMemsetAsync(r->out_bytes, 0, sizeof(unsigned long long), st));
    const uint32_t g1 = std::max<uint32_t>(1, std::min<uint32_t>((n + RS_BLOCK - 1) / RS_BLOCK, 4096));
    hipLaunchKernelGGL(reasm_collect, dim3(g1), dim3(RS_BLOCK), 0, st, a);
    RS_HIP(hipGetLastError());
    RS_HIP(hipMemcpyAsync(r->host, r->counts, 4, hipMemcpyDeviceToHost, st));
    RS_HIP(hipStreamSynchronize(st));
    const uint32_t F = r->host[0];
    memset(o, 0, sizeof(*o));
    if (F) {
        size_t tb = r->tmp_bytes;
        RS_HIP(rocprim::radix_sort_pairs(r->tmp, tb, r->k1, r->k1s, r->frag_list, r->v1s, (size_t)F, 0, 48, st));
        const uint32_t gF = std::max<uint32_t>(1, std::min<uint32_t>((F + RS_BLOCK - 1) / RS_BLOCK, 4096));
        hipLaunchKernelGGL(reasm_keys, dim3(gF), dim3(RS_BLOCK), 0, st, a, F);
        RS_HIP(hipGetLastError());
        tb = r->tmp_bytes;
        RS_HIP(rocprim::radix_sort_pairs(r->tmp, tb, r->k2, r->k2s, r->v1s, r->v2s, (size_t)F, 0, 64, st));
        a.tag_base = (r->calls++ & 0x3FFu) << 20;
        const uint32_t waves = (F + 63u) / 64u;
        const uint32_t gp = std::max<uint32_t>(1, std::min<uint32_t>((waves + RS_WAVES - 1) / RS_WAVES, 2048));
        hipLaunchKernelGGL(reasm_process, dim3(gp), dim3(RS_BLOCK), 0, st, a, F);
        RS_HIP(hipGetLastError());
    }
    RS_HIP(hipMemcpyAsync(r->host, r->counts, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    RS_HIP(hipMemcpyAsync(r->host + 4, r->out_bytes, 8, hipMemcpyDeviceToHost, st));
    RS_HIP(hipMemcpyAsync(r->host + 8, r->stats, UDPDK_RS_N * 8, hipMemcpyDeviceToHost, st));
    RS_HIP(hipStreamSynchronize(st));
    const uint32_t Cn = r->host[1], J = r->host[2];
    uint64_t ob;
    memcpy(&ob, r->host + 4, 8);
    memcpy(o->stats, r->host + 8, UDPDK_RS_N * 8);
    if (Cn) {
        if (ob + UDPDK_GPU_FRAMES_TAILROOM > r->out_cap) {
            if (r->out) RS_HIP(hipFree(r->out));
            r->out = nullptr;
            r->out_cap = 0;
            const uint64_t nc = std::max<uint64_t>(ob + UDPDK_GPU_FRAMES_TAILROOM, 1u << 20) * 2;
            RS_HIP(hipMalloc((void **)&r->out, nc));
            r->out_cap = nc;
        }
        // completions in origin (arrival) order, then their frame offsets
        const uint32_t gC = std::max<uint32_t>(1, std::min<uint32_t>((Cn + RS_BLOCK - 1) / RS_BLOCK, 4096));
        hipLaunchKernelGGL(reasm_origin_keys, dim3(gC), dim3(RS_BLOCK), 0, st,
                           (const ReasmDone *)r->done, r->dk, r->dv, Cn);
        RS_HIP(hipGetLastError());
        size_t tb = r->tmp_bytes;
        RS_HIP(rocprim::radix_sort_pairs(r->tmp, tb, r->dk, r->dks, r->dv, r->perm, (size_t)Cn, 0, 32, st));
        hipLaunchKernelGGL(reasm_sizes, dim3(gC), dim3(RS_BLOCK), 0, st, (const ReasmDone *)r->done,
                           (const uint32_t *)r->perm, r->sizes, Cn);
        RS_HIP(hipGetLastError());
        tb = r->tmp_bytes;
        RS_HIP(rocprim::exclusive_scan(r->tmp, tb, r->sizes, r->offs, 0u, (size_t)Cn,
                                       rocprim::plus<uint32_t>(), st));
        EmitArgs ea;
        ea.frames = bt->frames_dev;
        ea.offset = bt->offset_dev;
        ea.rsrc_bytes = a.rsrc_bytes;
        ea.ebuf = r->ebuf;
        ea.stride = r->stride;
        ea.done = r->done;
        ea.perm = r->perm;
        ea.out_off_in = r->offs;
        ea.out = r->out;
        ea.out_off = r->out_off;
        ea.out_len = r->out_len;
        ea.out_ptype = r->out_ptype;
        ea.out_origin = r->out_origin;
        ea.C = Cn;
        const uint32_t ge = std::max<uint32_t>(1, std::min<uint32_t>((Cn + RS_WAVES - 1) / RS_WAVES, 8192));
        hipLaunchKernelGGL(reasm_emit, dim3(ge), dim3(RS_BLOCK), 0, st, ea);
        RS_HIP(hipGetLastError());
    }
    if (J) {   // after every read of the entry buffers (reasm_emit)
        StoreArgs sa;
        sa.frames = bt->frames_dev;
        sa.offset = bt->offset_dev;
        sa.rsrc_bytes = a.rsrc_bytes;
        sa.ebuf = r->ebuf;
        sa.stride = r->stride;
        sa.jobs = r->jobs;
        sa.J = J;
        const uint32_t gs = std::max<uint32_t>(1, std::min<uint32_t>((J + RS_WAVES - 1) / RS_WAVES, 8192));
        hipLaunchKernelGGL(reasm_store, dim3(gs), dim3(RS_BLOCK), 0, st, sa);
        RS_HIP(hipGetLastError());
    }
    RS_HIP(hipStreamSynchronize(st));
    o->batch.frames_dev = r->out;
    o->batch.frames_bytes = Cn ? ob : 0;
    o->batch.offset_dev = r->out_off;
    o->batch.length_dev = r->out_len;
    o->batch.ptype_dev = r->out_ptype;
    o->batch.n = Cn;
    o->origin_dev = r->out_origin;
    return 0;
}

} // namespace udpdk
