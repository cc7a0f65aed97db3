// rx_reasm.hip — gfx950 RX reassembly of IPv4 fragments: the poller's
// rte_ipv4_frag_reassemble_packet step (udpdk_poller.c:338-361) over a whole batch, against a
// device-resident flow table with the geometry of the poller's rte_ip_frag_table_create
// (udpdk_poller.c:130: NUM_FLOWS_DEF buckets x IP_FRAG_TBL_BUCKET_ENTRIES, frag_cycles TTL).
//
// Semantics: oracle/udpdk_oracle_frag.c restates DPDK 20.05's table (ip_frag_lookup/find/process,
// ipv4_frag_reassemble) and is the parity checker; this file follows it fragment for fragment.
// The reference handles one fragment at a time in arrival order. Here the batch's fragments are
// grouped by flow key (two stable radix sorts: (id, index) then src|dst), and the result is the
// same as the reference's for every batch:
//  * flows only interact through the entries of their two buckets, and only at a lookup;
//  * a flow whose lookups fall in a span [first, last fragment] that no other flow's span
//    overlaps on a shared bucket, whose buckets hold no expired entry and not its key, that
//    ends (completes or fails) by its last fragment, and whose buckets are sure to have a free
//    entry, holds an entry only while no one else looks: it is reassembled in parallel without
//    the table (reasm_process);
//  * every other flow's fragments go through the table in arrival order on one wave
//    (reasm_serial), which is then exactly the reference's sequence of ip_frag_find calls.
// Launch sequence (udpdk_gpu_rx_reassemble, synchronous):
//   reasm_fsel_*    FRAG verdicts -> fragment list in arrival order (+ the stats block zeroed);
//                   the count launch's extra blocks make the bucket summary: valid entries per
//                   bucket, any expired (the table is unchanged until the analysis reads it)
//   reasm_scan      does every flow key form one run (grouped)? The per-position records and,
//                   as if grouped, each flow's walk: its completions (counted per chunk of the
//                   completion list), whether it is complex, its outcome (see the kernel)
//   [not grouped]   reasm_group (each key's group by an exact hash table) and one radix sort by
//                   (group, index); reasm_prep: the records in sorted order; reasm_flows: per
//                   flow its span, pending or not, key in the table, overlap records; radix sort
//                   4 + max scan + reasm_overlap: flows whose spans overlap on a shared bucket
//                   (grouped: no two spans overlap)
//   reasm_ec        a free entry guaranteed for every parallel flow, else all go serial
//   reasm_process   parallel flows without the table; the rest -> serial list (grouped with no
//                   complex flow: both add up reasm_scan's results)
//   radix sort 5    serial list by arrival; reasm_serial (the table in arrival order: one wave, or
//                   with the max_entries test not in play one per group of bucket components,
//                   reasm_cc)
//   reasm_clist_*   completions by origin (the arrival index of the completing fragment: where
//                   the reference delivers the datagram) and their output offsets: grouped, the
//                   positions holding one in order; else each record's position at its origin
//                   first (reasm_by_origin), then the origins holding one in order
//   reasm_emit      one wave per datagram: first fragment's header (total length, DF only, IPv4
//                   checksum) + every fragment's data at its offset, from the batch or the table
//   reasm_store     one wave per fragment left pending: its data (and header, for offset 0) into
//                   the flow's entry buffer, after every read of the table buffers
//
// Table memory: entries x 80 B of state + entries x stride bytes of fragment data (stride =
// 34 + max_dgram rounded to 256). Table words are accessed with agent-scope atomics (the per-XCD
// L2s are not coherent for plain accesses).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdint.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

namespace {

constexpr uint32_t RS_BLOCK = 256;
constexpr uint32_t RS_WAVES = RS_BLOCK / 64;
constexpr uint32_t RS_HELD = 0xFFFFFFFFu;       // fragment data lives in the entry buffer
constexpr uint32_t RS_NONE = 0xFFFFFFFFu;
// per-call device block: stats [UDPDK_RS_N], out_bytes [1], counts [10 x u32] (u64 words)
constexpr uint32_t RS_ZERO_WORDS = UDPDK_RS_N + 1 + 5;
constexpr uint32_t RS_MAX_FRAG = 4;             // RTE_LIBRTE_IP_FRAG_MAX_FRAG
#ifndef UDPDK_RS_FLOW_CHUNK
#define UDPDK_RS_FLOW_CHUNK 512
#endif
constexpr uint32_t RS_FLOW_CHUNK = UDPDK_RS_FLOW_CHUNK;   // sorted positions per reasm_flows block step (1024: +7 us per call)
// Positions per completion-list chunk (reasm_clist_*, and one reasm_scan block), 2 per thread
// (8: +6 us per call)
constexpr uint32_t RS_CL = 512;
constexpr uint32_t RS_PB = 6;         // reasm_scan's outcome words per block (pblk): DROP_LEN,
                                      // DROP_SHORT, DONE, HOLES, ERRORS, completed bytes

// Bits to hold every value in [0, v]
inline uint32_t bits_for(uint32_t v) { return v ? 32u - (uint32_t)__builtin_clz(v) : 1u; }

// One table entry (struct ip_frag_pkt) as 20 u32 words, every one accessed with agent-scope
// relaxed atomics; only reasm_serial writes them.
enum : uint32_t {
    E_LRU_IDX = 0,      // position in DPDK's LRU list: (E_LRU_CALL, E_LRU_IDX) = the call and the
                        // arrival index of the fragment that added or last reused the entry
    E_VALID = 1,        // key_len != 0
    E_SRC = 2, E_DST = 3, E_ID = 4,
    E_FSIZE = 5, E_TOTAL = 6, E_LAST = 7,
    E_START = 8,        // u64 start (lo, hi)
    E_FR = 10,          // [4] ofs | len << 16, 0 = empty slot (len > 0 when present)
    E_WHERE = 14,       // [4] frame index in the call E_CALL, or RS_HELD
    E_CALL = 18,        // the call whose fragments E_WHERE may name (older ones are held)
    E_LRU_CALL = 19,
    E_WORDS = 20
};

// Flags of a flow segment, at its first sorted position (pflag).
constexpr uint32_t PF_TOUCH = 1;      // has a fragment that reaches ip_frag_find
constexpr uint32_t PF_COMPLEX = 2;    // pending after its last fragment, key in the table, or an
                                      // expired entry in one of its buckets
constexpr uint32_t PF_SHARED = 4;     // its span overlaps another flow's on a shared bucket
constexpr uint32_t PF_START = 8;      // the first sorted position of a flow segment
// A flow's outcome as reasm_flows (or reasm_scan) found it walking the flow on its own (reasm_process uses it
// for a flow that runs without the table): 6-bit counts of length-class drops, completions,
// holes and errors, OC_OVF when a count or the completed bytes did not fit (the flow is then
// walked again by reasm_process).
constexpr uint32_t OC_OVF = 1u << 30;

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
    uint32_t ib;                       // index bits of the sort-1 key: n - 1 < 2^ib
    uint32_t *frag_list;               // [F] (unordered)
    unsigned long long *k1;            // [F] id << ib | index
    const uint32_t *v1s;               // [F] frame indices sorted by (id, index)
    unsigned long long *k2;            // [F] src | dst << 32 in v1s order
    const uint32_t *order;             // [F] frame indices sorted by (src, dst, id, index)
    // per sorted position (reasm_prep): frame index, key, crc32c signature, and
    // len | (fragment offset / 8) << 16 | MF << 29 | class << 30 (0 ok, 1 no data, 2 too long)
    uint32_t *s_i, *s_src, *s_dst, *s_id, *s_sig, *s_meta;
    // [0] F, [1] overlap records, [2] serial list, [3] fallback (every flow serial), [4] not
    // grouped, [5] in-place refused, [6] max_entries test, [7] flows the bound counts, [8] complex
    // flows (reasm_scan), [9] a completion reasm_scan could not count (the host tail then recounts)
    uint32_t *counts;
    unsigned long long *stats;         // [UDPDK_RS_N]
    unsigned long long *out_bytes;
    uint32_t *tab;                     // [entries][E_WORDS]
    uint8_t *ebuf;
    uint32_t mask, assoc, max_dgram, stride;
    unsigned long long max_cycles, tms;
    ReasmDone *done;                   // [F] at the completing fragment's position
    uint32_t *dk;                      // [F] origin of the completion there, or ~0
    uint32_t *dv;                      // [F] 0..F-1
    ReasmJob *jobs;                    // [F] at the stored fragment's position (frame ~0: none)
    // flow analysis (per first sorted position of a flow) and the serial path
    uint32_t assoc_log2, nbuckets;
    uint32_t *pflag, *sb1, *sb2, *tf, *tl;   // [F] flags, bucket pair, span
    uint32_t *oc, *ob;                 // [F] per flow start: outcome counts, completed bytes
    unsigned long long *rk;            // [2F] overlap records: bucket << ib | tf
    uint32_t *rv;                      // [2F] their flow's first position
    uint32_t *bsum, *cplx;             // [buckets] valid | stale << 31; complex flows
    uint32_t *sl_k, *sl_v;             // [F] serial list: arrival index, sorted position
    uint32_t *tpos;                    // [entries][4] sorted position of a slot's fragment (this call)
    uint32_t call;                     // this call's number (E_CALL), from 1
    // rte_ip_frag_table's max_entries / use_entries: the valid entries after the last call (only
    // reasm_serial changes the table, so it keeps the count); counts[6] = 1 when this call's
    // serial path must apply ip_frag_find's limit (reasm_ec), counts[7] = the flows the bound
    // counts (reasm_flows)
    uint32_t entries, max_entries;
    uint32_t *tab_used;
    // The run test (grouped or not): reasm_scan writes each run's first position into its key's
    // slot of rtab, reasm_ec reads the slots back; a run that lost its slot to another key goes
    // into hset, an exact set (run_insert)
    uint32_t *rtab;
    uint32_t rmask;
    unsigned long long *hset;
    uint32_t hmask;
    unsigned long long *gset;          // [hmask + 1] a batch that is not grouped: key -> group (reasm_group)
    uint32_t hset_tag;                 // hset's tag for this call, 1..65535
    uint32_t grouped;                  // every key one run in arrival order: no span overlaps
    uint32_t inplace;                  // udpdk_gpu_rx_reassemble_inplace: reasm_scan checks each completion
    // reasm_scan: per completion-list chunk its completions and their bytes ([2 x chunks], zeroed
    // by reasm_fsel_count_bsum), per block its outcome totals ([RS_PB x chunks])
    uint32_t *cblk;
    unsigned long long *pblk;
    uint32_t *cl_perm, *cl_offs;       // the grouped completion list (reasm_clist_write's perm, offs)
    const uint32_t *fcnt;              // FRAG frames per RS_FS frames (reasm_fsel_count_bsum)
    uint32_t nfs;
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

__device__ __forceinline__ uint4 load16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v)
{
    __attribute__((ext_vector_type(4))) uint32_t x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)off, 0, 0);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// crc32c (reflected, poly 0x82F63B78) of one dword, a byte at a time from a 256-entry table of
// the byte steps in LDS (crc_table_init): 4 lookups instead of 32 dependent bit steps (the
// bit-serial form was ~450 VALU instructions per fragment, a sixth of the run test's kernel).
__device__ __forceinline__ uint32_t crc32c_u32(const uint32_t *tab, uint32_t crc, uint32_t v)
{
    crc ^= v;
#pragma unroll
    for (int i = 0; i < 4; ++i) crc = (crc >> 8) ^ tab[crc & 0xFFu];
    return crc;
}

// The block's crc32c byte table (RS_BLOCK >= 256 threads, one entry each); the caller syncs.
__device__ __forceinline__ void crc_table_init(uint32_t *tab)
{
    if (threadIdx.x < 256u) {
        uint32_t c = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 8; ++i) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
        tab[threadIdx.x] = c;
    }
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

// As wave_copy, with 16-byte stores once the destination is 16-byte aligned (byte-aligned
// 16-byte loads from the source), up to four loads per lane in flight before their stores.
__device__ void wave_copy16(uint8_t *dst, __amdgpu_buffer_rsrc_t r, uint32_t src_off, uint32_t len)
{
    const uint32_t lane = __lane_id();
    const uint32_t head = std::min<uint32_t>((16u - ((uint32_t)(uintptr_t)dst & 15u)) & 15u, len);
    if (lane < head) dst[lane] = (uint8_t)ld32(r, src_off + lane);
    const uint32_t body = (len - head) >> 4;
    uint4 *d16 = reinterpret_cast<uint4 *>(dst + head);
    const uint32_t sb = src_off + head;
    for (uint32_t k0 = lane; k0 < body; k0 += 256u) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + 64u * u;
            if (k < body) {
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(sb + 16u * k), 0, 0);
                v[u] = make_uint4(x[0], x[1], x[2], x[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + 64u * u;
            if (k < body) d16[k] = v[u];
        }
    }
    const uint32_t done = head + 16u * body, tail = len - done;
    if (lane < tail) dst[done + lane] = (uint8_t)ld32(r, src_off + done + lane);
}

} // namespace

// rocPRIM select predicates, used for sizing its temporary storage only (the fragment list and
// the grouped completion list are built by reasm_fsel_* and reasm_clist_*).
struct IsFrag {
    const uint32_t *meta;
    __device__ bool operator()(uint32_t i) const { return (meta[i] & 0xFu) == UDPDK_V_FRAG; }
};
struct HasDone {
    const uint32_t *dk;
    __device__ bool operator()(uint32_t q) const { return dk[q] != RS_NONE; }
};

// The FRAG-verdict frames in arrival order (the fragment list, F to counts[0]): per block of
// RS_FS frames its FRAG count (reasm_fsel_count_bsum, whose workgroup 0 also zeroes the call's
// stats block), then reasm_scan's blocks each find and write their own positions of the list.
// (rocPRIM's select took a memset, its state initialisation and two passes.)
constexpr uint32_t RS_FS = 2048;                 // frames per block, 8 per thread

__device__ __forceinline__ uint32_t frag_bits8(const uint32_t *meta, uint32_t i0, uint32_t n)
{
    uint32_t m = 0;
    if (i0 + 8u <= n && ((uintptr_t)meta & 15u) == 0) {
        const uint4 a = *reinterpret_cast<const uint4 *>(meta + i0);
        const uint4 b = *reinterpret_cast<const uint4 *>(meta + i0 + 4u);
        const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) m |= (v[j] & 0xFu) == UDPDK_V_FRAG ? 1u << j : 0u;
    } else {
        for (uint32_t j = 0; j < 8 && i0 + j < n; ++j) m |= (meta[i0 + j] & 0xFu) == UDPDK_V_FRAG ? 1u << j : 0u;
    }
    return m;
}

__device__ __forceinline__ void fsel_count_block(const uint32_t *meta, uint32_t n, uint32_t *blk,
                                                 unsigned long long *stats_block, uint32_t b)
{
    __shared__ uint32_t red[RS_WAVES];
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    if (b == 0 && tid < RS_ZERO_WORDS) stats_block[tid] = 0ull;
    uint32_t c = (uint32_t)__builtin_popcount(frag_bits8(meta, b * RS_FS + 8u * tid, n));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if (lane == 0) red[w] = c;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
#pragma unroll
        for (uint32_t i = 0; i < RS_WAVES; ++i) t += red[i];
        blk[b] = t;
    }
}

// Per sorted position: the fragment's frame, key, signature and length class (all lanes in
// parallel, so the flow walk below reads one coalesced record per fragment).
// dv (the identity permutation the origin sort of an ungrouped batch starts from) is written by
// reasm_prep only; the store jobs are reset by the host right before reasm_serial, the only
// kernel that sets them (a grouped batch with no serial fragment never reads either).
// len | (fragment offset / 8) << 16 | MF << 29 | class << 30 (0 ok, 1 no data, 2 too long)
__device__ __forceinline__ uint32_t rec_meta(const ReasmArgs &a, const FragHdr &h)
{
    const int32_t ip_len = (int32_t)h.tl - 20;                        // l3_len = 20
    const uint32_t ofs = (h.ff & 0x1FFFu) * 8u;
    uint32_t cls = 0, len = 0;
    if (ip_len <= 0) {
        cls = 1;
    } else {
        len = (uint32_t)ip_len;
        if (34u + len > h.flen || ofs + len > a.max_dgram) cls = 2;
    }
    return (cls ? 0u : len) | ((h.ff & 0x1FFFu) << 16) | ((h.ff & 0x2000u) << 16) | (cls << 30);
}

// the key's crc32c signature (ipv4_frag_hash's first hash)
__device__ __forceinline__ uint32_t rec_sig(const uint32_t *crc_tab, const FragHdr &h)
{
    uint32_t v = crc32c_u32(crc_tab, 0xeaad8405u, h.src);
    v = crc32c_u32(crc_tab, v, h.dst);
    return crc32c_u32(crc_tab, v, h.id);
}

__device__ __forceinline__ void prep_record(const ReasmArgs &a, const uint32_t *crc_tab, uint32_t p, uint32_t i,
                                            const FragHdr &h)
{
    a.s_i[p] = i;
    a.s_src[p] = h.src;
    a.s_dst[p] = h.dst;
    a.s_id[p] = h.id;
    a.s_sig[p] = rec_sig(crc_tab, h);
    a.s_meta[p] = rec_meta(a, h);
    a.dv[p] = p;
    a.dk[p] = RS_NONE;                                           // no completion yet
}

__global__ void __launch_bounds__(RS_BLOCK) reasm_prep(ReasmArgs a, uint32_t F)
{
    __shared__ uint32_t crc_tab[256];
    crc_table_init(crc_tab);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    for (uint32_t p = blockIdx.x * RS_BLOCK + threadIdx.x; p < F; p += gridDim.x * RS_BLOCK) {
        const uint32_t i = a.order[p];
        prep_record(a, crc_tab, p, i, frag_hdr(a, fr, i));
    }
}

// The exact half of the run test: a run's first fragment inserts its key's 64-bit fingerprint
// into the per-call set; meeting the same fingerprint again marks the batch not grouped
// (counts[4]).
// The key's slot word and its home slot. Slot word: the call's 16-bit tag above a 48-bit
// fingerprint; a word with another tag is free (left by an earlier call), so the set needs no
// clearing between calls (the host clears it once every 65535 calls, when the tags come round).
__device__ __forceinline__ unsigned long long run_fp(uint32_t id, uint32_t src, uint32_t dst)
{
    unsigned long long fp = ((unsigned long long)dst << 32 | src) * 0x9E3779B97F4A7C15ull;
    fp ^= (unsigned long long)(id + 1u) * 0xC2B2AE3D27D4EB4Full;
    return fp ^ (fp >> 29);
}

// the key's slot in rtab
__device__ __forceinline__ uint32_t run_slot(const ReasmArgs &a, uint32_t id, uint32_t src, uint32_t dst)
{
    return (uint32_t)(run_fp(id, src, dst) >> 32) & a.rmask;
}

__device__ __forceinline__ void run_insert(const ReasmArgs &a, uint32_t id, uint32_t src, uint32_t dst)
{
    {
        unsigned long long *hset = a.hset;
        const uint32_t hmask = a.hmask;
        const unsigned long long fp = run_fp(id, src, dst);
        const unsigned long long val = ((unsigned long long)a.hset_tag << 48) | (fp >> 16);
        uint32_t slot = (uint32_t)fp & hmask, k = 0;
        unsigned long long cur = ld_a(&hset[slot]);
        while (k <= hmask) {
            if ((cur >> 48) != a.hset_tag) {
                const unsigned long long old = atomicCAS(&hset[slot], cur, val);
                if (old == cur) break;                  // claimed
                cur = old;                              // another run won the slot: look at it
                continue;
            }
            if (cur == val) {                           // the key (or its fingerprint) again
                a.counts[4] = 1u;
                break;
            }
            ++k;
            slot = (slot + 1u) & hmask;
            cur = ld_a(&hset[slot]);
        }
    }
}

// A batch that is not grouped: each fragment's key (src, dst, id) to a group, the position of the
// first fragment that claimed the key's slot in gset (insert-or-find; a slot word is the call's
// tag << 48 | 24 fingerprint bits << 24 | position, and a fingerprint match is checked against
// that position's frame header, so the grouping is exact), and the sort key group << ib | index:
// one radix sort then puts every key's fragments together in arrival order (it replaced two, by
// (id, index) then by src | dst: 38 + 64 key bits against 2 ib).
__global__ void __launch_bounds__(RS_BLOCK) reasm_group(ReasmArgs a, uint32_t F)
{
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    const unsigned long long tag = (unsigned long long)a.hset_tag << 48;
    for (uint32_t p = blockIdx.x * RS_BLOCK + threadIdx.x; p < F; p += gridDim.x * RS_BLOCK) {
        const uint32_t o = a.offset[a.frag_list[p]];
        const uint32_t id = ld32(fr, o + 16) >> 16, src = ld32(fr, o + 26), dst = ld32(fr, o + 30);
        const unsigned long long fp = run_fp(id, src, dst);
        const unsigned long long fpb = ((fp >> 40) & 0xFFFFFFull) << 24;
        const unsigned long long val = tag | fpb | p;
        uint32_t slot = (uint32_t)fp & a.hmask, group = p;
        unsigned long long cur = ld_a(&a.gset[slot]);
        for (uint32_t k = 0; k <= a.hmask;) {
            if ((cur >> 48) != a.hset_tag) {
                const unsigned long long old = atomicCAS(&a.gset[slot], cur, val);
                if (old == cur) break;                                  // claimed: a new group
                cur = old;
                continue;
            }
            if ((cur & (0xFFFFFFull << 24)) == fpb) {
                const uint32_t q = (uint32_t)(cur & 0xFFFFFFull);
                const uint32_t oq = a.offset[a.frag_list[q]];
                if ((ld32(fr, oq + 16) >> 16) == id && ld32(fr, oq + 26) == src && ld32(fr, oq + 30) == dst) {
                    group = q;                                         // the key's group
                    break;
                }
            }
            ++k;
            slot = (slot + 1u) & a.hmask;
            cur = ld_a(&a.gset[slot]);
        }
        a.k1[p] = ((unsigned long long)group << a.ib) | p;
    }
}

namespace {

// Orders a wave's LDS accesses across lanes (DS instructions of one wave execute in order).
__device__ __forceinline__ void wave_sync_rs()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Every store this wave issued has completed (CDNA counts stores in vmcnt).
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Exclusive prefix sum of v over the wave's lanes; *total gets the wave's sum. Called with every
// lane active (wave-uniform control flow). On the DPP network: six VALU ops and a readlane, where
// the __shfl_up form made seven ds_bpermute round trips through the LDS pipeline.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total)
{
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
}

// Fresh flow state (ip_frag_reset / ip_frag_tbl_add) for the key.
__device__ __forceinline__ void state_reset(uint32_t *st, uint32_t src, uint32_t dst, uint32_t id,
                                            unsigned long long tms, uint32_t call)
{
    st[E_VALID] = 1;
    st[E_SRC] = src;
    st[E_DST] = dst;
    st[E_ID] = id;
    st[E_FSIZE] = 0;
    st[E_TOTAL] = 0xFFFFFFFFu;
    st[E_LAST] = 2;
    st[E_START] = (uint32_t)tms;
    st[E_START + 1] = (uint32_t)(tms >> 32);
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) { st[E_FR + k] = 0; st[E_WHERE + k] = RS_HELD; }
    st[E_CALL] = call;
}

// ipv4_frag_reassemble's backward chain walk over the held fragments.
__device__ bool chain_ok(const uint32_t *st)
{
    const uint32_t *fr = st + E_FR;
    const uint32_t first_len = fr[0] >> 16;
    const uint32_t n = st[E_LAST] - 1u;
    uint32_t ofs = fr[1] & 0xFFFFu, curr = 1;
    for (uint32_t guard = 0; ofs != first_len && guard < 8; ++guard) {
        const uint32_t prev = curr;
        for (uint32_t i = n; i != 0 && ofs != first_len; i--) {
            if ((fr[i] & 0xFFFFu) + (fr[i] >> 16) == ofs) {
                curr = i;
                ofs = fr[i] & 0xFFFFu;
            }
        }
        if (curr == prev) return false;
    }
    return ofs == first_len;
}

// ip_frag_process of one fragment on flow state st: the fragment goes to slot *idx (FA_KEEP,
// FA_DONE, FA_HOLE, FA_ERR) or to none (FA_NOSLOT: duplicate first/last, more than 4). Every
// outcome but FA_KEEP ends the flow (the entry is invalidated).
enum : uint32_t { FA_KEEP = 0, FA_DONE = 1, FA_HOLE = 2, FA_ERR = 3, FA_NOSLOT = 4 };

__device__ uint32_t frag_apply(uint32_t *st, uint32_t len, uint32_t ofs, uint32_t mf, uint32_t where,
                               uint32_t *idx_out)
{
    uint32_t idx;
    st[E_FSIZE] += len;
    if (ofs == 0) {
        idx = st[E_FR + 0] == 0 ? 0u : RS_NONE;
    } else if (!mf) {
        st[E_TOTAL] = ofs + len;
        idx = st[E_FR + 1] == 0 ? 1u : RS_NONE;
    } else {
        idx = st[E_LAST];
        if (idx < RS_MAX_FRAG) st[E_LAST] = idx + 1u;
    }
    if (idx >= RS_MAX_FRAG) return FA_NOSLOT;
    *idx_out = idx;
    st[E_FR + idx] = ofs | (len << 16);
    st[E_WHERE + idx] = where;
    if (st[E_FSIZE] < st[E_TOTAL]) return FA_KEEP;
    const bool sized = st[E_FSIZE] == st[E_TOTAL] && st[E_FR + 0] != 0;
    if (sized && chain_ok(st)) return FA_DONE;
    return sized ? FA_HOLE : FA_ERR;
}

// Completion record of the flow in st, completed by the fragment at sorted position q (frame i).
__device__ void write_done(const ReasmArgs &a, const uint32_t *st, uint32_t q, uint32_t i, uint32_t entry)
{
    ReasmDone r;
    r.origin = i;
    r.total = st[E_TOTAL];
    r.n = st[E_LAST];
    r.entry = entry;
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
        r.fr[k] = st[E_FR + k];
        r.where[k] = st[E_WHERE + k];
    }
    a.done[q] = r;
    a.dk[q] = i;
}

__device__ __forceinline__ bool same_key(const ReasmArgs &a, uint32_t p, uint32_t q)
{
    return a.s_src[p] == a.s_src[q] && a.s_dst[p] == a.s_dst[q] && a.s_id[p] == a.s_id[q];
}

__device__ __forceinline__ bool seg_start(const ReasmArgs &a, uint32_t p)
{
    return p == 0 || !same_key(a, p, p - 1u);
}

__device__ __forceinline__ uint32_t bucket_of(const ReasmArgs &a, uint32_t sig)
{
    return (sig & a.mask) >> a.assoc_log2;
}

__device__ __forceinline__ uint32_t bucket2_of(const ReasmArgs &a, uint32_t sig)
{
    return (((sig << 7) + (sig >> 14)) & a.mask) >> a.assoc_log2;
}

} // namespace

// Per bucket of the table at call start: valid entries | (an expired valid entry) << 31; the
// bucket's count of complex flows (below) is reset. One lane per entry, assoc lanes per bucket.
__device__ __forceinline__ void bsum_rows(const ReasmArgs &a, uint32_t blk, uint32_t nblk)
{
    const uint32_t lane = __lane_id();
    const uint32_t g0 = lane & ~(a.assoc - 1u);                  // the bucket's first lane
    const unsigned long long gm = (a.assoc == 64u ? ~0ull : ((1ull << a.assoc) - 1ull)) << g0;
    const uint32_t ne = a.nbuckets * a.assoc;
    for (uint32_t x0 = blk * RS_BLOCK + (threadIdx.x & ~63u); x0 < ne; x0 += nblk * RS_BLOCK) {
        const uint32_t x = x0 + lane;
        bool v = false, old = false;
        if (x < ne) {
            const uint32_t *e = a.tab + (size_t)x * E_WORDS;
            v = ld_a(e + E_VALID) != 0;
            if (v) {
                const unsigned long long start =
                    ((unsigned long long)ld_a(e + E_START + 1) << 32) | ld_a(e + E_START);
                old = a.max_cycles + start < a.tms;
            }
        }
        const unsigned long long bv = __ballot(v), bo = __ballot(old);
        if (x < ne && lane == g0) {
            const uint32_t b = x >> a.assoc_log2;
            a.bsum[b] = (uint32_t)__popcll(bv & gm) | ((bo & gm) ? 1u << 31 : 0u);
            a.cplx[b] = 0;
        }
    }
}

// The fragment count per select block (blocks [0, nfs)) and, in the blocks after them, the
// bucket summary (reasm_bsum's rows) and reasm_scan's zeroed chunk counts: one launch at the
// start of a call, the table being unchanged until the flow analysis reads the summary.
__global__ void __launch_bounds__(RS_BLOCK) reasm_fsel_count_bsum(ReasmArgs a, uint32_t *blk, uint32_t nfs)
{
    if (blockIdx.x < nfs) {
        fsel_count_block(a.meta, a.n, blk, a.stats, blockIdx.x);
    } else {
        bsum_rows(a, blockIdx.x - nfs, gridDim.x - nfs);
        const uint32_t cw = 2u * ((a.n + RS_CL - 1u) / RS_CL);     // reasm_scan's chunk counts
        for (uint32_t x = (blockIdx.x - nfs) * RS_BLOCK + threadIdx.x; x < cw; x += (gridDim.x - nfs) * RS_BLOCK)
            a.cblk[x] = 0u;
    }
}

// One thread per flow segment (at its first sorted position p). The flow is walked on its own,
// as if every ip_frag_find it makes succeeded with a fresh entry: its span [tf, tl] (arrival
// indices of its first and last fragment that reaches ip_frag_find) and whether it is still
// pending after its last one. PF_COMPLEX when it is pending, its key is in the table, or one of
// its buckets holds an expired entry; complex flows are counted per bucket. Each flow adds one
// (bucket << ib | tf) record per distinct bucket of its pair for the overlap test. (A grouped
// batch's flows are walked by reasm_scan.)
// F = RS_F_DEV (reasm_ec, reasm_process): a speculative launch of the grouped path, made before
// the host knows F or whether the batch is grouped: F comes from counts[0], and the kernel does
// nothing when reasm_scan found a key in two runs (counts[4]).
constexpr uint32_t RS_F_DEV = 0xFFFFFFFFu;
__device__ __forceinline__ bool spec_f(const ReasmArgs &a, uint32_t &F)
{
    if (F != RS_F_DEV) return true;
    if (a.counts[4]) return false;
    F = a.counts[0];
    return true;
}

__global__ void __launch_bounds__(RS_BLOCK) reasm_flows(ReasmArgs a, uint32_t F)
{
    if (!spec_f(a, F)) return;
    constexpr uint32_t PER = RS_FLOW_CHUNK / RS_BLOCK;
    __shared__ uint32_t s_st[RS_BLOCK][E_WORDS];
    __shared__ unsigned long long s_rk[2 * RS_FLOW_CHUNK];   // the chunk's records, reserved at once
    __shared__ uint32_t s_rv[2 * RS_FLOW_CHUNK];
    __shared__ uint32_t s_nr, s_base, s_nb;
    uint32_t *st = s_st[threadIdx.x];
    const bool limit = a.max_entries < a.entries;
    for (uint32_t c0 = blockIdx.x * RS_FLOW_CHUNK; c0 < F; c0 += gridDim.x * RS_FLOW_CHUNK) {
        if (threadIdx.x == 0) { s_nr = 0; s_nb = 0; }
        __syncthreads();
        for (uint32_t j = 0; j < PER; ++j) {
            const uint32_t p = c0 + j * RS_BLOCK + threadIdx.x;
            uint32_t flag = 0, nrec = 0, bk1 = 0, bk2 = 0, tfirst = RS_NONE;
            if (p < F && seg_start(a, p)) {
                uint32_t tlast = 0;
                bool live = false;
                // the walk reasm_process makes for a flow without the table: its completions
                // are written now (and taken back below if the flow turns out complex) and its
                // outcome counted, so reasm_process only adds them up for such a flow
                uint32_t c_len = 0, c_short = 0, c_done = 0, c_holes = 0, c_err = 0;
                unsigned long long c_bytes = 0;
                for (uint32_t q = p; q < F && (q == p || same_key(a, p, q)); ++q) {
                    const uint32_t m = a.s_meta[q], cls = m >> 30;
                    if (cls) {
                        if (cls == 1) ++c_len;
                        else ++c_short;
                        continue;
                    }
                    const uint32_t i = a.s_i[q];
                    if (tfirst == RS_NONE) tfirst = i;
                    tlast = i;
                    if (!live) state_reset(st, 0, 0, 0, 0, 0);
                    uint32_t idx;
                    const uint32_t r = frag_apply(st, m & 0xFFFFu, ((m >> 16) & 0x1FFFu) * 8u, (m >> 29) & 1u, i, &idx);
                    live = r == FA_KEEP;
                    if (r == FA_DONE) {
                        write_done(a, st, q, i, RS_NONE);
                        ++c_done;
                        c_bytes += (34u + st[E_TOTAL] + 15u) & ~15u;
                    } else if (r == FA_HOLE) {
                        ++c_holes;
                    } else if (r != FA_KEEP) {
                        ++c_err;
                    }
                }
                const bool ovf = (c_len | c_short | c_done | c_holes | c_err) > 62u || c_bytes >= (1ull << 31);
                a.oc[p] = c_len | c_short << 6 | c_done << 12 | c_holes << 18 | c_err << 24 | (ovf ? OC_OVF : 0u);
                a.ob[p] = (uint32_t)c_bytes;
                flag = PF_START;
                if (tfirst != RS_NONE) {
                    flag |= PF_TOUCH | (live ? PF_COMPLEX : 0u);
                    const uint32_t sig = a.s_sig[p];
                    bk1 = bucket_of(a, sig);
                    bk2 = bucket2_of(a, sig);
                    const uint32_t s1 = a.bsum[bk1], s2 = a.bsum[bk2];
                    if ((s1 | s2) >> 31) {
                        flag |= PF_COMPLEX;                       // an expired entry to reclaim
                    } else if ((s1 | s2) & 0xFFFFu) {             // is the key in the table?
                        const uint32_t src = a.s_src[p], dst = a.s_dst[p], id = a.s_id[p];
                        for (uint32_t h = 0; h < 2; ++h) {
                            const uint32_t *e = a.tab + (size_t)(h ? bk2 : bk1) * a.assoc * E_WORDS;
                            for (uint32_t k = 0; k < a.assoc; ++k, e += E_WORDS)
                                if (ld_a(e + E_VALID) && ld_a(e + E_SRC) == src && ld_a(e + E_DST) == dst &&
                                    ld_a(e + E_ID) == id)
                                    flag |= PF_COMPLEX;
                        }
                    }
                    a.sb1[p] = bk1;
                    a.sb2[p] = bk2;
                    a.tf[p] = tfirst;
                    a.tl[p] = tlast;
                    nrec = a.grouped ? 0u : bk1 != bk2 ? 2u : 1u;
                    if (flag & PF_COMPLEX) {
                        atomicAdd(&a.cplx[bk1], 1u);
                        if (bk2 != bk1) atomicAdd(&a.cplx[bk2], 1u);
                        // a complex flow goes through the table: no completion of its own
                        if (c_done)
                            for (uint32_t q = p; q < F && (q == p || same_key(a, p, q)); ++q) a.dk[q] = RS_NONE;
                    }
                }
            }
            if (p < F) a.pflag[p] = flag;
            if (limit) {
                // the flows the max_entries bound counts (reasm_ec): grouped, the complex ones
                // (a simple flow's span holds no other flow's fragment); else every touching one
                const bool cnt = (flag & PF_TOUCH) && (!a.grouped || (flag & PF_COMPLEX));
                const uint32_t nb = (uint32_t)__popcll(__ballot(cnt));
                if (__lane_id() == 0 && nb) atomicAdd(&s_nb, nb);                  // LDS
            }
            uint32_t total;
            const uint32_t off = wave_excl_scan(nrec, &total);
            uint32_t base = 0;
            if (__lane_id() == 0 && total) base = atomicAdd(&s_nr, total);     // LDS
            base = __shfl(base, 0, 64) + off;
            if (nrec) {
                s_rk[base] = ((unsigned long long)bk1 << a.ib) | tfirst;
                s_rv[base] = p;
                if (nrec == 2) {
                    s_rk[base + 1] = ((unsigned long long)bk2 << a.ib) | tfirst;
                    s_rv[base + 1] = p;
                }
            }
        }
        __syncthreads();
        const uint32_t nr = s_nr;
        if (threadIdx.x == 0) s_base = nr ? atomicAdd(&a.counts[1], nr) : 0u;
        if (threadIdx.x == 0 && s_nb) atomicAdd(&a.counts[7], s_nb);
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nr; k += RS_BLOCK) {
            a.rk[s_base + k] = s_rk[k];
            a.rv[s_base + k] = s_rv[k];
        }
        __syncthreads();
    }
}

// Records sorted by (bucket, tf): x = bucket << 32 | tl, whose running maximum gives, per
// record, the latest end among the flows of its bucket that start before it.
__global__ void __launch_bounds__(RS_BLOCK) reasm_rec(ReasmArgs a, const unsigned long long *rks,
                                                      const uint32_t *rvs, unsigned long long *x, uint32_t R)
{
    for (uint32_t k = blockIdx.x * RS_BLOCK + threadIdx.x; k < R; k += gridDim.x * RS_BLOCK)
        x[k] = ((rks[k] >> a.ib) << 32) | a.tl[rvs[k]];
}

// A flow whose span overlaps the span of another flow on a bucket they share is PF_SHARED
// (counted as complex in both its buckets the first time it becomes complex).
__global__ void __launch_bounds__(RS_BLOCK) reasm_overlap(ReasmArgs a, const unsigned long long *rks,
                                                          const uint32_t *rvs, const unsigned long long *xs,
                                                          uint32_t R)
{
    const unsigned long long tmask = (1ull << a.ib) - 1ull;
    for (uint32_t k = blockIdx.x * RS_BLOCK + threadIdx.x; k < R; k += gridDim.x * RS_BLOCK) {
        const unsigned long long key = rks[k];
        const unsigned long long b = key >> a.ib;
        const uint32_t t1 = (uint32_t)(key & tmask), p = rvs[k], t2 = a.tl[p];
        bool ov = k > 0 && (xs[k - 1] >> 32) == b && (uint32_t)xs[k - 1] >= t1;
        ov = ov || (k + 1 < R && (rks[k + 1] >> a.ib) == b && (uint32_t)(rks[k + 1] & tmask) <= t2);
        if (ov) {
            const uint32_t old = atomicOr(&a.pflag[p], PF_SHARED);
            if (!(old & (PF_COMPLEX | PF_SHARED))) {
                atomicAdd(&a.cplx[a.sb1[p]], 1u);
                if (a.sb2[p] != a.sb1[p]) atomicAdd(&a.cplx[a.sb2[p]], 1u);
            }
        }
    }
}

// A flow that is neither complex nor shared runs without the table only if its ip_frag_find is
// sure to find a free entry: its buckets' free entries at call start minus the complex flows
// that could hold one of them. Otherwise every flow of the batch takes the serial path.
__device__ __forceinline__ void ec_block(const ReasmArgs &a, uint32_t F, uint32_t blk, uint32_t nblk)
{
    __shared__ unsigned long long s_sum[RS_WAVES][RS_PB];
    __shared__ uint32_t s_quick;
    if (!spec_f(a, F)) return;
    // ip_frag_find's max_entries test (rte_ip_frag_table_create's max_entries, NUM_FLOWS_MAX in
    // the reference): before any add in the call, use_entries <= the entries valid at call start
    // + the entries this call's earlier flows still hold. Grouped, a simple flow's span holds no
    // other flow's fragment, so that is at most the complex flows; otherwise at most the other
    // touching flows. When the bound cannot stay below max_entries, the whole batch takes the
    // serial path, which applies the test (and the LRU deletion) exactly.
    if (blk == 0 && threadIdx.x == 0 && a.max_entries < a.entries) {
        const uint64_t c = (uint64_t)a.counts[7] + (a.grouped ? 1u : 0u);
        if ((uint64_t)ld_a(a.tab_used) + c > a.max_entries) {
            a.counts[3] = 1u;
            a.counts[6] = 1u;
        }
    }
    // Grouped with no complex flow: no entry is held by another flow of the call, and reasm_scan
    // made the free-entry test (with no complex counts) for every simple flow. With no fallback
    // either, every flow runs without the table and reasm_scan has the call's outcome: workgroup 0
    // adds up its per-block totals, and reasm_process is not launched (the host launches it after
    // the read-back otherwise; the words added here are cleared if the batch is not grouped).
    const bool quick = a.grouped && a.counts[8] == 0u;
    if (blk == 0 && quick) {
        if (threadIdx.x == 0) s_quick = a.counts[3] == 0u;       // after the max_entries test above
        __syncthreads();
        if (s_quick) {
            const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
            unsigned long long v[RS_PB] = {0, 0, 0, 0, 0, 0};
            for (uint32_t x = threadIdx.x; x < (F + RS_CL - 1u) / RS_CL; x += RS_BLOCK)
#pragma unroll
                for (uint32_t k = 0; k < RS_PB; ++k) v[k] += a.pblk[(size_t)x * RS_PB + k];
#pragma unroll
            for (uint32_t k = 0; k < RS_PB; ++k) {
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) v[k] += __shfl_xor(v[k], d, 64);
                if (lane == 0) s_sum[w][k] = v[k];
            }
            __syncthreads();
            if (threadIdx.x < RS_PB) {
                unsigned long long t = 0;
#pragma unroll
                for (uint32_t i = 0; i < RS_WAVES; ++i) t += s_sum[i][threadIdx.x];
                constexpr uint32_t word[RS_PB] = {UDPDK_RS_DROP_LEN, UDPDK_RS_DROP_SHORT, UDPDK_RS_DONE,
                                                  UDPDK_RS_HOLES, UDPDK_RS_ERRORS, UDPDK_RS_N};
                if (t) atomicAdd(&a.stats[word[threadIdx.x]], t);        // [UDPDK_RS_N]: out_bytes
            }
        }
    }
    for (uint32_t p = blk * RS_BLOCK + threadIdx.x; p < F; p += nblk * RS_BLOCK) {
        const uint32_t f = a.pflag[p];
        if (a.grouped && (f & PF_START)) {
            // The run test's second half: a run that finds its own position in its key's slot, or
            // another run's of the same key (then the batch is not grouped), is done; one that
            // lost the slot to another key goes into the exact set. Two runs of one key meet:
            // one of them holds their common slot, or another key holds it and both are in the set.
            const uint32_t src = a.s_src[p], dst = a.s_dst[p], id = a.s_id[p];
            const uint32_t w = a.rtab[run_slot(a, id, src, dst)];
            if (w != p) {
                if (a.s_src[w] == src && a.s_dst[w] == dst && a.s_id[w] == id) a.counts[4] = 1u;
                else run_insert(a, id, src, dst);
            }
        }
        if (quick || !(f & PF_TOUCH) || (f & (PF_COMPLEX | PF_SHARED))) continue;
        const uint32_t b1 = a.sb1[p], b2 = a.sb2[p];
        int32_t fr = (int32_t)a.assoc - (int32_t)(a.bsum[b1] & 0xFFFFu) - (int32_t)a.cplx[b1];
        if (b2 != b1) fr += (int32_t)a.assoc - (int32_t)(a.bsum[b2] & 0xFFFFu) - (int32_t)a.cplx[b2];
        if (fr < 1) a.counts[3] = 1u;
    }
}

__global__ void __launch_bounds__(RS_BLOCK) reasm_ec(ReasmArgs a, uint32_t F)
{
    ec_block(a, F, blockIdx.x, gridDim.x);
}

// One thread per flow segment. A flow that cannot see or be seen by another flow (not complex,
// not shared, and no fallback) is reassembled here on its own state, never touching the table:
// a reference that processes the batch one fragment at a time gives it a free entry at its
// first fragment and frees it at its last, with no other lookup in its buckets in between.
// Every other flow's fragments that reach ip_frag_find go to the serial list (arrival index,
// sorted position). Length-class drops are counted for every flow.
__global__ void __launch_bounds__(RS_BLOCK) reasm_process(ReasmArgs a, uint32_t F)
{
    if (!spec_f(a, F)) return;
    __shared__ uint32_t s_st[RS_BLOCK][E_WORDS];
    __shared__ unsigned long long s_cnt[UDPDK_RS_N + 1];    // block totals: stats, out bytes
    uint32_t *st = s_st[threadIdx.x];
    if (threadIdx.x <= UDPDK_RS_N) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const bool fallback = a.counts[3] != 0;
    const uint32_t step = gridDim.x * RS_BLOCK;
    unsigned long long c_len = 0, c_short = 0, c_done = 0, c_holes = 0, c_err = 0, c_bytes = 0;
    // The wave's positions are taken PF grid strides at a time with every flag and outcome word of
    // the batch loaded at once (clamped indices, unconditional): the per-position loads were one
    // dependent round trip per grid stride (8 strides per wave at 512 K fragments).
    constexpr uint32_t PF = 8;
    const uint32_t fl = F ? F - 1u : 0u;
    for (uint32_t pb = blockIdx.x * RS_BLOCK + (threadIdx.x & ~63u); pb < F; pb += step * PF) {
        uint32_t fv[PF], ocv[PF], obv[PF];
#pragma unroll
        for (uint32_t it = 0; it < PF; ++it) {
            const uint32_t p = pb + it * step + __lane_id();
            fv[it] = p < F ? a.pflag[min(p, fl)] : 0u;
            ocv[it] = a.oc[min(p, fl)];
            obv[it] = a.ob[min(p, fl)];
        }
#pragma unroll 1
        for (uint32_t it = 0; it < PF; ++it) {
            const uint32_t p0 = pb + it * step;
            if (p0 >= F) break;                                      // wave-uniform
            const uint32_t p = p0 + __lane_id();
            uint32_t nser = 0;
            bool serial = false;
            const uint32_t f = fv[it];
            const uint32_t oc = (f & PF_START) ? ocv[it] : 0u;
            serial = (f & PF_TOUCH) && (fallback || (f & (PF_COMPLEX | PF_SHARED)));
            if ((f & PF_START) && !serial && !(oc & OC_OVF)) {
                // reasm_flows walked this flow on its own and wrote its completions: add up
                c_len += oc & 63u;
                c_short += (oc >> 6) & 63u;
                c_done += (oc >> 12) & 63u;
                c_holes += (oc >> 18) & 63u;
                c_err += (oc >> 24) & 63u;
                c_bytes += obv[it];
            } else if (f & PF_START) {
                bool live = false;
                for (uint32_t q = p; q < F && (q == p || same_key(a, p, q)); ++q) {
                    const uint32_t m = a.s_meta[q], cls = m >> 30;
                    if (cls) {
                        if (cls == 1) ++c_len;
                        else ++c_short;
                        continue;
                    }
                    if (serial) {
                        ++nser;
                        a.dk[q] = RS_NONE;                 // reasm_flows' completion, if any, is void
                        continue;
                    }
                    const uint32_t i = a.s_i[q];
                    if (!live) state_reset(st, 0, 0, 0, 0, 0);
                    uint32_t idx;
                    const uint32_t r = frag_apply(st, m & 0xFFFFu, ((m >> 16) & 0x1FFFu) * 8u, (m >> 29) & 1u, i, &idx);
                    live = r == FA_KEEP;
                    if (r == FA_DONE) {
                        write_done(a, st, q, i, RS_NONE);
                        ++c_done;
                        c_bytes += (34u + st[E_TOTAL] + 15u) & ~15u;
                    } else if (r == FA_HOLE) {
                        ++c_holes;
                    } else if (r != FA_KEEP) {
                        ++c_err;
                    }
                }
            }
            uint32_t total;
            const uint32_t off = wave_excl_scan(nser, &total);
            uint32_t base = 0;
            if (__lane_id() == 0 && total) base = atomicAdd(&a.counts[2], total);
            base = __shfl(base, 0, 64) + off;
            if (nser) {
                for (uint32_t q = p; q < F && (q == p || same_key(a, p, q)); ++q) {
                    if (a.s_meta[q] >> 30) continue;
                    a.sl_k[base] = a.s_i[q];
                    a.sl_v[base] = q;
                    ++base;
                }
            }
        }
    }
    if (c_len) atomicAdd(&s_cnt[UDPDK_RS_DROP_LEN], c_len);
    if (c_short) atomicAdd(&s_cnt[UDPDK_RS_DROP_SHORT], c_short);
    if (c_done) atomicAdd(&s_cnt[UDPDK_RS_DONE], c_done);
    if (c_holes) atomicAdd(&s_cnt[UDPDK_RS_HOLES], c_holes);
    if (c_err) atomicAdd(&s_cnt[UDPDK_RS_ERRORS], c_err);
    if (c_bytes) atomicAdd(&s_cnt[UDPDK_RS_N], c_bytes);
    __syncthreads();
    if (threadIdx.x < UDPDK_RS_N && s_cnt[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], s_cnt[threadIdx.x]);
    if (threadIdx.x == UDPDK_RS_N && s_cnt[UDPDK_RS_N]) atomicAdd(a.out_bytes, s_cnt[UDPDK_RS_N]);
}

// TAILQ_FIRST(&tbl->lru): the valid entry with the smallest (E_LRU_CALL, E_LRU_IDX). The wave keeps
// one minimum per lane, over the entries x with x % 64 == lane (its partition), built by one scan
// of the table (eight entries per lane in flight per round) the first time a call needs the head.
// A lane's minimum goes stale in two ways. (1) The entry it names is invalidated or moved to the
// list's tail: the head is the smallest cached minimum once that one is checked against its
// entry, and a stale one costs a scan of its own partition (entries / 64, spread over the wave),
// not of the table. (2) An entry is inserted into a partition whose cache holds a larger key or
// none (~0: empty when scanned): the cache then misses it. Such an entry was created in this call
// (a new key is larger than every key already in the table), so its start is this call's time
// and it cannot be the expired head ip_frag_find would evict; nor can it be the head ahead of an
// older cached entry. So the head found this way is the true head whenever an eviction needs it;
// a rule that could evict an entry of the current call would have to refresh the cache on insert.
struct LruMin {
    unsigned long long key;                  // this lane's partition minimum, ~0 when none
    uint32_t idx;
};

__device__ __forceinline__ unsigned long long lru_key(const ReasmArgs &a, uint32_t x, bool *valid)
{
    const uint32_t *e = a.tab + (size_t)x * E_WORDS;
    *valid = ld_a(e + E_VALID) != 0;
    return ((unsigned long long)ld_a(e + E_LRU_CALL) << 32) | ld_a(e + E_LRU_IDX);
}

__device__ LruMin lru_scan_all(const ReasmArgs &a)
{
    const uint32_t lane = __lane_id();
    LruMin m{~0ull, RS_NONE};
    for (uint32_t x0 = 0; x0 < a.entries; x0 += 512u) {
        uint32_t v[8], hi[8], lo[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t x = x0 + 64u * u + lane;
            const uint32_t *e = a.tab + (size_t)min(x, a.entries - 1u) * E_WORDS;
            v[u] = x < a.entries ? ld_a(e + E_VALID) : 0u;
            hi[u] = ld_a(e + E_LRU_CALL);
            lo[u] = ld_a(e + E_LRU_IDX);
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const unsigned long long key = ((unsigned long long)hi[u] << 32) | lo[u];
            if (v[u] && key < m.key) {
                m.key = key;
                m.idx = x0 + 64u * u + lane;
            }
        }
    }
    return m;
}

// the minimum of partition `part` (entries part, part + 64, ...), by the whole wave; wave-uniform
__device__ LruMin lru_scan_part(const ReasmArgs &a, uint32_t part)
{
    const uint32_t lane = __lane_id();
    unsigned long long best = ~0ull;
    uint32_t bi = RS_NONE;
    for (uint32_t x = part + 64u * lane; x < a.entries; x += 64u * 64u) {
        bool v;
        const unsigned long long key = lru_key(a, x, &v);
        if (v && key < best) {
            best = key;
            bi = x;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long ob = __shfl_xor(best, d, 64);
        const uint32_t oi = __shfl_xor(bi, d, 64);
        if (ob < best || (ob == best && oi < bi)) {
            best = ob;
            bi = oi;
        }
    }
    return LruMin{best, bi};
}

// The head from the lanes' cached minima (refreshing the stale ones it meets); RS_NONE when the
// table is empty. Wave-uniform.
__device__ uint32_t lru_head(const ReasmArgs &a, LruMin &mine)
{
    const uint32_t lane = __lane_id();
    for (;;) {
        unsigned long long best = mine.key;
        uint32_t bi = mine.idx, owner = lane;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const unsigned long long ob = __shfl_xor(best, d, 64);
            const uint32_t oi = __shfl_xor(bi, d, 64), oo = __shfl_xor(owner, d, 64);
            if (ob < best || (ob == best && oi < bi)) {
                best = ob;
                bi = oi;
                owner = oo;
            }
        }
        if (bi == RS_NONE) return RS_NONE;
        bool v;
        const unsigned long long key = lru_key(a, bi, &v);
        if (v && key == best) return bi;
        const LruMin fresh = lru_scan_part(a, owner);      // that partition's minimum had gone
        if (lane == owner) mine = fresh;
    }
}

// The serial path: one wave takes the listed fragments in arrival order, exactly as the
// reference's per-fragment rte_ipv4_frag_reassemble_packet does: ip_frag_find (the lanes load the
// key's 2 x assoc candidate entries at once; match, else the first expired, else the first free
// entry in ip_frag_lookup's order, the free one subject to the max_entries test when counts[6]
// says the call needs it), ip_frag_process on the entry's words in LDS, write-back or
// invalidation. It is the only writer of the table while it runs, and keeps its count of valid
// entries (use_entries) across calls. A fragment that stays in a pending entry gets a store job;
// a flow that ends later in the call cancels its jobs.
// comp != nullptr (the max_entries test not in play): workgroup b of the launch takes the listed
// fragments whose bucket component (reasm_cc) maps to it, in arrival order. Components share no
// bucket, so their fragments commute: each one's table operations are exactly the reference's
// sequence for its fragments, and the waves run side by side.
__device__ __forceinline__ uint32_t cc_owner(uint32_t root, uint32_t nw)
{
    return (uint32_t)(((unsigned long long)(root * 0x9E3779B1u) * nw) >> 32);
}

__global__ void __launch_bounds__(64) reasm_serial(ReasmArgs a, const uint32_t *list, uint32_t K,
                                                   const uint32_t *comp)
{
    __shared__ uint32_t st[E_WORDS];
    const uint32_t lane = __lane_id();
    unsigned long long c_ns = 0, c_err = 0, c_holes = 0, c_exp = 0, c_done = 0, c_bytes = 0;
    long long c_stored = 0;
    const uint32_t nslot = 2u * a.assoc;
    const bool limit = comp == nullptr && a.counts[6] != 0u;
    const uint32_t use0 = ld_a(a.tab_used);
    uint32_t use = use0;
    uint32_t head = RS_NONE;                 // the LRU head, while head_ok
    bool head_ok = false, lru_built = false;
    LruMin lru{~0ull, RS_NONE};              // this lane's partition minimum (lru_head)
    unsigned long long mine = 0;             // comp: this workgroup's entries of the current 64
    for (uint32_t k = 0; k < K; ++k) {
        if (comp) {
            if ((k & 63u) == 0u) {
                const uint32_t kk = k + lane;
                mine = __ballot(kk < K && cc_owner(comp[kk], gridDim.x) == blockIdx.x);
            }
            if (!((mine >> (k & 63u)) & 1ull)) continue;
        }
        const uint32_t q = list[k];
        const uint32_t i = a.s_i[q], m = a.s_meta[q];
        const uint32_t src = a.s_src[q], dst = a.s_dst[q], id = a.s_id[q], sig = a.s_sig[q];
        const uint32_t p1 = sig & a.mask, p2 = ((sig << 7) + (sig >> 14)) & a.mask;
        // lanes scan p1[0], p2[0], p1[1], p2[1], ... (ip_frag_lookup's order), whole entries
        const uint32_t slot = (lane & 1u ? p2 : p1) + (lane >> 1);
        uint32_t w[E_WORDS];
        bool match = false, empty = false, stale = false;
        if (lane < nslot) {
            const uint32_t *e = a.tab + (size_t)slot * E_WORDS;
#pragma unroll
            for (uint32_t j = 0; j < E_WORDS; ++j) w[j] = ld_a(e + j);
            const unsigned long long start = ((unsigned long long)w[E_START + 1] << 32) | w[E_START];
            match = w[E_VALID] && w[E_SRC] == src && w[E_DST] == dst && w[E_ID] == id;
            stale = w[E_VALID] && !match && a.max_cycles + start < a.tms;
            empty = !w[E_VALID];
        }
        const unsigned long long mm = __ballot(match), ms = __ballot(stale), me = __ballot(empty);
        const unsigned long long pick = mm ? mm : ms ? ms : me;
        if (!pick) {
            ++c_ns;                                          // ip_frag_find: no space
            continue;
        }
        if (limit && !mm && !ms && use >= a.max_entries) {
            // a free entry, but max_entries in use: the LRU head goes if it has expired, else
            // the fragment is dropped (ip_frag_find's fail_nospace)
            if (!head_ok) {
                if (!lru_built) {
                    lru = lru_scan_all(a);
                    lru_built = true;
                }
                head = lru_head(a, lru);
                head_ok = true;
            }
            bool del = false;
            if (head != RS_NONE) {
                const uint32_t *he = a.tab + (size_t)head * E_WORDS;
                const unsigned long long hs = ((unsigned long long)ld_a(he + E_START + 1) << 32) | ld_a(he + E_START);
                del = a.max_cycles + hs < a.tms;
            }
            if (!del) {
                ++c_ns;
                continue;
            }
            if (lane == 0) {                                 // ip_frag_tbl_del(lru)
                ++c_exp;
                uint32_t *he = a.tab + (size_t)head * E_WORDS;
                // (this call's fragments of an expired entry cannot exist: a fragment that
                // reached it this call would have restarted it; kept for the invariant)
                if (ld_a(he + E_CALL) == a.call)
                    for (uint32_t j = 0; j < RS_MAX_FRAG; ++j)
                        if (ld_a(he + E_FR + j) && ld_a(he + E_WHERE + j) != RS_HELD) {
                            a.jobs[a.tpos[(size_t)head * RS_MAX_FRAG + j]].frame = RS_NONE;
                            --c_stored;
                        }
                st_a(he + E_VALID, 0u);
            }
            --use;
            head_ok = false;
            stores_done();
            wave_sync_rs();
        }
        const uint32_t cl = (uint32_t)__ffsll((long long)pick) - 1u;
        const uint32_t cand = __shfl(slot, cl, 64);
        if (lane == cl) {
#pragma unroll
            for (uint32_t j = 0; j < E_WORDS; ++j) st[j] = w[j];
        }
        wave_sync_rs();
        uint32_t inval = 0, moved = 0;
        if (lane == 0) {
            bool fresh = !mm;                                // ip_frag_tbl_add (after del if stale)
            if (ms && !mm) ++c_exp;
            if (mm && a.max_cycles + (((unsigned long long)st[E_START + 1] << 32) | st[E_START]) < a.tms) {
                ++c_exp;                                     // ip_frag_tbl_reuse
                fresh = true;
            }
            if (fresh) {
                state_reset(st, src, dst, id, a.tms, a.call);
                st[E_LRU_CALL] = a.call;                     // to the LRU list's tail
                st[E_LRU_IDX] = i;
                moved = 1;
            } else if (st[E_CALL] != a.call) {               // fragments of earlier calls are held
                for (uint32_t j = 0; j < RS_MAX_FRAG; ++j) st[E_WHERE + j] = RS_HELD;
                st[E_CALL] = a.call;
            }
            uint32_t idx = RS_NONE;
            const uint32_t r = frag_apply(st, m & 0xFFFFu, ((m >> 16) & 0x1FFFu) * 8u, (m >> 29) & 1u, i, &idx);
            uint32_t *tp = a.tpos + (size_t)cand * RS_MAX_FRAG;
            if (r == FA_KEEP) {
                tp[idx] = q;
                ReasmJob jb;
                jb.frame = i;
                jb.entry = cand;
                jb.fr = st[E_FR + idx];
                jb.pad = 0;
                a.jobs[q] = jb;
                ++c_stored;
            } else {
                if (r == FA_DONE) {
                    write_done(a, st, q, i, cand);
                    ++c_done;
                    c_bytes += (34u + st[E_TOTAL] + 15u) & ~15u;
                } else if (r == FA_HOLE) {
                    ++c_holes;
                } else {
                    ++c_err;
                }
                // the flow ends: this call's fragments it held no longer go to the table
                for (uint32_t j = 0; j < RS_MAX_FRAG; ++j) {
                    if (j == idx || !st[E_FR + j] || st[E_WHERE + j] == RS_HELD) continue;
                    a.jobs[tp[j]].frame = RS_NONE;
                    --c_stored;
                }
                inval = 1;
            }
        }
        wave_sync_rs();
        inval = __shfl(inval, 0, 64);
        moved = __shfl(moved, 0, 64);
        if (!mm && !ms) ++use;                               // an empty entry taken
        if (inval) --use;
        if (head_ok && cand == head && (inval || moved)) head_ok = false;
        uint32_t *e = a.tab + (size_t)cand * E_WORDS;
        if (inval) {
            if (lane == 0) st_a(e + E_VALID, 0u);
        } else if (lane < E_WORDS) {
            st_a(e + lane, st[lane]);
        }
        stores_done();
        wave_sync_rs();
    }
    if (lane == 0) {
        if (comp) atomicAdd(a.tab_used, use - use0);     // (wraps for a net release)
        else st_a(a.tab_used, use);
    }
    if (lane == 0) {
        unsigned long long *s = a.stats;
        if (c_ns) atomicAdd(&s[UDPDK_RS_NO_SPACE], c_ns);
        if (c_err) atomicAdd(&s[UDPDK_RS_ERRORS], c_err);
        if (c_holes) atomicAdd(&s[UDPDK_RS_HOLES], c_holes);
        if (c_exp) atomicAdd(&s[UDPDK_RS_EXPIRED], c_exp);
        if (c_done) atomicAdd(&s[UDPDK_RS_DONE], c_done);
        if (c_stored) atomicAdd(&s[UDPDK_RS_STORED], (unsigned long long)c_stored);
        if (c_bytes) atomicAdd(a.out_bytes, c_bytes);
    }
}

// The serial fragments' bucket components: union-find over the buckets in LDS (one workgroup,
// tables of up to RS_CC_MAX buckets), each listed fragment joining its key's two buckets; comp[k]
// = the root of list entry k's first bucket.
constexpr uint32_t RS_CC_MAX = 16384;
constexpr uint32_t RS_CC_BLOCK = 1024;

__global__ void __launch_bounds__(RS_CC_BLOCK) reasm_cc(ReasmArgs a, const uint32_t *list, uint32_t K, uint32_t *comp)
{
    __shared__ uint32_t par[RS_CC_MAX];
    for (uint32_t b = threadIdx.x; b < a.nbuckets; b += RS_CC_BLOCK) par[b] = b;
    __syncthreads();
    auto find = [&](uint32_t x) {
        for (;;) {
            const uint32_t p = __hip_atomic_load(&par[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (p == x) return x;
            const uint32_t g = __hip_atomic_load(&par[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (g != p) atomicCAS(&par[x], p, g);                     // path halving
            x = p;
        }
    };
    for (uint32_t k = threadIdx.x; k < K; k += RS_CC_BLOCK) {
        const uint32_t sig = a.s_sig[list[k]];
        uint32_t x = bucket_of(a, sig), y = bucket2_of(a, sig);
        for (;;) {
            x = find(x);
            y = find(y);
            if (x == y) break;
            if (x < y) { const uint32_t t = x; x = y; y = t; }         // the larger root under the smaller
            if (atomicCAS(&par[x], x, y) == x) break;
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < K; k += RS_CC_BLOCK) comp[k] = find(bucket_of(a, a.s_sig[list[k]]));
}


// Grouped path: the completions in position (= arrival) order and their output offsets in two
// launches (per RS_CL-position block: count and bytes; then each block's base from its
// predecessors' totals and a block scan), instead of a rocPRIM select, a size pass and a rocPRIM
// scan (three passes, six launches with the scans' state initialisation). The speculative tail
// takes the counts reasm_scan made and runs reasm_clist_write beside reasm_ec (reasm_ec_clist).

// The grouped path's tail (completion list and offsets beside reasm_ec, then the emit) launched
// before the host has read the call's counts back (counts == nullptr: an ordinary launch). It runs
// only when the batch was grouped, no flow went through the table (so no fragment is held or
// stored, and every datagram's bytes are in the batch) and the output fits the buffer; F and
// the completion count then come from the device. The host re-derives the same decision from the
// read-back and runs the tail itself otherwise, so a grouped batch makes one host round trip.
struct SpecTail {
    const uint32_t *counts;                      // ReasmArgs::counts
    const unsigned long long *stats;             // [UDPDK_RS_DONE] completions, [UDPDK_RS_N] bytes
    unsigned long long out_cap;
    // in place (udpdk_gpu_rx_reassemble_inplace): reasm_scan checks every completion's fragments
    // (back to back in the frame buffer, in data order, no padding) and raises refuse (counts[5])
    // for one that is not; reasm_emit_either then moves in place if none did, and copies if one did
    uint32_t inplace;
    uint32_t *refuse;
};

// Waves per SIMD of the emit launches (the in-place emit loads the next datagram's header dwords
// with its bytes: loaded in their own step instead, 8 VGPRs fewer, measured slower).
#ifndef UDPDK_RS_EMIT_WPE
#define UDPDK_RS_EMIT_WPE 7
#endif

// A load through the constant address space: with a wave-uniform address it is a scalar load
// (s_load, counted by lgkmcnt), so waiting for it does not wait for the wave's older vector
// stores, which vmcnt counts in order with vector loads. For data no launch writes while it runs
// (the completion records, their order, the batch's descriptors).
template <typename T>
__device__ __forceinline__ T cload(const T *p)
{
#if __HIP_DEVICE_COMPILE__
    return *(const __attribute__((address_space(4))) T *)(uintptr_t)p;
#else
    return *p;                                   // (host pass: never called)
#endif
}

// x[i] for a runtime i without indexing a register array (which would go to scratch)
__device__ __forceinline__ uint32_t pick4(const uint32_t (&x)[RS_MAX_FRAG], uint32_t i)
{
    return i == 0u ? x[0] : i == 1u ? x[1] : i == 2u ? x[2] : x[3];
}

// The fragments of completion r in data order (slot 0 holds offset 0; the others sorted by
// offset): their number; sl[] the slots. Wave-uniform (r is).
__device__ __forceinline__ uint32_t data_order(const ReasmDone &r, uint32_t (&sl)[RS_MAX_FRAG])
{
    // rank of every used slot among the used ones by data offset (slot 0 holds offset 0), then
    // sl[rank] = slot: compare-and-count with static indices only (no private-memory arrays)
    uint32_t m = 0;
    bool use[RS_MAX_FRAG];
#pragma unroll
    for (uint32_t q = 0; q < RS_MAX_FRAG; ++q) {
        use[q] = q < r.n && r.fr[q] != 0u;
        m += use[q] ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < RS_MAX_FRAG; ++i) sl[i] = 0u;
#pragma unroll
    for (uint32_t q = 0; q < RS_MAX_FRAG; ++q) {
        uint32_t rank = 0;
#pragma unroll
        for (uint32_t p = 0; p < RS_MAX_FRAG; ++p)
            rank += use[p] && p != q &&
                    ((r.fr[p] & 0xFFFFu) < (r.fr[q] & 0xFFFFu) || ((r.fr[p] & 0xFFFFu) == (r.fr[q] & 0xFFFFu) && p < q)) ? 1u : 0u;
#pragma unroll
        for (uint32_t i = 0; i < RS_MAX_FRAG; ++i)
            if (use[q] && rank == i) sl[i] = q;
    }
    return m;
}

__device__ __forceinline__ bool spec_tail_go(const SpecTail &g, uint32_t &F, uint32_t &C)
{
    if (!g.counts) return true;
    // grouped, no flow through the table (reasm_ec's quick case: counts[2] stays 0 until a later
    // reasm_process), every completion counted by reasm_scan
    if (g.counts[4] || g.counts[8] || g.counts[3] || g.counts[9]) return false;
    const unsigned long long c = g.stats[UDPDK_RS_DONE];
    if (!c) return false;
    F = g.counts[0];
    C = (uint32_t)c;
    return true;
}

// the copying emit of a speculative tail: the output must fit the buffer it was launched with
__device__ __forceinline__ bool spec_copy_fits(const SpecTail &g)
{
    return !g.counts || g.stats[UDPDK_RS_N] + UDPDK_GPU_FRAMES_TAILROOM <= g.out_cap;
}

__device__ __forceinline__ uint32_t done_bytes(const ReasmDone *done, uint32_t q)
{
    return (34u + done[q].total + 15u) & ~15u;    // the output frame's 16-byte aligned size
}

// by_origin: dk is indexed by origin (a completion's arrival index, the position of its record
// as the value, ~0 for none), so the list comes out in origin order (a batch that is not grouped)
__global__ void __launch_bounds__(RS_BLOCK) reasm_clist_count(const uint32_t *dk, const ReasmDone *done,
                                                             uint32_t F, uint32_t *blk, SpecTail g, uint32_t by_origin)
{
    __shared__ uint32_t red[2 * RS_WAVES];
    uint32_t C_unused;
    if (!spec_tail_go(g, F, C_unused) || blockIdx.x * RS_CL >= F) return;
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    const uint32_t p0 = blockIdx.x * RS_CL + tid * (RS_CL / RS_BLOCK);
    uint32_t c = 0, by = 0;
#pragma unroll
    for (uint32_t j = 0; j < RS_CL / RS_BLOCK; ++j) {
        const uint32_t q = p0 + j;
        if (q < F && dk[q] != RS_NONE) {
            ++c;
            by += done_bytes(done, by_origin ? dk[q] : q);
        }
    }
    uint32_t tc, tb;
    (void)wave_excl_scan(c, &tc);
    (void)wave_excl_scan(by, &tb);
    if (lane == 0) { red[w] = tc; red[RS_WAVES + w] = tb; }
    __syncthreads();
    if (tid == 0) {
        uint32_t sc = 0, sb = 0;
        for (uint32_t i = 0; i < RS_WAVES; ++i) { sc += red[i]; sb += red[RS_WAVES + i]; }
        blk[2 * blockIdx.x] = sc;
        blk[2 * blockIdx.x + 1] = sb;
    }
}

__device__ __forceinline__ void clist_write_block(const uint32_t *dk, const ReasmDone *done, uint32_t F,
                                                  const uint32_t *blk, uint32_t *perm, uint32_t *offs,
                                                  const SpecTail &g, uint32_t b, bool in_ec, bool by_origin = false)
{
    __shared__ uint32_t red[4 * RS_WAVES];
    uint32_t C_unused;
    if (in_ec) {
        // beside reasm_ec, which may still set counts[3], [4] and the outcome words: only
        // reasm_scan's verdicts are final here (the emit checks the rest)
        if (g.counts[8] || g.counts[9]) return;
        F = g.counts[0];
    } else if (!spec_tail_go(g, F, C_unused)) {
        return;
    }
    if (b * RS_CL >= F) return;
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    // this block's base: the earlier blocks' totals
    uint32_t pc = 0, pb = 0;
    for (uint32_t i = tid; i < b; i += RS_BLOCK) { pc += blk[2 * i]; pb += blk[2 * i + 1]; }
    uint32_t t0, t1;
    (void)wave_excl_scan(pc, &t0);
    (void)wave_excl_scan(pb, &t1);
    // the thread's positions, then a block scan of their counts and bytes
    constexpr uint32_t PT = RS_CL / RS_BLOCK;
    const uint32_t p0 = b * RS_CL + tid * PT;
    uint32_t c = 0, by = 0, sz[PT], at[PT];
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
        const uint32_t q = p0 + j;
        const uint32_t d = q < F ? dk[q] : RS_NONE;
        at[j] = by_origin ? d : q;                          // the completion record's position
        sz[j] = d != RS_NONE ? done_bytes(done, at[j]) : 0u;
        c += sz[j] ? 1u : 0u;
        by += sz[j];
    }
    uint32_t wc, wb;
    uint32_t ec = wave_excl_scan(c, &wc), eb = wave_excl_scan(by, &wb);
    if (lane == 0) { red[w] = wc; red[RS_WAVES + w] = wb; red[2 * RS_WAVES + w] = t0; red[3 * RS_WAVES + w] = t1; }
    __syncthreads();
    uint32_t bc = 0, bb = 0;
#pragma unroll
    for (uint32_t i = 0; i < RS_WAVES; ++i) {
        bc += red[2 * RS_WAVES + i] + (i < w ? red[i] : 0u);
        bb += red[3 * RS_WAVES + i] + (i < w ? red[RS_WAVES + i] : 0u);
    }
    ec += bc;
    eb += bb;
#pragma unroll
    for (uint32_t j = 0; j < PT; ++j) {
        if (sz[j]) {
            perm[ec] = at[j];
            offs[ec] = eb;
            ++ec;
            eb += sz[j];
        }
    }
}

__global__ void __launch_bounds__(RS_BLOCK) reasm_clist_write(const uint32_t *dk, const ReasmDone *done,
                                                             uint32_t F, const uint32_t *blk,
                                                             uint32_t *perm, uint32_t *offs, SpecTail g,
                                                             uint32_t by_origin)
{
    clist_write_block(dk, done, F, blk, perm, offs, g, blockIdx.x, false, by_origin != 0u);
}

// Each completion's record position at its origin (unique: a frame completes one datagram at
// most), for the origin-ordered list of a batch that is not grouped.
__global__ void __launch_bounds__(RS_BLOCK) reasm_by_origin(const uint32_t *dk, uint32_t F, uint32_t *slot)
{
    for (uint32_t q = blockIdx.x * RS_BLOCK + threadIdx.x; q < F; q += gridDim.x * RS_BLOCK)
        if (dk[q] != RS_NONE) slot[dk[q]] = q;
}

// The grouped path's reasm_ec (workgroups [0, nec)) with the speculative tail's completion list
// behind it (the workgroups after them, one per chunk: reasm_clist_write from reasm_scan's chunk
// counts). The list needs nothing reasm_ec computes: it is written while the run test may still
// find the batch not grouped, and the emit behind it checks that first.
__global__ void __launch_bounds__(RS_BLOCK) reasm_ec_clist(ReasmArgs a, uint32_t nec, SpecTail g)
{
    if (blockIdx.x < nec)
        ec_block(a, RS_F_DEV, blockIdx.x, nec);
    else
        clist_write_block(a.dk, a.done, RS_F_DEV, a.cblk, a.cl_perm, a.cl_offs, g, blockIdx.x - nec, true);
}

// ------------------------------------------------------------------------------------------
// reasm_scan: the grouped path's analysis in one launch (it replaced four: the fragment list's
// write pass, the run test, the flow walk of reasm_flows and the grouped tail's
// reasm_clist_count). One block per RS_CL positions of the fragment list, each wave RS_SCAN_PW
// consecutive ones as two slots of 64:
//  * the block's positions of the fragment list, found from the FRAG counts (and written);
//  * the run test's first half: a run's first position into its key's slot of rtab (reasm_ec
//    reads them back);
//  * the per-position records reasm_prep would write (reasm_process and the serial path read
//    them), and the same records in LDS for the walk;
//  * reasm_flows' walk of every flow from its first position, from LDS within the wave's
//    positions and from the frames past them, under the assumption that the batch is grouped;
//  * per completion: its chunk's count and bytes (cblk, what reasm_clist_write starts from) and,
//    in place, whether its fragments can be joined where they lie (else counts[5]);
//  * per block the outcome totals (pblk), which stand for reasm_process's sum when no flow is
//    complex, and for each simple flow reasm_ec's free-entry test with no complex flow counted.
// When the run test finds a key in two runs (counts[4], by reasm_ec) only the records are used:
// the host clears the counters the walk touched and the batch takes the sorts.
constexpr uint32_t RS_SCAN_PW = 128;
static_assert(RS_WAVES * RS_SCAN_PW == RS_CL, "a scan block's positions are one completion-list chunk");

// A flow's state in registers for reasm_scan's walk (the entry words frag_apply keeps in LDS:
// E_FSIZE, E_TOTAL, E_LAST, E_FR, E_WHERE), plus each slot's frame offset and whether that frame
// is exactly 34 header bytes + its data (the in-place test). Static indices only.
struct FlowReg {
    uint32_t fsize, total, last;
    uint32_t fr[RS_MAX_FRAG], wh[RS_MAX_FRAG], fo[RS_MAX_FRAG];
    uint32_t okm;
};

__device__ __forceinline__ void flow_reset(FlowReg &s)
{
    s.fsize = 0;
    s.total = 0xFFFFFFFFu;
    s.last = 2;
#pragma unroll
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
        s.fr[k] = 0;
        s.wh[k] = RS_HELD;
    }
}

// chain_ok on the registers: the same backward walk, the inner loop unrolled over slots 3..1
__device__ __forceinline__ bool flow_chain_ok(const FlowReg &s)
{
    const uint32_t first_len = s.fr[0] >> 16;
    const uint32_t n = s.last - 1u;
    uint32_t ofs = s.fr[1] & 0xFFFFu, curr = 1;
    for (uint32_t guard = 0; ofs != first_len && guard < 8; ++guard) {
        const uint32_t prev = curr;
#pragma unroll
        for (uint32_t i = RS_MAX_FRAG - 1u; i >= 1u; --i) {
            if (i <= n && ofs != first_len && (s.fr[i] & 0xFFFFu) + (s.fr[i] >> 16) == ofs) {
                curr = i;
                ofs = s.fr[i] & 0xFFFFu;
            }
        }
        if (curr == prev) return false;
    }
    return ofs == first_len;
}

// frag_apply on the registers (same outcomes); fo/ok: the fragment's frame offset and size test
__device__ __forceinline__ uint32_t flow_apply(FlowReg &s, uint32_t len, uint32_t ofs, uint32_t mf, uint32_t where,
                                               uint32_t fo, bool ok)
{
    uint32_t idx;
    s.fsize += len;
    if (ofs == 0) {
        idx = s.fr[0] == 0 ? 0u : RS_NONE;
    } else if (!mf) {
        s.total = ofs + len;
        idx = s.fr[1] == 0 ? 1u : RS_NONE;
    } else {
        idx = s.last;
        if (idx < RS_MAX_FRAG) s.last = idx + 1u;
    }
    if (idx >= RS_MAX_FRAG) return FA_NOSLOT;
#pragma unroll
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
        if (k == idx) {
            s.fr[k] = ofs | (len << 16);
            s.wh[k] = where;
            s.fo[k] = fo;
        }
    }
    s.okm = (s.okm & ~(1u << idx)) | (ok ? 1u << idx : 0u);
    if (s.fsize < s.total) return FA_KEEP;
    const bool sized = s.fsize == s.total && s.fr[0] != 0;
    if (sized && flow_chain_ok(s)) return FA_DONE;
    return sized ? FA_HOLE : FA_ERR;
}

// write_done from the registers
__device__ __forceinline__ void flow_done(const ReasmArgs &a, const FlowReg &s, uint32_t q, uint32_t i)
{
    ReasmDone r;
    r.origin = i;
    r.total = s.total;
    r.n = s.last;
    r.entry = RS_NONE;
#pragma unroll
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
        r.fr[k] = s.fr[k];
        r.where[k] = s.wh[k];
    }
    a.done[q] = r;
    a.dk[q] = i;
}

// inplace_ok on the registers (no fragment is held: the flow never met the table)
__device__ __forceinline__ bool flow_inplace_ok(const FlowReg &s)
{
    ReasmDone r;
    r.n = s.last;
#pragma unroll
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) r.fr[k] = s.fr[k];
    uint32_t sl[RS_MAX_FRAG];
    const uint32_t m = data_order(r, sl);
    if (m < 2u || (pick4(r.fr, sl[0]) & 0xFFFFu) != 0u) return false;
    uint32_t end = 0;
    bool ok = true;
#pragma unroll
    for (uint32_t k = 0; k < RS_MAX_FRAG; ++k) {
        if (k >= m) break;
        const uint32_t q = sl[k], o = pick4(s.fo, q);
        ok = ok && ((s.okm >> q) & 1u) && (k == 0u || o == end);
        end = o + 34u + (pick4(r.fr, q) >> 16);
    }
    return ok;
}

__global__ void __launch_bounds__(RS_BLOCK) reasm_scan(ReasmArgs a)
{
    __shared__ uint32_t crc_tab[256];
    // per wave: each position's record (frame, meta, frame offset, frame length), and per flow
    // start by rank its position, key, signature and bucket summary words
    __shared__ uint32_t r_i[RS_WAVES][RS_SCAN_PW], r_m[RS_WAVES][RS_SCAN_PW], r_o[RS_WAVES][RS_SCAN_PW],
        r_l[RS_WAVES][RS_SCAN_PW];
    __shared__ uint32_t w_pos[RS_WAVES][RS_SCAN_PW], w_src[RS_WAVES][RS_SCAN_PW], w_dst[RS_WAVES][RS_SCAN_PW],
        w_id[RS_WAVES][RS_SCAN_PW], w_sig[RS_WAVES][RS_SCAN_PW], w_s1[RS_WAVES][RS_SCAN_PW],
        w_s2[RS_WAVES][RS_SCAN_PW];
    __shared__ unsigned long long s_red[RS_WAVES][RS_PB];
    __shared__ uint32_t s_red32[RS_WAVES][4];
    __shared__ uint32_t s_fl[RS_CL + 1];                      // the frames of positions L0 .. P1 - 1
    __shared__ uint32_t s_x[RS_WAVES], s_j0, s_pre0, s_F, s_ug;
    __shared__ uint32_t w_ht[RS_WAVES][2 * RS_SCAN_PW];       // per wave: its run keys by start rank
    crc_table_init(crc_tab);
    const uint32_t tid = threadIdx.x, lane = __lane_id(), w = tid >> 6;
    const uint32_t b = blockIdx.x, P0 = b * RS_CL, tgt = P0 ? P0 - 1u : 0u;
    // The fragment list's positions of this block (and the one before them, the run test's left
    // neighbour) from the FRAG counts per RS_FS frames: F and the count block holding position
    // tgt by a scan of the counts, then the FRAG frames of the count blocks from there on in
    // order (the fragment list is written here: no launch of its own)
    {
        uint32_t base = 0;
        for (uint32_t j0 = 0; j0 < a.nfs; j0 += RS_BLOCK * 8u) {       // block-uniform
            uint32_t c[8], t = 0;
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t j = j0 + tid * 8u + u;
                c[u] = j < a.nfs ? a.fcnt[j] : 0u;
                t += c[u];
            }
            uint32_t wt;
            uint32_t run = wave_excl_scan(t, &wt);
            if (lane == 0) s_x[w] = wt;
            __syncthreads();
            uint32_t tot = 0;
#pragma unroll
            for (uint32_t x = 0; x < RS_WAVES; ++x) {
                run += x < w ? s_x[x] : 0u;
                tot += s_x[x];
            }
            run += base;
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                if (c[u] && tgt >= run && tgt < run + c[u]) {
                    s_j0 = j0 + tid * 8u + u;
                    s_pre0 = run;
                }
                run += c[u];
            }
            base += tot;
            __syncthreads();
        }
        if (tid == 0) s_F = base;
    }
    __syncthreads();
    const uint32_t F = s_F;
    if (b == 0 && tid == 0) a.counts[0] = F;
    if (P0 >= F) return;                                          // the whole block
    const uint32_t P1 = min(P0 + RS_CL, F), L0 = tgt;
    for (uint32_t j = s_j0, pos = s_pre0; pos < P1; ++j) {          // block-uniform
        const uint32_t i0 = j * RS_FS + 8u * tid;
        const uint32_t m = frag_bits8(a.meta, i0, a.n);
        uint32_t wt;
        uint32_t q = wave_excl_scan((uint32_t)__builtin_popcount(m), &wt);
        if (lane == 0) s_x[w] = wt;
        __syncthreads();
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t x = 0; x < RS_WAVES; ++x) {
            q += x < w ? s_x[x] : 0u;
            tot += s_x[x];
        }
        q += pos;
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            if ((m >> u) & 1u) {
                if (q >= L0 && q < P1) s_fl[q - L0] = i0 + u;
                ++q;
            }
        }
        pos += tot;
        __syncthreads();
    }
    for (uint32_t x = P0 + tid; x < P1; x += RS_BLOCK) a.frag_list[x] = s_fl[x - L0];
    // a block found a key in two runs already: the fragment list is all the sorts need
    if (tid == 0) s_ug = ld_a(&a.counts[4]);
    for (uint32_t x = lane; x < 2u * RS_SCAN_PW; x += 64u) w_ht[w][x] = 0xFFFFFFFFu;
    __syncthreads();
    if (s_ug) return;                                             // the whole block
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    const uint32_t wb = b * RS_CL + w * RS_SCAN_PW;
    constexpr uint32_t OOR = 0x80000000u;
    // the two slots' fragments, each level of the chains (list, offset, header) in one round trip
    // with lane 0's previous position (the run test's left neighbour of the wave's first)
    uint32_t i[2], o[2], w16[2], w20[2], src[2], dst[2], fl[2], id[2];
    bool valid[2];
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        valid[k] = wb + 64u * k + lane < F;
        i[k] = valid[k] ? s_fl[wb + 64u * k + lane - L0] : 0u;
    }
    const bool prev = lane == 0u && valid[0] && wb > 0u;
    const uint32_t ip = prev ? s_fl[wb - 1u - L0] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) o[k] = a.offset[i[k]];
    const uint32_t op = prev ? a.offset[ip] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        w16[k] = ld32(fr, o[k] + 16);
        w20[k] = ld32(fr, o[k] + 20);
        src[k] = ld32(fr, o[k] + 26);
        dst[k] = ld32(fr, o[k] + 30);
        fl[k] = a.length[i[k]];
        id[k] = w16[k] >> 16;
    }
    const uint32_t pw16 = ld32(fr, prev ? op + 16 : OOR), pws = ld32(fr, prev ? op + 26 : OOR),
                   pwd = ld32(fr, prev ? op + 30 : OOR);
    bool start[2];
    {
        uint32_t pid = __shfl_up(id[0], 1, 64), ps = __shfl_up(src[0], 1, 64), pd = __shfl_up(dst[0], 1, 64);
        if (prev) {
            pid = pw16 >> 16;
            ps = pws;
            pd = pwd;
        }
        start[0] = valid[0] && (wb + lane == 0u || pid != id[0] || ps != src[0] || pd != dst[0]);
        uint32_t qid = __shfl_up(id[1], 1, 64), qs = __shfl_up(src[1], 1, 64), qd = __shfl_up(dst[1], 1, 64);
        const uint32_t lid = (uint32_t)__builtin_amdgcn_readlane((int)id[0], 63),
                       ls = (uint32_t)__builtin_amdgcn_readlane((int)src[0], 63),
                       ld = (uint32_t)__builtin_amdgcn_readlane((int)dst[0], 63);
        if (lane == 0u) {
            qid = lid;
            qs = ls;
            qd = ld;
        }
        start[1] = valid[1] && (qid != id[1] || qs != src[1] || qd != dst[1]);
    }
    // The wave's flows in position order, one per lane (a wave of 2-fragment flows walks once,
    // not once per slot): each start's position and key by its rank (signature and bucket words
    // below).
    const unsigned long long m0 = __ballot(start[0]), m1 = __ballot(start[1]);
    const uint32_t n0 = (uint32_t)__popcll(m0), S = n0 + (uint32_t)__popcll(m1);
    uint32_t rank[2] = {0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        if (start[k]) {
            rank[k] = (k ? n0 : 0u) + __builtin_amdgcn_mbcnt_hi((uint32_t)((k ? m1 : m0) >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)(k ? m1 : m0), 0u));
            w_pos[w][rank[k]] = 64u * k + lane;
            w_src[w][rank[k]] = src[k];
            w_dst[w][rank[k]] = dst[k];
            w_id[w][rank[k]] = id[k];
        }
    }
    wave_sync_rs();
    // Two runs of one key in the wave's positions: the batch is not grouped (interleaved flows
    // show it here, long before reasm_ec's run test), and nothing but the fragment list is needed
    // from this launch. Insert-or-find of each run's key in an LDS table by rank.
    bool dup = false;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        if (!start[k]) continue;
        uint32_t h = ((src[k] * 0x9E3779B1u) ^ (dst[k] * 0x85EBCA77u) ^ (id[k] * 0xC2B2AE3Du)) >> 24;
        for (uint32_t t = 0; t < 2u * RS_SCAN_PW; ++t, h = (h + 1u) & (2u * RS_SCAN_PW - 1u)) {
            const uint32_t old = atomicCAS(&w_ht[w][h], 0xFFFFFFFFu, rank[k]);
            if (old == 0xFFFFFFFFu) break;
            if (w_src[w][old] == src[k] && w_dst[w][old] == dst[k] && w_id[w][old] == id[k]) {
                dup = true;
                break;
            }
        }
    }
    const bool ug = __ballot(dup) != 0ull;
    if (ug && lane == 0) a.counts[4] = 1u;
    const bool skip = ug || __builtin_amdgcn_readfirstlane((int)ld_a(&a.counts[4])) != 0;
    unsigned long long t_len = 0, t_short = 0, t_done = 0, t_holes = 0, t_err = 0, t_bytes = 0;
    uint32_t t_cc = 0, t_cb = 0, t_cplx = 0, t_nb = 0;
    if (!skip) {
    // The run test's first half (each run's first position into its key's slot of rtab: plain
    // stores, read back by reasm_ec) and the flow's bucket summary words.
    uint32_t sig[2], s1v[2] = {0u, 0u}, s2v[2] = {0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        FragHdr h;
        h.src = src[k];
        h.dst = dst[k];
        h.id = id[k];
        sig[k] = rec_sig(crc_tab, h);
        if (start[k]) {
            a.rtab[run_slot(a, id[k], src[k], dst[k])] = wb + 64u * k + lane;
            s1v[k] = a.bsum[bucket_of(a, sig[k])];
            s2v[k] = a.bsum[bucket2_of(a, sig[k])];
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        FragHdr h;
        h.src = src[k];
        h.dst = dst[k];
        h.id = id[k];
        h.tl = bswap16(w16[k] & 0xFFFFu);
        h.ff = bswap16(w20[k] & 0xFFFFu);
        h.flen = fl[k];
        const uint32_t m = rec_meta(a, h);
        const uint32_t p = wb + 64u * k + lane;
        if (valid[k]) {
            a.s_i[p] = i[k];
            a.s_src[p] = src[k];
            a.s_dst[p] = dst[k];
            a.s_id[p] = id[k];
            a.s_sig[p] = sig[k];
            a.s_meta[p] = m;
        }
        r_i[w][64u * k + lane] = i[k];
        r_m[w][64u * k + lane] = m;
        r_o[w][64u * k + lane] = o[k];
        r_l[w][64u * k + lane] = fl[k];
        if (start[k]) {
            w_sig[w][rank[k]] = sig[k];
            w_s1[w][rank[k]] = s1v[k];
            w_s2[w][rank[k]] = s2v[k];
        } else if (valid[k]) {
            a.pflag[p] = 0u;
        }
    }
    wave_sync_rs();
    const bool limit = a.max_entries < a.entries;
#pragma unroll 1
    for (uint32_t j = lane; j < ((S + 63u) & ~63u); j += 64u) {   // wave-uniform trip count
        if (j >= S) continue;
        const uint32_t p = wb + w_pos[w][j];
        const uint32_t ksrc = w_src[w][j], kdst = w_dst[w][j], kid = w_id[w][j], ksig = w_sig[w][j];
        FlowReg s;
        s.okm = 0;
        s.last = 2;
        bool live = false;
        uint32_t tfirst = RS_NONE;
        uint32_t c_len = 0, c_short = 0, c_done = 0, c_holes = 0, c_err = 0;
        unsigned long long c_bytes = 0;
        // completions in this block's chunk, in one later chunk (x_chunk), in more (x_ovf)
        uint32_t own_c = 0, own_b = 0, x_c = 0, x_b = 0, x_chunk = 0;
        bool x_ovf = false;
        uint32_t q = p, last_fi = 0;
        for (; q < F; ++q) {
            uint32_t m, fi, fo, ffl;
            const uint32_t d = q - wb;
            if (d < RS_SCAN_PW) {
                if (q != p && (((d < 64u ? m0 >> d : m1 >> (d - 64u)) & 1ull) != 0ull)) break;
                m = r_m[w][d];
                fi = r_i[w][d];
                fo = r_o[w][d];
                ffl = r_l[w][d];
            } else {                                                 // past the wave's positions
                if (q < P1) {
                    fi = s_fl[q - L0];
                } else {            // past the block's: the next FRAG frame after the previous one
                    fi = last_fi + 1u;
                    while ((a.meta[fi] & 0xFu) != UDPDK_V_FRAG) ++fi;
                }
                fo = a.offset[fi];
                const uint32_t x16 = ld32(fr, fo + 16), x20 = ld32(fr, fo + 20), xs = ld32(fr, fo + 26),
                               xd = ld32(fr, fo + 30);
                if ((x16 >> 16) != kid || xs != ksrc || xd != kdst) break;
                FragHdr h;
                h.src = xs;
                h.dst = xd;
                h.id = x16 >> 16;
                h.tl = bswap16(x16 & 0xFFFFu);
                h.ff = bswap16(x20 & 0xFFFFu);
                h.flen = a.length[fi];
                m = rec_meta(a, h);
                ffl = h.flen;
            }
            last_fi = fi;
            const uint32_t cls = m >> 30;
            if (cls) {
                if (cls == 1) ++c_len;
                else ++c_short;
                a.dk[q] = RS_NONE;
                continue;
            }
            if (tfirst == RS_NONE) tfirst = fi;
            if (!live) flow_reset(s);
            const uint32_t len = m & 0xFFFFu;
            const uint32_t r = flow_apply(s, len, ((m >> 16) & 0x1FFFu) * 8u, (m >> 29) & 1u, fi, fo, ffl == 34u + len);
            live = r == FA_KEEP;
            if (r == FA_DONE) {
                flow_done(a, s, q, fi);
                ++c_done;
                const uint32_t by = (34u + s.total + 15u) & ~15u;
                c_bytes += by;
                const uint32_t cq = q / RS_CL;
                if (cq == b) {
                    ++own_c;
                    own_b += by;
                } else if (x_c == 0u || cq == x_chunk) {
                    x_chunk = cq;
                    ++x_c;
                    x_b += by;
                } else {
                    x_ovf = true;
                }
                if (a.inplace && !flow_inplace_ok(s)) atomicOr(&a.counts[5], 1u);      // rare
            } else {
                a.dk[q] = RS_NONE;
                if (r == FA_HOLE) ++c_holes;
                else if (r != FA_KEEP) ++c_err;
            }
        }
        const bool ovf = (c_len | c_short | c_done | c_holes | c_err) > 62u || c_bytes >= (1ull << 31);
        a.oc[p] = c_len | c_short << 6 | c_done << 12 | c_holes << 18 | c_err << 24 | (ovf ? OC_OVF : 0u);
        a.ob[p] = (uint32_t)c_bytes;
        t_len += c_len;
        t_short += c_short;
        uint32_t flag = PF_START;
        if (tfirst != RS_NONE) {
            flag |= PF_TOUCH | (live ? PF_COMPLEX : 0u);
            const uint32_t bk1 = bucket_of(a, ksig), bk2 = bucket2_of(a, ksig);
            const uint32_t s1 = w_s1[w][j], s2 = w_s2[w][j];
            if ((s1 | s2) >> 31) {
                flag |= PF_COMPLEX;                           // an expired entry to reclaim
            } else if ((s1 | s2) & 0xFFFFu) {                 // is the key in the table?
                for (uint32_t h = 0; h < 2; ++h) {
                    const uint32_t *e = a.tab + (size_t)(h ? bk2 : bk1) * a.assoc * E_WORDS;
                    for (uint32_t x = 0; x < a.assoc; ++x, e += E_WORDS)
                        if (ld_a(e + E_VALID) && ld_a(e + E_SRC) == ksrc && ld_a(e + E_DST) == kdst &&
                            ld_a(e + E_ID) == kid)
                            flag |= PF_COMPLEX;
                }
            }
            a.sb1[p] = bk1;
            a.sb2[p] = bk2;
            if (flag & PF_COMPLEX) {
                atomicAdd(&a.cplx[bk1], 1u);
                if (bk2 != bk1) atomicAdd(&a.cplx[bk2], 1u);
                ++t_cplx;
                if (limit) ++t_nb;
                // a complex flow goes through the table: no completion of its own
                if (c_done)
                    for (uint32_t v = p; v < q; ++v) a.dk[v] = RS_NONE;
            } else {
                // reasm_ec's test with no complex flow: a free entry in one of its buckets
                int32_t f0 = (int32_t)a.assoc - (int32_t)(s1 & 0xFFFFu);
                if (bk2 != bk1) f0 += (int32_t)a.assoc - (int32_t)(s2 & 0xFFFFu);
                if (f0 < 1) a.counts[3] = 1u;
            }
        }
        if (!(flag & PF_COMPLEX)) {
            t_done += c_done;
            t_holes += c_holes;
            t_err += c_err;
            t_bytes += c_bytes;
            t_cc += own_c;
            t_cb += own_b;
            if (x_c) {
                atomicAdd(&a.cblk[2u * x_chunk], x_c);
                atomicAdd(&a.cblk[2u * x_chunk + 1u], x_b);
            }
            if (x_ovf) a.counts[9] = 1u;
        }
        a.pflag[p] = flag;
    }
    }                                                             // !skip
    // the block's totals: outcome words, its chunk's completions, complex and bound-counted flows
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        t_len += __shfl_xor(t_len, d, 64);
        t_short += __shfl_xor(t_short, d, 64);
        t_done += __shfl_xor(t_done, d, 64);
        t_holes += __shfl_xor(t_holes, d, 64);
        t_err += __shfl_xor(t_err, d, 64);
        t_bytes += __shfl_xor(t_bytes, d, 64);
        t_cc += __shfl_xor(t_cc, d, 64);
        t_cb += __shfl_xor(t_cb, d, 64);
        t_cplx += __shfl_xor(t_cplx, d, 64);
        t_nb += __shfl_xor(t_nb, d, 64);
    }
    if (lane == 0) {
        s_red[w][0] = t_len;
        s_red[w][1] = t_short;
        s_red[w][2] = t_done;
        s_red[w][3] = t_holes;
        s_red[w][4] = t_err;
        s_red[w][5] = t_bytes;
        s_red32[w][0] = t_cc;
        s_red32[w][1] = t_cb;
        s_red32[w][2] = t_cplx;
        s_red32[w][3] = t_nb;
    }
    __syncthreads();
    if (threadIdx.x < RS_PB) {
        unsigned long long v = 0;
#pragma unroll
        for (uint32_t x = 0; x < RS_WAVES; ++x) v += s_red[x][threadIdx.x];
        a.pblk[(size_t)b * RS_PB + threadIdx.x] = v;
    } else if (threadIdx.x < RS_PB + 4u) {
        const uint32_t j = threadIdx.x - RS_PB;
        uint32_t v = 0;
#pragma unroll
        for (uint32_t x = 0; x < RS_WAVES; ++x) v += s_red32[x][j];
        if (v) {
            if (j < 2u) atomicAdd(&a.cblk[2u * b + j], v);        // with other blocks' flows' counts
            else atomicAdd(&a.counts[j == 2u ? 8 : 7], v);
        }
    }
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
    SpecTail g;                   // speculative launch: C from the device, or nothing to do
    uint32_t cksum_zero;          // UDPDK_FRAG_CKSUM_DPDK: header checksum left 0 (DPDK's)
};

// One wave per datagram. The output datagram is written as aligned 16-byte chunks (lane =
// chunk, 64 chunks = 1 KiB per wave store): its bytes come from at most a few segments, the first
// fragment's frame bytes [0, 34 + len0) (Ethernet + IPv4 header + its data: the header is the
// first fragment's, as ipv4_frag_reassemble keeps the first mbuf's) and every other fragment's
// data at 34 + its offset, each from the batch or, when held, from the flow's entry buffer
// (where they sit at the same offsets). A chunk's source bytes are read from the dword at or
// below their start (one 16-byte load, the fifth dword from the next lane or its own 4-byte
// load) and funnelled by the start's offset & 3; a chunk that straddles a fragment boundary
// (every boundary does: 34 + 8k is never 16-aligned) merges two such reads by byte mask. The
// former form (byte-aligned 16-byte loads and stores per fragment piece) ran at 3.7 TB/s.
// The header's total length, fragment field (DF only) and IPv4 checksum are patched in chunks
// 0-2 (lanes 0-2 of the first round).
__device__ __forceinline__ uint4 funnel4(const uint4 x, uint32_t hi, uint32_t sh)
{
    return make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, sh), __builtin_amdgcn_alignbyte(x.z, x.y, sh),
                      __builtin_amdgcn_alignbyte(x.w, x.z, sh), __builtin_amdgcn_alignbyte(hi, x.w, sh));
}

// byte i of the result from y where i >= k (0 <= k <= 16), else from x
__device__ __forceinline__ uint4 merge_at(const uint4 x, const uint4 y, uint32_t k)
{
    auto m = [&](uint32_t d) -> uint32_t {      // bytes of dword d taken from x
        const int b = (int)k - 4 * (int)d;
        return b >= 4 ? 0xFFFFFFFFu : b <= 0 ? 0u : (1u << (8 * b)) - 1u;
    };
    const uint32_t m0 = m(0), m1 = m(1), m2 = m(2), m3 = m(3);
    return make_uint4((x.x & m0) | (y.x & ~m0), (x.y & m1) | (y.y & ~m1),
                      (x.z & m2) | (y.z & ~m2), (x.w & m3) | (y.w & ~m3));
}

// the copying emit of C datagrams (reasm_emit; reasm_emit_either when in place was refused)
__device__ __forceinline__ void emit_copy(const EmitArgs &a, uint32_t C)
{
    // the wave index as a scalar: the datagram record and everything derived from it are
    // wave-uniform scalar loads and SGPRs, not per-lane copies
    const uint32_t lane = __lane_id(), w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t fr = rsrc(a.frames, a.rsrc_bytes);
    // The next datagram's record and output offset are loaded while this one is copied.
    const uint32_t stride = gridDim.x * RS_WAVES;
    uint32_t k = blockIdx.x * RS_WAVES + w;
    ReasmDone rn{};
    uint32_t oon = 0;
    if (k < C) {
        rn = cload(&a.done[cload(&a.perm[k])]);
        oon = cload(&a.out_off_in[k]);
    }
    constexpr uint32_t OOR = 0x80000000u;         // out of any buffer's range: no access, zeros
    for (; k < C; k += stride) {
        const ReasmDone r = rn;
        const uint32_t oo = oon;
        if (k + stride < C) {
            rn = cload(&a.done[cload(&a.perm[k + stride])]);
            oon = cload(&a.out_off_in[k + stride]);
        }
        const uint32_t L = 34u + r.total;
        const uint8_t *eb = a.ebuf + (size_t)r.entry * a.stride;
        const __amdgpu_buffer_rsrc_t er = rsrc(eb, a.stride);
        const __amdgpu_buffer_rsrc_t orr = rsrc(a.out + oo, (L + 15u) & ~15u);
        // segments: destination start d0, end d1, source offset of d0 (s0), held
        uint32_t d0[RS_MAX_FRAG], d1[RS_MAX_FRAG], s0[RS_MAX_FRAG];
        bool held[RS_MAX_FRAG];
        bool any_held = false, any_frame = false, small = false;
#pragma unroll
        for (uint32_t q = 0; q < RS_MAX_FRAG; ++q) {
            const bool use = q < r.n && r.fr[q] != 0u;
            const uint32_t ofs = r.fr[q] & 0xFFFFu, ln = r.fr[q] >> 16;
            held[q] = use && r.where[q] == RS_HELD;
            // the fragment at offset 0 carries the header: its segment starts at byte 0
            d0[q] = !use ? 0xFFFFFFFFu : ofs == 0u ? 0u : 34u + ofs;
            d1[q] = !use ? 0xFFFFFFFFu : 34u + ofs + ln;
            const uint32_t fo = use && !held[q] ? cload(&a.offset[r.where[q]]) : 0u;
            s0[q] = held[q] ? d0[q] : fo + (ofs == 0u ? 0u : 34u);
            if (use) {
                any_held = any_held || held[q];
                any_frame = any_frame || !held[q];
                small = small || (d1[q] - d0[q] < 16u);
            }
        }
        const bool mixed = any_held && any_frame;
        const __amdgpu_buffer_rsrc_t one = any_held ? er : fr;
        // the segment holding destination byte b (segments tile [0, L))
        auto seg_of = [&](uint32_t b) -> uint32_t {
            uint32_t s = 0;
#pragma unroll
            for (uint32_t q = 0; q < RS_MAX_FRAG; ++q) s = (b >= d0[q] && b < d1[q]) ? q : s;
            return s;
        };
        auto pick = [&](const uint32_t (&x)[RS_MAX_FRAG], uint32_t q) {
            return q == 0u ? x[0] : q == 1u ? x[1] : q == 2u ? x[2] : x[3];
        };
        auto pickb = [&](uint32_t q) {
            return q == 0u ? held[0] : q == 1u ? held[1] : q == 2u ? held[2] : held[3];
        };
        // chunk c's bytes as read from segment q (source start s0 + 16 c - d0, funnelled)
        auto read_seg = [&](uint32_t c, uint32_t q, bool want) -> uint4 {
            const uint32_t src = pick(s0, q) + 16u * c - pick(d0, q);
            const uint32_t sa = src & ~3u, sh = src & 3u;
            uint4 x;
            uint32_t hi;
            if (!mixed) {
                x = load16(one, want ? sa : OOR);
                hi = ld32(one, want && sh ? sa + 16u : OOR);
            } else {
                const bool h = pickb(q);
                const uint4 x1 = load16(er, want && h ? sa : OOR), x2 = load16(fr, want && !h ? sa : OOR);
                x = make_uint4(x1.x | x2.x, x1.y | x2.y, x1.z | x2.z, x1.w | x2.w);
                hi = ld32(er, want && h && sh ? sa + 16u : OOR) | ld32(fr, want && !h && sh ? sa + 16u : OOR);
            }
            return funnel4(x, hi, sh);
        };
        const uint32_t nch = (L + 15u) >> 4;
        // (two rounds in flight per wave, the fifth dword shuffled from the next chunk: 5 %
        // slower than one round with its own 4-byte load)
        for (uint32_t c0 = 0; c0 < nch; c0 += 64u) {
            const uint32_t c = c0 + lane;
            const bool in = c < nch;
            const uint32_t b0 = 16u * c, b1 = min(b0 + 15u, L - 1u);
            const uint32_t qa = seg_of(min(b0, L - 1u)), qb = seg_of(b1);
            uint4 v = read_seg(c, qa, in);
            const bool two = in && qb != qa;
            if (__ballot(two)) {
                const uint4 y = read_seg(c, qb, two);
                if (two) v = merge_at(v, y, pick(d0, qb) - b0);
            }
            // a middle fragment shorter than a chunk: a chunk may hold three segments
            if (small) {
#pragma unroll
                for (uint32_t q = 0; q < RS_MAX_FRAG; ++q) {
                    const bool mid = in && q != qa && q != qb && d0[q] != 0xFFFFFFFFu &&
                                     d0[q] > b0 && d1[q] <= b0 + 16u;
                    if (__ballot(mid)) {
                        const uint4 y = read_seg(c, q, mid);
                        if (mid) {
                            const uint4 t = merge_at(v, y, d0[q] - b0);
                            v = merge_at(t, v, d1[q] - b0);
                        }
                    }
                }
            }
            if (c0 == 0u) {
                // header: dword 4 (bytes 16-19) total length, dword 5 (20-23) fragment field
                // DF only, dword 6 (24-27) checksum; RFC 1071 over bytes 14..33 (dword 3's high
                // half, dwords 4-7, dword 8's low half)
                if (lane == 1u) {
                    v.x = (v.x & 0xFFFF0000u) | bswap16(r.total + 20u);
                    v.y = (v.y & 0xFFFF0000u) | (v.y & 0x40u);
                    v.z &= 0xFFFF0000u;
                }
                uint32_t part = lane == 0u ? v.w >> 16
                              : lane == 1u ? (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) +
                                             (v.z & 0xFFFFu) + (v.z >> 16) + (v.w & 0xFFFFu) + (v.w >> 16)
                              : lane == 2u ? v.x & 0xFFFFu : 0u;
                part += __shfl_down(part, 1, 64);
                part += __shfl_down(part, 2, 64);
                uint32_t sum = (uint32_t)__builtin_amdgcn_readfirstlane((int)part);
                sum = (sum >> 16) + (sum & 0xFFFFu);
                sum = (sum >> 16) + (sum & 0xFFFFu);
                if (lane == 1u && !a.cksum_zero) v.z |= ~sum & 0xFFFFu;
            }
            if (in) store16(orr, b0, v);
        }
        if (lane == 0) {
            a.out_off[k] = oo;
            a.out_len[k] = (uint16_t)L;
            a.out_ptype[k] = 0x211u;              // L2_ETHER | L3_IPV4 | L4_UDP
            a.out_origin[k] = r.origin;
        }
    }
}

// Bytes [lo, hi) of the 16-byte chunk v at buffer offset D (16-byte aligned; 0 <= lo < hi <= 16):
// the whole dwords as dword stores, the at most three bytes at either end as a byte store and a
// 2-byte store. At most 10 store instructions per wave for any ranges of its lanes, where a store
// per byte took 16 (in place, the texture address unit was 72 % busy, mostly with byte stores).
__device__ __forceinline__ void store_part(__amdgpu_buffer_rsrc_t r, uint32_t D, const uint4 v, uint32_t lo, uint32_t hi)
{
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d)
        if (4u * d >= lo && 4u * d + 4u <= hi) __builtin_amdgcn_raw_buffer_store_b32(vv[d], r, (int)(D + 4u * d), 0, 0);
    auto word = [&](uint32_t x) { return x < 4u ? vv[0] : x < 8u ? vv[1] : x < 12u ? vv[2] : vv[3]; };
    auto bytes = [&](uint32_t a, uint32_t b) {            // [a, b) inside one dword, b - a <= 3
        if (a < b && (a & 1u)) {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(word(a) >> (8u * (a & 3u))), r, (int)(D + a), 0, 0);
            ++a;
        }
        if (a + 2u <= b) {
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(word(a) >> (8u * (a & 2u))), r, (int)(D + a), 0, 0);
            a += 2u;
        }
        if (a < b) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(word(a) >> (8u * (a & 3u))), r, (int)(D + a), 0, 0);
    };
    const uint32_t ha = (lo & 3u) ? min(hi, (lo + 3u) & ~3u) : lo;
    bytes(lo, ha);
    bytes((hi & 3u) ? max(ha, hi & ~3u) : hi, hi);
}

// In place (one wave per datagram): the first fragment's frame is extended over its followers.
// Fragment k (data order, k >= 1) moves 34 k bytes back, over the headers before it, as aligned
// 16-byte chunk rounds in ascending address order: a round's stores land below every byte a later
// round (or fragment k itself) still reads, and fragment k + 1 starts only after fragment k's
// last round (its destination covers the tail of fragment k's source). Then the header's total
// length, fragment field (DF only) and checksum are patched. Datagrams are disjoint regions (the
// caller's frames do not overlap), so waves never touch each other's bytes.
__device__ __forceinline__ void emit_inplace(const EmitArgs &a, uint8_t *frames, uint32_t C)
{
    const uint32_t lane = __lane_id(), w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t fr = rsrc(frames, a.rsrc_bytes);
    constexpr uint32_t OOR = 0x80000000u;
    const uint32_t stride = gridDim.x * RS_WAVES;
    uint32_t k = blockIdx.x * RS_WAVES + w;
    // Software pipeline over the wave's datagrams: the next datagram's fragment offsets (which
    // need its record) are loaded while this one moves, and the record after it is loaded then.
    auto offsets = [&](const ReasmDone &x, uint32_t (&o)[RS_MAX_FRAG], uint32_t (&sx)[RS_MAX_FRAG]) -> uint32_t {
        const uint32_t mx = data_order(x, sx);
#pragma unroll
        for (uint32_t f = 0; f < RS_MAX_FRAG; ++f) o[f] = f < mx ? cload(&a.offset[pick4(x.where, sx[f])]) : 0u;
        return mx;
    };
    // Quick moves: a datagram of two fragments whose move is one round (<= 128 chunks, the
    // MTU-sized case) has its bytes and its header dwords loaded one datagram ahead, before the
    // previous datagram's stores, so the wait for them leaves the next datagram's loads in flight
    // (two datagrams per wave at 8 waves per SIMD). gfx9 counts stores in vmcnt with the loads, in
    // order, so that wait must not also wait for the previous datagram's stores: a quick step
    // issues the same VMEM instructions whatever its geometry (loads at out-of-range offsets when
    // there is nothing to load; every chunk one 16-byte store, dropped out of range; the header
    // patch six byte stores; the outputs stored by every lane), and quick steps run in a loop of
    // their own entered with nothing outstanding, so the compiler's count for that wait (the
    // step's 12 stores and the next datagram's 7 loads younger than it) holds on every path. The first chunk's bytes below the destination (the first
    // fragment's data) are loaded with the move's bytes and stored back merged; the last chunk's
    // bytes past the datagram's end land in the second fragment's old frame (its 34 header bytes
    // are more than a chunk), which nothing reads again. Other datagrams take the round loop.
    struct Quick {
        uint32_t D0, dst, De, shift, nch;
        uint4 x[2];
        uint32_t hi[2];
        uint4 orig;                          // lane 0: the 16 bytes at D0 before the move
        uint32_t hw[6];                      // lane 0: header dwords from the one at or below byte 14
    };
    auto quick_geom = [&](const ReasmDone &x, const uint32_t (&o)[RS_MAX_FRAG], const uint32_t (&sx)[RS_MAX_FRAG],
                          uint32_t mx, bool have, Quick &g) -> bool {
        const uint32_t fq = pick4(x.fr, sx[1]);
        g.dst = o[0] + 34u + (fq & 0xFFFFu);
        g.D0 = g.dst & ~15u;
        g.De = g.dst + (fq >> 16);
        g.shift = o[1] + 34u - g.dst;
        g.nch = (g.De - g.D0 + 15u) >> 4;
        return have && mx == 2u && g.nch <= 128u;
    };
    // header dwords of the datagram whose first frame is at o0 (any datagram: the patch needs
    // them), then the move's bytes when quick
    auto header_load = [&](uint32_t (&hw)[6], bool have, uint32_t o0) {
        const uint32_t ha = (o0 + 14u) & ~3u;
        const uint4 h4 = load16(fr, have && lane == 0u ? ha : OOR);
        const auto h2 = __builtin_amdgcn_raw_buffer_load_b64(fr, (int)(have && lane == 0u ? ha + 16u : OOR), 0, 0);
        hw[0] = h4.x; hw[1] = h4.y; hw[2] = h4.z; hw[3] = h4.w; hw[4] = h2[0]; hw[5] = h2[1];
    };
    auto quick_load = [&](Quick &g, bool on, bool have, uint32_t o0) {
        header_load(g.hw, have, o0);
#pragma unroll
        for (uint32_t u = 0; u < 2; ++u) {
            const uint32_t c = 64u * u + lane;
            const bool in = on && c < g.nch;
            const uint32_t S = g.D0 + 16u * c + g.shift, sa = S & ~3u;
            g.x[u] = load16(fr, in ? sa : OOR);
            g.hi[u] = ld32(fr, in && (S & 3u) ? sa + 16u : OOR);
        }
        g.orig = load16(fr, on && lane == 0u ? g.D0 : OOR);
    };
    ReasmDone r{}, rn{};
    uint32_t fo[RS_MAX_FRAG] = {0, 0, 0, 0}, sl[RS_MAX_FRAG] = {0, 0, 0, 0}, m = 0;
    if (k < C) {
        r = cload(&a.done[cload(&a.perm[k])]);
        m = offsets(r, fo, sl);
    }
    if (k + stride < C) rn = cload(&a.done[cload(&a.perm[k + stride])]);
    // the current datagram's loads sit in one of two register sets and the next one's go to the
    // other (a quick run alternates them: a copy from the next set to the current one would wait
    // for the next datagram's loads to land)
    Quick q0, q1;
    bool qc_on = quick_geom(r, fo, sl, m, k < C, q0);
    quick_load(q0, qc_on, k < C, fo[0]);
    // one datagram (k): the next one's loads, this one's move, header patch and outputs; then the
    // pipeline advances
    auto step = [&](bool quick, Quick &qc, Quick &qn) {
        uint32_t fon[RS_MAX_FRAG] = {0, 0, 0, 0}, sln[RS_MAX_FRAG] = {0, 0, 0, 0}, mn = 0;
        ReasmDone rnn{};
        if (k + stride < C) mn = offsets(rn, fon, sln);
        if (k + 2u * stride < C) rnn = cload(&a.done[cload(&a.perm[k + 2u * stride])]);
        const uint32_t o0 = fo[0], hs = (o0 + 14u) & 3u;
        const uint32_t (&hw)[6] = qc.hw;
        const bool qn_on = quick_geom(rn, fon, sln, mn, k + stride < C, qn);
        quick_load(qn, qn_on, k + stride < C, fon[0]);             // the next datagram in flight
        // (pinned: the scheduler otherwise hoists this datagram's first uses, and their waits,
        // above the next datagram's loads, which then issue only once these bytes have landed)
        __builtin_amdgcn_sched_barrier(0);
        if (quick) {
#pragma unroll
            for (uint32_t u = 0; u < 2; ++u) {
                const uint32_t c = 64u * u + lane;
                const uint32_t D = qc.D0 + 16u * c;
                uint4 v = funnel4(qc.x[u], qc.hi[u], (D + qc.shift) & 3u);
                if (u == 0u) {                   // (per component: a uint4 select went through scratch)
                    const uint4 mv = merge_at(qc.orig, v, qc.dst - qc.D0);
                    const bool l0 = lane == 0u;
                    v.x = l0 ? mv.x : v.x;
                    v.y = l0 ? mv.y : v.y;
                    v.z = l0 ? mv.z : v.z;
                    v.w = l0 ? mv.w : v.w;
                }
                store16(fr, c < qc.nch ? D : OOR, v);
            }
        } else {
#pragma unroll
            for (uint32_t f = 1; f < RS_MAX_FRAG; ++f) {            // static indices: no scratch
                if (f >= m) break;
                const uint32_t q = sl[f];
                const uint32_t fq = pick4(r.fr, q);
                const uint32_t len = fq >> 16, ofs = fq & 0xFFFFu;
                const uint32_t src = fo[f] + 34u, dst = o0 + 34u + ofs;
                // bytes [dst, dst + len) <- [src, src + len), dst < src: destination-aligned
                // 16-byte chunks (lane = chunk), two rounds' loads in flight before their stores (a
                // round's stores land below every byte a later round reads); the two partial end
                // chunks store only their own bytes
                const uint32_t D0 = dst & ~15u, De = dst + len, shift = src - dst;
                const uint32_t nch = (De - D0 + 15u) >> 4;
                for (uint32_t c0 = 0; c0 < nch; c0 += 128u) {
                    uint4 v[2];
                    uint32_t Dv[2];
                    bool inv[2];
#pragma unroll
                    for (uint32_t u = 0; u < 2; ++u) {
                        const uint32_t c = c0 + 64u * u + lane;
                        inv[u] = c < nch;
                        Dv[u] = D0 + 16u * c;
                        const uint32_t S = Dv[u] + shift, sa = S & ~3u, sh = S & 3u;
                        const uint4 x = load16(fr, inv[u] ? sa : OOR);
                        const uint32_t hi = ld32(fr, inv[u] && sh ? sa + 16u : OOR);
                        v[u] = funnel4(x, hi, sh);
                    }
#pragma unroll
                    for (uint32_t u = 0; u < 2; ++u) {
                        const uint32_t D = Dv[u];
                        if (inv[u] && D >= dst && D + 16u <= De)
                            store16(fr, D, v[u]);
                        else if (inv[u])
                            store_part(fr, D, v[u], D >= dst ? 0u : dst - D, min(De - D, 16u));
                    }
                }
            }
        }
        // header: total length (16-17), fragment field DF only (20-21), checksum (24-25) over
        // bytes 14..33 (lane 0's values; the other lanes' stores drop)
        {
            uint32_t h[5];
#pragma unroll
            for (uint32_t j = 0; j < 5; ++j) h[j] = __builtin_amdgcn_alignbyte(hw[j + 1], hw[j], hs);
            // h[0] = bytes 14-17, h[1] = 18-21, h[2] = 22-25, h[3] = 26-29, h[4] = 30-33
            const uint32_t tl = r.total + 20u;
            h[0] = (h[0] & 0x0000FFFFu) | ((tl >> 8) & 0xFFu) << 16 | (tl & 0xFFu) << 24;
            h[1] = (h[1] & 0x0000FFFFu) | (h[1] & 0x00400000u);
            h[2] = h[2] & 0x0000FFFFu;
            uint32_t sum = 0;
#pragma unroll
            for (uint32_t j = 0; j < 5; ++j) sum += (h[j] & 0xFFFFu) + (h[j] >> 16);
            sum = (sum >> 16) + (sum & 0xFFFFu);
            sum = (sum >> 16) + (sum & 0xFFFFu);
            const uint32_t ck = a.cksum_zero ? 0u : ~sum & 0xFFFFu;
            const uint16_t pw[3] = {(uint16_t)(h[0] >> 16), (uint16_t)(h[1] >> 16), (uint16_t)ck};
            const uint32_t po[3] = {16, 20, 24};
#pragma unroll
            for (uint32_t j = 0; j < 3; ++j) {
                const uint32_t at = lane == 0u ? o0 + po[j] : OOR;
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)pw[j], fr, (int)at, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(pw[j] >> 8), fr, (int)(at + 1u), 0, 0);
            }
            a.out_off[k] = o0;
            a.out_len[k] = (uint16_t)(34u + r.total);
            a.out_ptype[k] = 0x211u;
            a.out_origin[k] = r.origin;
        }
        r = rn;
        rn = rnn;
        m = mn;
#pragma unroll
        for (uint32_t f = 0; f < RS_MAX_FRAG; ++f) { fo[f] = fon[f]; sl[f] = sln[f]; }
        qc_on = qn_on;
        k += stride;
    };
    while (k < C) {
        if (qc_on) {
            // the run's first datagram's loads land here (vmcnt(0)), so on entry nothing the
            // loop's waits count is outstanding and they follow the loop's own steady state
            __builtin_amdgcn_s_waitcnt(0x0F70);
            for (;;) {
                step(true, q0, q1);
                if (!(k < C && qc_on)) {
                    q0 = q1;
                    break;
                }
                step(true, q1, q0);
                if (!(k < C && qc_on)) break;
            }
        } else {
            step(false, q0, q1);
            q0 = q1;
        }
    }
}

// Both emits at 8 waves per SIMD: their SGPR budget alone allows 7 (106 SGPRs), and the move is
// latency-bound, so the eighth wave is worth its SGPR spills to VGPR lanes (copy 514-521 -> 474-480
// us per call, in place 447-472 -> 402-408 us; same-box A/Bs)
__global__ void __launch_bounds__(RS_BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8)))
reasm_emit(EmitArgs a)
{
    uint32_t F_unused, C = a.C;
    if (!spec_tail_go(a.g, F_unused, C) || !spec_copy_fits(a.g)) return;
    emit_copy(a, C);
}

// A call that may reassemble in place: one launch takes whichever emit the device-side check
// chose (in place unless reasm_scan refused it, then the copy when its buffer fits), so
// the call has no second, empty emit launch.
__global__ void __launch_bounds__(RS_BLOCK) __attribute__((amdgpu_waves_per_eu(UDPDK_RS_EMIT_WPE, 8)))
reasm_emit_either(EmitArgs a, uint8_t *frames)
{
    uint32_t F_unused, C = a.C;
    if (!spec_tail_go(a.g, F_unused, C)) return;
    if (!__hip_atomic_load(a.g.refuse, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        emit_inplace(a, frames, C);
    else if (spec_copy_fits(a.g))
        emit_copy(a, C);
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
        if (jb.frame == RS_NONE) continue;
        uint8_t *eb = a.ebuf + (size_t)jb.entry * a.stride;
        const uint32_t ofs = jb.fr & 0xFFFFu, len = jb.fr >> 16, fo = a.offset[jb.frame];
        if (ofs == 0) wave_copy(eb, fr, fo, 34u);
        wave_copy16(eb + 34 + ofs, fr, fo + 34u, len);
    }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct Reasm {
    int device = 0;
    uint32_t *tab = nullptr;                 // [entries][E_WORDS]
    uint8_t *ebuf = nullptr;
    uint32_t entries = 0, assoc = 0, mask = 0, max_dgram = 0, stride = 0, assoc_log2 = 0, nbuckets = 0;
    uint32_t max_entries = 0, flags = 0;
    uint32_t *tab_used = nullptr;            // device: valid entries (reasm_serial keeps it)
    uint64_t max_cycles = 0;
    uint32_t cap = 0;                        // fragments per call (= context max_frames)
    uint32_t *frag_list = nullptr, *v1 = nullptr, *v1s = nullptr, *v2s = nullptr;
    unsigned long long *k1 = nullptr, *k1s = nullptr, *k2 = nullptr, *k2s = nullptr;
    uint32_t *counts = nullptr;              // device [10] (ReasmArgs::counts)
    unsigned long long *hset = nullptr;      // [hcap] the run test's exact set (run_insert)
    uint32_t *rtab = nullptr;                // [2 x hcap] the run test's slots (reasm_scan, reasm_ec)
    uint32_t *ccomp = nullptr;               // [cap] the serial fragments' bucket components
    unsigned long long *gset = nullptr;      // [hcap] key groups of a batch that is not grouped
    uint32_t *cblk = nullptr;                // [2 x chunks] reasm_scan's completion counts
    unsigned long long *pblk = nullptr;      // [RS_PB x chunks] reasm_scan's outcome per block
    uint32_t hcap = 0;
    unsigned long long *stats = nullptr;     // device [UDPDK_RS_N]
    unsigned long long *out_bytes = nullptr;
    ReasmDone *done = nullptr;
    ReasmJob *jobs = nullptr;
    uint32_t *dk = nullptr, *dks = nullptr;
    uint32_t *dv = nullptr, *perm = nullptr, *sizes = nullptr, *offs = nullptr;
    uint32_t *pflag = nullptr, *sb1 = nullptr, *sb2 = nullptr, *tf = nullptr, *tl = nullptr;
    uint32_t *oc = nullptr, *ob = nullptr;
    unsigned long long *rk = nullptr, *rks = nullptr, *rx = nullptr;
    uint32_t *rv = nullptr, *rvs = nullptr, *bsum = nullptr, *cplx = nullptr, *tpos = nullptr;
    uint32_t *sl_k = nullptr, *sl_ks = nullptr, *sl_v = nullptr, *sl_vs = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    uint32_t *host = nullptr;                // pinned readback: counts + out_bytes + stats
    uint8_t *out = nullptr;
    uint64_t out_cap = 0;
    uint32_t *out_off = nullptr, *out_ptype = nullptr, *out_origin = nullptr;
    uint16_t *out_len = nullptr;
    uint32_t calls = 0;
    bool no_cc = false;                      // UDPDK_RS_CC=0 (tests, A/B): the serial list on one wave
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
    void *dev[] = {r->tab, r->tab_used, r->ebuf, r->frag_list, r->v1, r->v1s, r->v2s, r->k1, r->k1s, r->k2,
                   r->k2s, r->stats, r->done, r->jobs, r->dk, r->dks,
                   r->dv, r->perm, r->sizes, r->offs, r->tmp, r->out, r->out_off, r->out_ptype,
                   r->out_origin, r->out_len, r->pflag, r->sb1, r->sb2, r->tf, r->tl, r->oc, r->ob, r->rk, r->rks,
                   r->rx, r->rv, r->rvs, r->bsum, r->cplx, r->tpos, r->sl_k, r->sl_ks, r->sl_v, r->sl_vs, r->hset,
                   r->cblk, r->pblk, r->rtab, r->ccomp, r->gset};
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
        cfg->bucket_entries > 32 || want > (1u << 22) || !cfg->max_dgram || cfg->max_dgram > 65515u ||
        (cfg->flags & ~UDPDK_FRAG_CKSUM_DPDK) || cfg->reserved)
        return -EINVAL;
    uint64_t entries = 1;
    while (entries < want) entries <<= 1;
    if (cfg->max_entries > entries) return -EINVAL;        // rte_ip_frag_table_create's check
    Reasm *r = new (std::nothrow) Reasm;
    if (!r) return -ENOMEM;
    r->device = device;
    r->entries = (uint32_t)entries;
    r->assoc = cfg->bucket_entries;
    r->assoc_log2 = (uint32_t)__builtin_ctz(r->assoc);
    r->nbuckets = r->entries / r->assoc;
    r->mask = (r->entries - 1u) & ~(r->assoc - 1u);
    r->max_cycles = cfg->max_cycles;
    r->max_dgram = cfg->max_dgram;
    r->max_entries = cfg->max_entries ? cfg->max_entries : r->entries;
    if (const char *ev = getenv("UDPDK_RS_CC")) r->no_cc = atoi(ev) == 0;
    r->flags = cfg->flags;
    r->stride = (34u + cfg->max_dgram + 4u + 255u) & ~255u;   // + 4: dword loads of the last bytes
    r->cap = std::max<uint32_t>(max_frames, 1);
    int rc = 0;
    auto fail = [&](hipError_t e) { *hip_err = (int)e; rc = e == hipErrorOutOfMemory ? -ENOMEM : -EIO; };
    hipError_t e = hipSuccess;
    const size_t C = r->cap, C2 = 2 * (size_t)r->cap;
    if ((e = dalloc(&r->tab, (size_t)r->entries * E_WORDS)) != hipSuccess ||
        (e = hipMemset(r->tab, 0, (size_t)r->entries * E_WORDS * sizeof(uint32_t))) != hipSuccess ||
        (e = dalloc(&r->tab_used, 1)) != hipSuccess || (e = hipMemset(r->tab_used, 0, 4)) != hipSuccess ||
        (e = hipMalloc((void **)&r->ebuf, (size_t)r->entries * r->stride)) != hipSuccess ||
        (e = dalloc(&r->frag_list, C)) != hipSuccess || (e = dalloc(&r->v1s, C)) != hipSuccess ||
        (e = dalloc(&r->v2s, C)) != hipSuccess || (e = dalloc(&r->k1, C)) != hipSuccess ||
        (e = dalloc(&r->k1s, C)) != hipSuccess || (e = dalloc(&r->k2, C)) != hipSuccess ||
        (e = dalloc(&r->k2s, C)) != hipSuccess || (e = dalloc(&r->stats, RS_ZERO_WORDS)) != hipSuccess ||
        (e = dalloc(&r->done, C)) != hipSuccess || (e = dalloc(&r->jobs, C)) != hipSuccess ||
        (e = dalloc(&r->dk, C)) != hipSuccess || (e = dalloc(&r->dks, C)) != hipSuccess ||
        (e = dalloc(&r->dv, C)) != hipSuccess || (e = dalloc(&r->perm, C)) != hipSuccess ||
        (e = dalloc(&r->sizes, C)) != hipSuccess || (e = dalloc(&r->offs, C)) != hipSuccess ||
        (e = dalloc(&r->out_off, C)) != hipSuccess || (e = dalloc(&r->out_len, C)) != hipSuccess ||
        (e = dalloc(&r->out_ptype, C)) != hipSuccess || (e = dalloc(&r->out_origin, C)) != hipSuccess ||
        (e = dalloc(&r->pflag, C)) != hipSuccess || (e = dalloc(&r->sb1, C)) != hipSuccess ||
        (e = dalloc(&r->oc, C)) != hipSuccess || (e = dalloc(&r->ob, C)) != hipSuccess ||
        (e = dalloc(&r->sb2, C)) != hipSuccess || (e = dalloc(&r->tf, C)) != hipSuccess ||
        (e = dalloc(&r->tl, C)) != hipSuccess || (e = dalloc(&r->rk, C2)) != hipSuccess ||
        (e = dalloc(&r->rks, C2)) != hipSuccess || (e = dalloc(&r->rx, C2)) != hipSuccess ||
        (e = dalloc(&r->rv, C2)) != hipSuccess || (e = dalloc(&r->rvs, C2)) != hipSuccess ||
        (e = dalloc(&r->bsum, r->nbuckets)) != hipSuccess || (e = dalloc(&r->cplx, r->nbuckets)) != hipSuccess ||
        (e = dalloc(&r->tpos, (size_t)r->entries * RS_MAX_FRAG)) != hipSuccess ||
        (e = dalloc(&r->sl_k, C)) != hipSuccess || (e = dalloc(&r->sl_ks, C)) != hipSuccess ||
        (e = dalloc(&r->sl_v, C)) != hipSuccess || (e = dalloc(&r->sl_vs, C)) != hipSuccess ||
        (e = dalloc(&r->cblk, 2 * (C / RS_CL + 1))) != hipSuccess || (e = dalloc(&r->ccomp, C)) != hipSuccess ||
        (e = dalloc(&r->pblk, RS_PB * (C / RS_CL + 1))) != hipSuccess ||
        (e = hipHostMalloc((void **)&r->host, 4096)) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    // stats, out_bytes and counts share one block, zeroed by one memset per call
    r->out_bytes = r->stats + UDPDK_RS_N;
    r->counts = reinterpret_cast<uint32_t *>(r->stats + UDPDK_RS_N + 1);
    // rocPRIM temporary storage for the largest call (sorts of u64 keys / u32 values, u32 scan,
    // u64 max scan)
    size_t t[7] = {0, 0, 0, 0, 0, 0, 0};
    if ((e = rocprim::radix_sort_pairs(nullptr, t[0], r->k1, r->k1s, r->v1s, r->v2s, C, 0, 64)) != hipSuccess ||
        (e = rocprim::radix_sort_pairs(nullptr, t[1], r->dk, r->dks, r->v1s, r->v2s, C, 0, 32)) != hipSuccess ||
        (e = rocprim::exclusive_scan(nullptr, t[2], r->sizes, r->offs, 0u, C, rocprim::plus<uint32_t>())) != hipSuccess ||
        (e = rocprim::radix_sort_pairs(nullptr, t[3], r->rk, r->rks, r->rv, r->rvs, C2, 0, 64)) != hipSuccess ||
        (e = rocprim::inclusive_scan(nullptr, t[4], r->rk, r->rx, C2, rocprim::maximum<unsigned long long>())) != hipSuccess ||
        (e = rocprim::select(nullptr, t[5], rocprim::counting_iterator<uint32_t>(0u), r->frag_list, r->counts, C,
                             IsFrag{nullptr})) != hipSuccess ||
        (e = rocprim::select(nullptr, t[6], rocprim::counting_iterator<uint32_t>(0u), r->perm, r->counts, C,
                             HasDone{nullptr})) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    r->tmp_bytes = std::max<size_t>(*std::max_element(t, t + 7), 256);
    r->hcap = 1024;                                         // >= 2 x fragments per call, power of 2
    while (r->hcap < 2u * r->cap) r->hcap <<= 1;
    if ((e = dalloc(&r->hset, r->hcap)) != hipSuccess || (e = dalloc(&r->rtab, 2 * (size_t)r->hcap)) != hipSuccess ||
        (e = dalloc(&r->gset, r->hcap)) != hipSuccess || (e = hipMemset(r->gset, 0, r->hcap * 8)) != hipSuccess ||
        (e = hipMemset(r->hset, 0, r->hcap * 8)) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    if ((e = hipMalloc(&r->tmp, r->tmp_bytes)) != hipSuccess) {
        fail(e);
        reasm_destroy(r);
        return rc;
    }
    *out = r;
    return 0;
}

int reasm_run(Reasm *r, hipStream_t st, const udpdk_rx_batch_t *bt, const uint32_t *meta_dev,
              uint64_t tms, udpdk_reasm_out_t *o, int *hip_err, bool inplace)
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
    a.dk = r->dk;
    a.dv = r->dv;
    a.jobs = r->jobs;
    a.assoc_log2 = r->assoc_log2;
    a.nbuckets = r->nbuckets;
    a.pflag = r->pflag;
    a.oc = r->oc;
    a.ob = r->ob;
    a.sb1 = r->sb1;
    a.sb2 = r->sb2;
    a.tf = r->tf;
    a.tl = r->tl;
    a.rk = r->rk;
    a.rv = r->rv;
    a.bsum = r->bsum;
    a.cplx = r->cplx;
    a.sl_k = r->sl_k;
    a.sl_v = r->sl_v;
    a.tpos = r->tpos;
    a.cblk = r->cblk;
    a.pblk = r->pblk;
    a.cl_perm = r->perm;
    a.cl_offs = r->offs;
    a.inplace = inplace ? 1u : 0u;
    if (++r->calls == 0) r->calls = 1;          // 0 marks entries never touched
    a.call = r->calls;
    a.entries = r->entries;
    a.max_entries = r->max_entries;
    a.tab_used = r->tab_used;
    a.ib = bits_for(n - 1u);
    if (!n) RS_HIP(hipMemsetAsync(r->stats, 0, RS_ZERO_WORDS * sizeof(unsigned long long), st));
    // per-position records (written by reasm_scan for a grouped batch, else by reasm_prep after
    // the sorts, when the sort keys sharing their buffers are dead): cap-strided halves
    a.s_i = reinterpret_cast<uint32_t *>(r->k1);
    a.s_src = a.s_i + r->cap;
    a.s_dst = reinterpret_cast<uint32_t *>(r->k1s);
    a.s_id = a.s_dst + r->cap;
    a.s_sig = reinterpret_cast<uint32_t *>(r->k2);
    a.s_meta = a.s_sig + r->cap;
    uint32_t hsize = 1024;                   // the run-key set: >= 2 x fragments, power of 2
    while (hsize < 2u * n && hsize < r->hcap) hsize <<= 1;
    a.hset = r->hset;
    a.hmask = hsize - 1u;
    a.gset = r->gset;
    a.rtab = r->rtab;
    a.rmask = 2u * hsize - 1u;                // >= 4 x fragments: few runs lose their slot
    // the fragment list in arrival order (F to counts[0]), then its sort keys and the run test
    size_t tb = r->tmp_bytes;
    if (n) {
        const uint32_t nfs = (n + RS_FS - 1) / RS_FS;   // blocks of the fragment count (their
        a.fcnt = r->sizes;
        a.nfs = nfs;
        const uint32_t gb = std::max<uint32_t>(1, std::min<uint32_t>((r->entries + RS_BLOCK - 1) / RS_BLOCK, 4096));
        hipLaunchKernelGGL(reasm_fsel_count_bsum, dim3(nfs + gb), dim3(RS_BLOCK), 0, st, a, r->sizes,
                           nfs);                 // counts sit in sizes, dead until the completion list)
        RS_HIP(hipGetLastError());
        a.hset_tag = (a.call - 1u) % 65535u + 1u;
        if (a.hset_tag == 1u) {               // the tags come round: no word may carry one
            RS_HIP(hipMemsetAsync(r->hset, 0, (size_t)r->hcap * sizeof(unsigned long long), st));
            RS_HIP(hipMemsetAsync(r->gset, 0, (size_t)r->hcap * sizeof(unsigned long long), st));
        }
        hipLaunchKernelGGL(reasm_scan, dim3((n + RS_CL - 1) / RS_CL), dim3(RS_BLOCK), 0, st, a);
        RS_HIP(hipGetLastError());
    }
    // Flow analysis and the parallel flows (see the top of this file). Fk = RS_F_DEV: the
    // grouped path launched speculatively (grids sized for n, F read on the device, every kernel
    // returning at once if the batch is not grouped), so a grouped batch makes no host round trip
    // between the run test and the stats read-back.
    // Completion list + output offsets + emit (the grouped path's list by clist_count/write, else a
    // sort by origin + sizes + scan). spec: launched before the read-back (grids from the batch
    // size, counts from the device, see SpecTail).
    const SpecTail g_spec{r->counts, r->stats, (unsigned long long)r->out_cap, inplace ? 1u : 0u, r->counts + 5};
    auto tail = [&](bool grp, uint32_t Fn, uint32_t Cn, bool spec) -> int {
        SpecTail g{nullptr, nullptr, 0, 0u, nullptr};
        if (spec) g = g_spec;
        if (grp) {
            // speculative: the list was written beside reasm_ec (reasm_ec_clist, from reasm_scan's
            // chunk counts: no flow went to the table); else counted and written here (the serial
            // path's completions)
            const uint32_t nb = (Fn + RS_CL - 1) / RS_CL;
            if (!spec) {
                hipLaunchKernelGGL(reasm_clist_count, dim3(nb), dim3(RS_BLOCK), 0, st, (const uint32_t *)r->dk,
                                   (const ReasmDone *)r->done, Fn, r->sizes, g, 0u);
                hipLaunchKernelGGL(reasm_clist_write, dim3(nb), dim3(RS_BLOCK), 0, st, (const uint32_t *)r->dk,
                                   (const ReasmDone *)r->done, Fn, (const uint32_t *)r->sizes, r->perm, r->offs, g,
                                   0u);
            }
            RS_HIP(hipGetLastError());
        } else {
            // origin order: each completion's record position at its origin, then the list over
            // the origins as the grouped path makes it over positions (a sort by origin before)
            const uint32_t gF = std::max<uint32_t>(1, std::min<uint32_t>((Fn + RS_BLOCK - 1) / RS_BLOCK, 4096));
            const uint32_t nb = (n + RS_CL - 1) / RS_CL;
            RS_HIP(hipMemsetAsync(r->dks, 0xFF, (size_t)n * sizeof(uint32_t), st));
            hipLaunchKernelGGL(reasm_by_origin, dim3(gF), dim3(RS_BLOCK), 0, st, (const uint32_t *)r->dk, Fn,
                               r->dks);
            hipLaunchKernelGGL(reasm_clist_count, dim3(nb), dim3(RS_BLOCK), 0, st, (const uint32_t *)r->dks,
                               (const ReasmDone *)r->done, n, r->sizes, g, 1u);
            hipLaunchKernelGGL(reasm_clist_write, dim3(nb), dim3(RS_BLOCK), 0, st, (const uint32_t *)r->dks,
                               (const ReasmDone *)r->done, n, (const uint32_t *)r->sizes, r->perm, r->offs, g,
                               1u);
            RS_HIP(hipGetLastError());
        }
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
        ea.g = g;
        ea.cksum_zero = (r->flags & UDPDK_FRAG_CKSUM_DPDK) ? 1u : 0u;
        // (a grid of 2048 or 4096 workgroups, one resident generation with longer per-wave
        // pipelines, measured even or slower: same-box A/B, 4 pairs)
        const uint32_t ge = std::max<uint32_t>(1, std::min<uint32_t>((Cn + RS_WAVES - 1) / RS_WAVES, 8192));
        if (g.inplace)
            hipLaunchKernelGGL(reasm_emit_either, dim3(ge), dim3(RS_BLOCK), 0, st, ea,
                               const_cast<uint8_t *>(bt->frames_dev));
        else
            hipLaunchKernelGGL(reasm_emit, dim3(ge), dim3(RS_BLOCK), 0, st, ea);
        RS_HIP(hipGetLastError());
        return 0;
    };
    // at most 256 workgroups: each adds its six block totals to the call's stats words with
    // agent-scope atomics on the same six addresses, which serialise (2048 workgroups: 27 us)
    auto process = [&](uint32_t Fk, uint32_t Fgrid) -> int {
        const uint32_t gF = std::max<uint32_t>(1, std::min<uint32_t>((Fgrid + RS_BLOCK - 1) / RS_BLOCK, 256));
        hipLaunchKernelGGL(reasm_process, dim3(gF), dim3(RS_BLOCK), 0, st, a, Fk);
        RS_HIP(hipGetLastError());
        return 0;
    };
    auto analysis = [&](uint32_t Fk, uint32_t Fgrid, bool grp) -> int {
        const uint32_t gF = std::max<uint32_t>(1, std::min<uint32_t>((Fgrid + RS_BLOCK - 1) / RS_BLOCK, 4096));
        // (the bucket summary: made by reasm_fsel_count_bsum at the call's start; the table and
        // the complex-flow counts are untouched until here, a speculative grouped analysis that
        // found the batch not grouped having returned at once)
        // (grouped: the flows were walked by reasm_scan)
        const uint32_t gfl = std::max<uint32_t>(1, std::min<uint32_t>((Fgrid + RS_FLOW_CHUNK - 1) / RS_FLOW_CHUNK, 2048));
        if (!grp) hipLaunchKernelGGL(reasm_flows, dim3(gfl), dim3(RS_BLOCK), 0, st, a, Fk);
        RS_HIP(hipGetLastError());
        uint32_t R = 0;                      // overlap records (none when grouped)
        if (!grp) {
            RS_HIP(hipMemcpyAsync(r->host, r->counts, 8, hipMemcpyDeviceToHost, st));
            RS_HIP(hipStreamSynchronize(st));
            R = r->host[1];
        }
        if (R) {
            size_t tbr = r->tmp_bytes;
            RS_HIP(rocprim::radix_sort_pairs(r->tmp, tbr, r->rk, r->rks, r->rv, r->rvs, (size_t)R, 0,
                                             a.ib + bits_for(r->nbuckets - 1u), st));
            const uint32_t gR = std::max<uint32_t>(1, std::min<uint32_t>((R + RS_BLOCK - 1) / RS_BLOCK, 4096));
            hipLaunchKernelGGL(reasm_rec, dim3(gR), dim3(RS_BLOCK), 0, st, a,
                               (const unsigned long long *)r->rks, (const uint32_t *)r->rvs, r->rk, R);
            RS_HIP(hipGetLastError());
            tbr = r->tmp_bytes;
            RS_HIP(rocprim::inclusive_scan(r->tmp, tbr, r->rk, r->rx, (size_t)R,
                                           rocprim::maximum<unsigned long long>(), st));
            hipLaunchKernelGGL(reasm_overlap, dim3(gR), dim3(RS_BLOCK), 0, st, a,
                               (const unsigned long long *)r->rks, (const uint32_t *)r->rvs,
                               (const unsigned long long *)r->rx, R);
            RS_HIP(hipGetLastError());
        }
        if (grp && (r->out || inplace))
            hipLaunchKernelGGL(reasm_ec_clist, dim3(gF + (Fgrid + RS_CL - 1) / RS_CL), dim3(RS_BLOCK), 0, st, a, gF,
                               g_spec);
        else
            hipLaunchKernelGGL(reasm_ec, dim3(gF), dim3(RS_BLOCK), 0, st, a, Fk);
        RS_HIP(hipGetLastError());
        // (grouped: reasm_process only after the read-back, for a batch with a flow through the
        // table; reasm_ec finishes the others)
        if (!grp) {
            if (int e = process(Fk, Fgrid)) return e;
        }
        if (grp && (r->out || inplace))
            if (int e = tail(true, Fgrid, Fgrid, true)) return e;
        // the serial list's size comes back with the stats and counts
        RS_HIP(hipMemcpyAsync(r->host, r->stats, RS_ZERO_WORDS * 8, hipMemcpyDeviceToHost, st));
        RS_HIP(hipStreamSynchronize(st));
        return 0;
    };
    const uint32_t *hc = reinterpret_cast<const uint32_t *>(r->host + 2 * (UDPDK_RS_N + 1));   // counts
    uint32_t F = 0;
    bool grouped = true;
    uint32_t K = 0;                          // fragments on the serial path
    bool read_back = true;                   // the stats block still to be read back
    bool spec_done = false;                  // the speculative tail ran (see SpecTail)
    bool in_place = false;                   // ... and reassembled every datagram in place
    const uint8_t *spec_out = r->out;        // the buffer it wrote to
    const uint64_t spec_cap = r->out_cap;
    memset(o, 0, sizeof(*o));
    if (n) {
        // every key one run in arrival order: the list is already grouped, and no flow's span can
        // overlap another's (each span holds only its own fragments)
        a.grouped = 1u;
        a.order = r->frag_list;
        if (int e = analysis(RS_F_DEV, n, true)) return e;
        F = hc[0];
        grouped = hc[4] == 0u;
        // reasm_ec's quick case: no complex flow, no fallback (every flow ran without the table)
        const bool quick = hc[8] == 0u && hc[3] == 0u;
        {
            uint64_t ob0;
            memcpy(&ob0, r->host + 2 * UDPDK_RS_N, 8);
            const uint64_t c0 = reinterpret_cast<const uint64_t *>(r->host)[UDPDK_RS_DONE];
            const bool spec_grouped = (spec_out || inplace) && grouped && quick && hc[9] == 0u && c0;
            in_place = inplace && spec_grouped && hc[5] == 0u;
            spec_done = in_place || (spec_out && spec_grouped && ob0 + UDPDK_GPU_FRAMES_TAILROOM <= spec_cap);
        }
        if (F && grouped && !quick) {          // flows through the table: the serial list, outcomes
            if (int e = process(F, F)) return e;
            RS_HIP(hipMemcpyAsync(r->host, r->stats, RS_ZERO_WORDS * 8, hipMemcpyDeviceToHost, st));
            RS_HIP(hipStreamSynchronize(st));
        }
        if (F && !grouped) {
            // group by key keeping arrival order: stable sorts by (id, index), then src|dst; the
            // sort keys are then dead and their buffers take the records in sorted order
            a.grouped = 0u;
            a.order = r->v2s;
            // what reasm_scan's walk and reasm_ec (made as if grouped) left in the shared counters
            // and the outcome words (counts[0] = F stays)
            RS_HIP(hipMemsetAsync(r->cplx, 0, (size_t)r->nbuckets * sizeof(uint32_t), st));
            RS_HIP(hipMemsetAsync(r->stats, 0, (UDPDK_RS_N + 1) * sizeof(unsigned long long), st));
            RS_HIP(hipMemsetAsync(r->counts + 2, 0, 8 * sizeof(uint32_t), st));
            const uint32_t gF = std::max<uint32_t>(1, std::min<uint32_t>((F + RS_BLOCK - 1) / RS_BLOCK, 4096));
            hipLaunchKernelGGL(reasm_group, dim3(gF), dim3(RS_BLOCK), 0, st, a, F);
            RS_HIP(hipGetLastError());
            tb = r->tmp_bytes;
            RS_HIP(rocprim::radix_sort_pairs(r->tmp, tb, r->k1, r->k1s, r->frag_list, r->v2s, (size_t)F, 0,
                                             2 * a.ib, st));
            hipLaunchKernelGGL(reasm_prep, dim3(gF), dim3(RS_BLOCK), 0, st, a, F);
            RS_HIP(hipGetLastError());
            if (int e = analysis(F, F, false)) return e;
        }
    }
    if (F) {
        K = hc[2];
        read_back = K != 0;
        if (K) {
            RS_HIP(hipMemsetAsync(r->jobs, 0xFF, (size_t)F * sizeof(ReasmJob), st));   // no store job
            tb = r->tmp_bytes;
            RS_HIP(rocprim::radix_sort_pairs(r->tmp, tb, r->sl_k, r->sl_ks, r->sl_v, r->sl_vs, (size_t)K, 0,
                                             bits_for(n - 1u), st));
            // bucket components side by side when the max_entries test is not in play (it couples
            // every flow through use_entries and the LRU list), else one wave in arrival order
            const bool cc = hc[6] == 0u && r->nbuckets <= RS_CC_MAX && K >= 64u && !r->no_cc;
            if (cc) {
                hipLaunchKernelGGL(reasm_cc, dim3(1), dim3(RS_CC_BLOCK), 0, st, a, (const uint32_t *)r->sl_vs, K,
                                   r->ccomp);
                hipLaunchKernelGGL(reasm_serial, dim3(std::min<uint32_t>(K / 2u, 512u)), dim3(64), 0, st, a,
                                   (const uint32_t *)r->sl_vs, K, (const uint32_t *)r->ccomp);
            } else {
                hipLaunchKernelGGL(reasm_serial, dim3(1), dim3(64), 0, st, a, (const uint32_t *)r->sl_vs, K,
                                   (const uint32_t *)nullptr);
            }
            RS_HIP(hipGetLastError());
        }
    }
    if (read_back) {
        RS_HIP(hipMemcpyAsync(r->host, r->stats, RS_ZERO_WORDS * 8, hipMemcpyDeviceToHost, st));
        RS_HIP(hipStreamSynchronize(st));
    }
    uint64_t ob;
    memcpy(&ob, r->host + 2 * UDPDK_RS_N, 8);
    memcpy(o->stats, r->host, UDPDK_RS_N * 8);
    o->stats[UDPDK_RS_FRAGS] = F;
    o->stats[UDPDK_RS_SERIAL] = K;
    o->stats[UDPDK_RS_SORTED] = F && !grouped ? 1u : 0u;
    const uint32_t Cn = (uint32_t)o->stats[UDPDK_RS_DONE], J = (uint32_t)o->stats[UDPDK_RS_STORED];
    if (Cn && !spec_done) {
        if (ob + UDPDK_GPU_FRAMES_TAILROOM > r->out_cap) {
            if (r->out) RS_HIP(hipFree(r->out));
            r->out = nullptr;
            r->out_cap = 0;
            const uint64_t nc = std::max<uint64_t>(ob + UDPDK_GPU_FRAMES_TAILROOM, 1u << 20) * 2;
            RS_HIP(hipMalloc((void **)&r->out, nc));
            r->out_cap = nc;
        }
        // completions in origin (arrival) order, then their frame offsets. Grouped: positions are
        // in arrival order, so the positions holding one, in order; else a sort by origin
        // (positions without one have all-ones keys and sort last)
        if (int e = tail(grouped, F, Cn, false)) return e;
    }
    if (J) {   // after every read of the entry buffers (reasm_emit)
        StoreArgs sa;
        sa.frames = bt->frames_dev;
        sa.offset = bt->offset_dev;
        sa.rsrc_bytes = a.rsrc_bytes;
        sa.ebuf = r->ebuf;
        sa.stride = r->stride;
        sa.jobs = r->jobs;
        sa.J = F;                  // positional: waves skip positions without a job
        const uint32_t gs = std::max<uint32_t>(1, std::min<uint32_t>((F + RS_WAVES - 1) / RS_WAVES, 8192));
        hipLaunchKernelGGL(reasm_store, dim3(gs), dim3(RS_BLOCK), 0, st, sa);
        RS_HIP(hipGetLastError());
    }
    RS_HIP(hipStreamSynchronize(st));
    o->batch.frames_dev = in_place ? bt->frames_dev : r->out;
    o->batch.frames_bytes = in_place ? bt->frames_bytes : Cn ? ob : 0;
    o->batch.offset_dev = r->out_off;
    o->batch.length_dev = r->out_len;
    o->batch.ptype_dev = r->out_ptype;
    o->batch.n = Cn;
    o->origin_dev = r->out_origin;
    return 0;
}

} // namespace udpdk
