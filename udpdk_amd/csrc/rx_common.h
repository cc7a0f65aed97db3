// rx_common.h — kernel argument blocks and launch constants shared by the HIP kernels and the
// C-ABI host code (udpdk_gpu.hip). Device-internal; not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace udpdk {

constexpr int RX_BLOCK  = 256;              // rx_classify workgroup (4 waves)
constexpr int RX_WAVES  = RX_BLOCK / 64;
constexpr int RX_UNROLL = 4;                // 16-byte chunk loads in flight per lane
#ifndef UDPDK_RX_ROUND
#define UDPDK_RX_ROUND 1024
#endif
constexpr uint32_t RX_TILE_MIN = UDPDK_RX_ROUND;   // frames per tile (histogram granularity)
constexpr uint32_t RX_TILE_MAX = 8192;   // classify LDS: <= 143 KiB at 16384 lanes
#ifndef UDPDK_RX_HIST_CAP
#define UDPDK_RX_HIST_CAP (1u << 21)
#endif
constexpr uint32_t RX_HIST_CAP = UDPDK_RX_HIST_CAP;  // target bound on lanes x tiles
#ifndef UDPDK_SCAN_MIN_WG
#define UDPDK_SCAN_MIN_WG 128u                // rx_scan_cols: fewest workgroups before narrowing columns
#endif
#ifndef UDPDK_CLS_BLOCK
#define UDPDK_CLS_BLOCK 256
#endif
#ifndef UDPDK_CLS_WPE
#define UDPDK_CLS_WPE 4                      // rx_classify minimum waves per SIMD (VGPR budget)
#endif
constexpr int CLS_BLOCK = UDPDK_CLS_BLOCK;  // rx_classify workgroup
constexpr int CLS_WAVES = CLS_BLOCK / 64;

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_TOP_BLOCK = 1024;
constexpr uint32_t COMPACT1_DIRECT_TILES = 4096; // rx_compact1 sums its predecessors' counts itself
constexpr uint32_t SCAN_COL_CHUNK = 32;     // tiles per chunk of the 3-pass column scan
constexpr uint32_t SCAN_SMALL_MAX = 16384;  // single-workgroup scan up to this many elements
constexpr uint32_t SCAN_SMALL_TILES = 32;   // ... and this many tiles (serial per lane)

constexpr int TX_BLOCK = 256;

// rx_classify LDS carve (one dynamic array, 16-byte aligned offsets: cdna_hip_programming.md
// Guideline 17): the tail pass's per-wave arrays (chunk starts, frame offsets, datagram ends);
// per-wave counter rows; the descriptors of one or two rounds of RX_ROUND frames (offset,
// length | ptype bit); the tile's per-lane delivery histogram; the tile's verdict words; the
// round's datagram ends + window sums (frames whose UDP checksum waits for the tail pass);
// the round's port-table lookups (dst port, dst IPv4).
constexpr uint32_t RX_ROUND = UDPDK_RX_ROUND;     // frames per descriptor-staging / tail round
constexpr int TP_OFF      = 0;                    // [CLS_WAVES][3][64] chunk base, datagram left, mark
constexpr int CNT_OFF     = TP_OFF + CLS_WAVES * 3 * 64 * 4;     // [CLS_WAVES][16] counter rows
constexpr int DSC_OFF     = CNT_OFF + CLS_WAVES * 16 * 4;

// descriptor buffers: one round for a single-round tile, two (double-buffered) otherwise
__host__ __device__ constexpr uint32_t classify_dsc_bufs(uint32_t tile_frames)
{
    return tile_frames > RX_ROUND ? 2u : 1u;
}

// verdict words staged in LDS: the whole tile when it is one round (stored once at the tile end,
// 16 B per lane), else one round (each round stored at the end of its demux pass)
__host__ __device__ constexpr uint32_t classify_stage_frames(uint32_t tile_frames)
{
    return tile_frames > RX_ROUND ? RX_ROUND : tile_frames;
}

// LDS words of the tile histogram: n_lanes, or half as many u16 pairs (hist16), rounded up to 4
__host__ __device__ constexpr uint32_t classify_hist_words(uint32_t n_lanes, bool hist16)
{
    return ((hist16 ? (n_lanes + 1u) >> 1 : n_lanes) + 3u) & ~3u;
}

__host__ __device__ constexpr uint32_t classify_lds_bytes(uint32_t n_lanes, uint32_t tile_frames, bool hist16 = false)
{
    return (uint32_t)DSC_OFF + 8u * RX_ROUND * classify_dsc_bufs(tile_frames) +
           4u * classify_hist_words(n_lanes, hist16) + 4u * classify_stage_frames(tile_frames) +
           4u * RX_ROUND + 8u * RX_ROUND;
}
// Span sweep (rx_classify<2, 0>, RxArgs::span): per wave a ring of two 1 KiB blocks of the step's
// byte span plus a 64-byte copy of the even block's first pieces (a window that wraps the ring
// reads on into it), after the classify carve
constexpr uint32_t SPAN_RING_DW = 2u * 256u + 16u;
constexpr uint32_t SPAN_LDS_BYTES = (uint32_t)CLS_WAVES * SPAN_RING_DW * 4u;
constexpr uint32_t SPAN_MIN_AVG = 96;        // a step sweeps its span when its frames average this
constexpr uint32_t SPAN_MAX_GAP = 128;       // ... and each frame starts < this after the previous ends

// Port table entry (16 B per raw port): x = bindings on the port, y = index of the first in the
// binding array, z/w = the first binding itself (ip, sockfd | reuse << 31), so single-binding
// ports demultiplex with one load. Binding array entries: x = raw IPv4, y = sockfd | reuse << 31.
struct RxArgs {
    const uint8_t  *frames;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *ptype;
    const uint4    *port_tab;
    const uint2    *binds;
    uint32_t *meta;
    uint32_t *hist;       // [n_tiles][n_lanes] per-tile per-lane delivery counts (tile-major)
    uint32_t *tile_cnt;   // [n_tiles][16] per-tile counters
    unsigned long long *dbg;        // diagnostic stamps (UDPDK_STAMPS builds), may be null
    uint32_t key_bits;
    uint32_t frames_bytes;
    uint32_t rsrc_bytes;  // buffer-resource range (frames_bytes rounded up to 16)
    uint32_t n;
    uint32_t tile_frames;
    uint32_t n_tiles;
    uint32_t lane_mask;
    uint32_t n_lanes;
    uint32_t hist16;      // hist rows are u16[(n_lanes + 1) & ~1] (multi-lane, no fan-out)
    // single lane, no fan-out, one-round 1024-frame tiles: each tile also writes its deliveries
    // at tile x tile_frames + rank, their place if every earlier tile delivered all its frames
    // (rx_compact1 then only checks that); null otherwise
    uint32_t *spec_pkt;
    uint32_t spec_cap;
    uint32_t spec_epoch;
    unsigned long long *spec_nonfull;   // [UDPDK_SPEC_WORDS] atomicMax of epoch << 32 | ~tile, tiles not full
    // fused completion (spec entries, at most UDPDK_FUSE_MAX_TILES tiles): the last workgroup
    // writes lane_off / total (rx_compact1's work); fan-in words [16 x (UDPDK_FUSE_SHARDS + 1)],
    // zero between calls; null: rx_compact1 follows
    unsigned long long *fuse;
    uint32_t *lane_off;
    uint32_t *total;
    // host-visible kernel hints (pinned memory, may be null): hint[UDPDK_HINT_TAIL] = seq when the
    // call ran a tail pass, hint[UDPDK_HINT_NONFULL] = seq when a tile before the last was not full
    uint32_t *hint;
    uint32_t seq;
    // a bind table of at most UDPDK_INLINE_PORTS bound ports rides in the arguments (inl != 0):
    // the demux compares the frame's raw dst port with inl_port[0 .. n_inl) and takes that port's
    // 16-byte entry from inl_ent, no port-table load (the bindings list still comes from binds)
    uint32_t inl;
    uint32_t n_inl;
    uint32_t inl_port[8];
    uint4 inl_ent[8];
    // rx_classify<2, 0> with one-round tiles: a step whose frames lie in ascending order, each
    // within SPAN_MAX_GAP bytes of the previous one's end, reads its whole byte span once on a
    // line grid (header windows taken from the sweep through an LDS ring, UDP checksums from
    // prefix sums over the span) instead of per-frame windows and tail chunks. The ring follows
    // the classify carve (SPAN_LDS_BYTES more dynamic LDS)
    uint32_t span;
};
#define UDPDK_INLINE_PORTS 8u
#define UDPDK_FUSE_SHARDS 8u

// Launch completion by the last workgroup (rx_classify's fused single-lane completion, rss_hash's
// fused queue bases): called by ONE thread of each workgroup after every wave of it drained its
// written-through stores behind a barrier (cdna_hip_programming.md Guideline 16). Adds
// {1 arrival << 48 | payload} to the fan-in word of its shard (tile mod 8, fuse[16 s], 128 B
// apart: 1024 arrivals on one word serialise, tools/probe/ticket_probe.hip); the shard's last
// arrival adds the shard's payload sum to the top word fuse[16 x 8]; the top's last arrival
// returns true with the launch's payload sum (< 2^48) in *fin. Each word is zeroed again by its
// last arrival, so the next launch on the same words starts from zeros.
// *left (optional): how many of the shard's workgroups arrive after this one.
__device__ __forceinline__ bool fanin_arrive(unsigned long long *fuse, uint32_t tile, uint32_t n_tiles,
                                             unsigned long long payload, unsigned long long *fin,
                                             uint32_t *left = nullptr)
{
    constexpr unsigned long long LOW = (1ull << 48) - 1ull;
    const uint32_t s = tile & (UDPDK_FUSE_SHARDS - 1u);
    const uint32_t ns = (n_tiles - 1u - s) / UDPDK_FUSE_SHARDS + 1u;     // tiles of shard s
    const unsigned long long mine = (1ull << 48) | payload;
    unsigned long long *sw = fuse + 16u * s;
    const unsigned long long now = __hip_atomic_fetch_add(sw, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + mine;
    if (left) *left = ns - (uint32_t)(now >> 48);
    if ((uint32_t)(now >> 48) != ns) return false;
    __hip_atomic_store(sw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long m2 = (1ull << 48) | (now & LOW);
    unsigned long long *tw = fuse + 16u * UDPDK_FUSE_SHARDS;
    const unsigned long long now2 = __hip_atomic_fetch_add(tw, m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + m2;
    if ((uint32_t)(now2 >> 48) != (n_tiles < UDPDK_FUSE_SHARDS ? n_tiles : UDPDK_FUSE_SHARDS)) return false;
    __hip_atomic_store(tw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *fin = now2 & LOW;
    return true;
}
#define UDPDK_FUSE_MAX_TILES 4096u           // fused single-lane calls (the repair's LDS tile bases)
// Words after the fan-in lines (fuse[16 k], one 128-byte line each): the repair of a fused call
// with a short tile (rx_classify's classify_complete). FLAG = max of the call epochs that had a
// short tile, DONE = epoch of the latest call whose repair opened, WORK = epoch << 32 | next chunk.
#define UDPDK_FUSE_FLAG (16u * (UDPDK_FUSE_SHARDS + 1u))
#define UDPDK_FUSE_DONE (16u * (UDPDK_FUSE_SHARDS + 2u))
#define UDPDK_FUSE_WORK (16u * (UDPDK_FUSE_SHARDS + 3u))
#define UDPDK_FUSE_LINES (UDPDK_FUSE_SHARDS + 4u)
#ifndef UDPDK_FIX_HELPERS
#define UDPDK_FIX_HELPERS 8u                // repair helpers: a shard's last arrivals that may join
#endif
#define UDPDK_FIX_CHUNK 4u                   // tiles per repair work item
#define UDPDK_FIX_SPIN 200000u               // a helper's bounded wait for the call's last arrival
#define UDPDK_HINT_TAIL 0
#define UDPDK_HINT_NONFULL 16                // its own 64-byte line
#define UDPDK_HINT_DONE 32                   // seq of the latest call whose first tile ran
#ifndef UDPDK_SPEC_COMPACT
#define UDPDK_SPEC_COMPACT 1
#endif
#define UDPDK_SPEC_WORDS 64u                 // flag words of the speculative compaction
#ifndef UDPDK_COMPACT1_SPEC_GRID
#define UDPDK_COMPACT1_SPEC_GRID 256u        // rx_compact1 workgroups after a speculative classify
#endif

struct ScanArgs {
    uint32_t *hist;
    uint32_t *partial;
    uint32_t *lane_off;
    uint32_t *total;
    uint32_t *tot;        // rx_scan_cols: [n_lanes] lane totals
    uint32_t n_elems;
    uint32_t n_tiles;
    uint32_t n_lanes;
    // rx_scan_cols only: absolute positions out (base[tile][lane] = lane_off + column prefix), the
    // lane-block look-back words (epoch << 32 | flag << 30 | value) and the block ticket
    uint32_t *base;
    unsigned long long *agg;
    uint32_t *ticket;
    uint32_t epoch;
    uint32_t hist16;
    uint32_t row_mask;    // rx_scan_cols: base rows written only for tiles t with t & row_mask == 0
    unsigned long long *dbg;   // diagnostic stamps (UDPDK_STAMPS builds), may be null
};

// rx_scan_cols<B>: one launch, workgroup = a block of 2^lb lanes x every tile (B = 512 or 1024
// threads); each thread keeps up to scan_cols_tpt(B) tiles of one lane in registers, so tiles <=
// scan_cols_tpt(B) * (B >> lb): 16384 tiles at one lane per workgroup, whatever B.
__host__ __device__ constexpr uint32_t scan_cols_tpt(uint32_t block) { return 16384u / block; }
constexpr uint32_t SCAN_COLS_MAX_TILES = 16384;

struct ScatterArgs {
    const uint32_t *meta;
    const uint32_t *base;  // [tiles][lanes] absolute start of each tile's deliveries per lane
    uint32_t *total;
    const uint8_t  *frames;
    const uint32_t *offset;
    const uint4    *port_tab;
    const uint2    *binds;
    uint32_t *lane_pkt;
    uint32_t n;
    uint32_t tile_frames;
    uint32_t n_tiles;
    uint32_t n_lanes;
    uint32_t lane_mask;
    uint32_t key_bits;
    uint32_t lane_cap;
    uint32_t row_step;         // base row of scatter tile s: s x row_step (classify tiles per scatter tile)
    unsigned long long *dbg;   // diagnostic stamps (UDPDK_STAMPS builds), may be null
};

// Single-lane compaction (rx_compact1): lane_pkt = indices of delivered frames in frame order,
// from the classify kernel's verdict words and per-tile delivery counts (hist, one lane).
struct Compact1Args {
    const uint32_t *meta;
    const uint32_t *tile_count;   // [n_tiles] deliveries per tile
    uint32_t *lane_pkt;
    uint32_t *lane_off;           // [2]
    uint32_t *total;
    uint32_t n;
    uint32_t tile_frames;
    uint32_t n_tiles;
    uint32_t lane_cap;
    const uint32_t *base;         // [n_tiles] exclusive prefix of tile_count (rx_tile_base), or null
    uint32_t spec;                // rx_classify wrote speculative entries (RxArgs::spec_pkt)
    uint32_t spec_epoch;
    const unsigned long long *spec_nonfull;
    uint32_t *hint;               // see RxArgs::hint (compact1 reports a tile that was not full)
    uint32_t seq;
};

struct TxArgs {
    const uint8_t  *payload;
    const uint32_t *payload_off;
    const uint16_t *payload_len;
    const int32_t  *sockfd;
    const uint32_t *dst_ip;
    const uint16_t *dst_port;
    const uint32_t *frame_off;
    const uint4    *slots;     // x = ip, y = udp_port, z = bound
    uint8_t *frames;
    uint32_t n;
    uint32_t n_slots;
    uint32_t payload_bytes;
    uint32_t payload_rsrc;
    uint32_t frames_bytes;
    uint32_t src_ip;
    uint32_t mtu;              // 0: no fragmentation; else IPv4 MTU ((mtu - 20) % 8 == 0)
    uint32_t mac_lo[3];        // 12 MAC bytes: dst(6) src(6) as three LE dwords
    uint32_t parts;            // waves sharing one group of 64 datagrams' chunk sweep (>= 1)
};

// Payload delivery (rx_gather): lane entries [first, first + count) -> payload slots + source
// addresses (the batch form of udpdk_recvfrom, udpdk_syscall.c:401-488).
constexpr int GATHER_BLOCK = 256;
struct GatherArgs {
    const uint8_t  *frames;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *lane_pkt;
    uint8_t  *payload;
    uint32_t *len_out;
    uint32_t *src_ip;
    uint16_t *src_port;
    uint32_t first;
    uint32_t count;
    uint32_t slot_bytes;
    uint32_t rsrc_bytes;
    uint32_t n;
    const uint32_t *slot_off;   // [count + 1] packed slots (udpdk_gpu_rx_gather_packed), or null
};

// G: tail chunk groups in flight (1, 2); MR: tiles of several rounds, whose next round's
// descriptors are loaded a round ahead (in registers) instead of when they are staged
template <int G, int MR> __global__ void rx_classify(RxArgs a);
__global__ void rx_gather(GatherArgs a);
template <uint32_t B> __global__ void rx_scan_cols(ScanArgs a, uint32_t lb);
__global__ void rx_scan_reduce(ScanArgs a);
__global__ void rx_scan_top(ScanArgs a, uint32_t n_part);
__global__ void rx_scan_down(ScanArgs a);
__global__ void rx_scatter(ScatterArgs a);
template <uint32_t W> __global__ void rx_scatterw(ScatterArgs a);
#ifndef UDPDK_SCATTER_WAVES
#define UDPDK_SCATTER_WAVES 8
#endif
constexpr uint32_t SCATTER_WAVES = UDPDK_SCATTER_WAVES;   // rx_scatterw workgroup: waves per tile
constexpr uint32_t SCATTERW_MAX_LANES = 4096;   // rx_scatterw LDS: (4 + 2 x 8) x lanes bytes
constexpr uint32_t SCATTERW_MV = RX_TILE_MAX / (64 * SCATTER_WAVES);   // verdict words per lane
// rx_scatterw takes G consecutive classify tiles as one scatter tile (the base row of its first):
// fewer (tile, lane) pieces, so fewer partly written lane_pkt lines (config 5: 1.07 M line
// touches at 8192 frames, 0.80 M at 16384), up to this many frames, 16 waves past 8192
#ifndef UDPDK_SCATTER_GROUP_FRAMES
#define UDPDK_SCATTER_GROUP_FRAMES 16384u
#endif
#ifndef UDPDK_SCATTER_MIN_WG
#define UDPDK_SCATTER_MIN_WG 256u               // ... while the grid keeps this many workgroups
#endif
__host__ __device__ constexpr uint32_t scatterw_lds_bytes(uint32_t n_lanes, uint32_t waves = SCATTER_WAVES)
{
    // cursors (at least one word per wave: the key scan's wave totals) + per-wave slice offsets
    // (u16): 80 KiB at 4096 lanes and 8 waves, so two workgroups share a CU's 160 KiB; 144 KiB at
    // 16 waves (one per CU)
    return 4u * (n_lanes > waves ? n_lanes : waves) + 2u * waves * n_lanes;
}
constexpr int SCATTER1_BLOCK = 256;             // rx_scatter: prologue by 4 waves, walk by wave 0
__host__ __device__ constexpr uint32_t scatter1_lds_bytes(uint32_t n_lanes)
{
    return 4u * n_lanes + 64u;                  // cursors
}
__global__ void rx_compact1(Compact1Args a);
__global__ void rx_tile_base(const uint32_t *cnt, uint32_t *base, uint32_t n);
__global__ void rx_counters(const uint32_t *tile_cnt, uint32_t n_tiles, unsigned long long *counters);
// Receive-side scaling (rx_rss.hip).
constexpr uint32_t RSS_BLOCK = 256;
constexpr uint32_t RSS_TILE = 1024;          // frames per workgroup
constexpr uint32_t RSS_RETA_MAX = 512;
constexpr uint32_t RSS_BASE_MAX = 32768;    // histogram entries scanned by one rss_base workgroup
constexpr uint32_t RSS_MAX_QUEUES = 64;
struct RssArgs {
    const uint8_t  *frames;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *ptype;
    const uint16_t *reta;     // [reta_size] queue per redirection entry
    const uint32_t *ktab;     // [12][256] Toeplitz key windows per input byte (host-built)
    uint32_t *hash;           // [n] mbuf.hash.rss
    uint8_t  *qid;            // [n] queue per frame
    uint32_t *hist;           // queue counts per tile -> scanned start positions; [n_queues][tiles]
                              // when qmajor (the rss_base scan), else [tiles][n_queues]
    uint32_t *queue_pkt;      // [n] frame indices grouped by queue
    uint64_t frames_bytes;
    uint32_t rsrc_bytes;
    uint32_t n;
    uint32_t reta_size;       // power of two <= RSS_RETA_MAX
    uint32_t n_queues;        // <= RSS_MAX_QUEUES
    uint32_t q_bits;          // bits of a queue index
    uint32_t hash_types;      // bit 0: IPv4 2-tuple, bit 1: unfragmented IPv4 UDP 4-tuple
    uint32_t n_tiles;
    uint32_t qmajor;
    // fused queue bases (qmajor): the last rss_hash workgroup scans the histogram into
    // queue_off / total / the scatter's bases (fan-in words, zero between calls); null: rss_base
    unsigned long long *fuse;
    uint32_t *queue_off;
    uint32_t *total;
};
__global__ void rss_hash(RssArgs a);
__global__ void rss_scatter(RssArgs a);
__global__ void rss_base(uint32_t *hist, uint32_t n, uint32_t T, uint32_t *queue_off, uint32_t *total);

// RX reassembly (rx_reasm.hip): host-side table object driven by udpdk_gpu_rx_reassemble.
struct Reasm;
int  reasm_create(Reasm **out, int device, uint32_t max_frames, const udpdk_frag_table_cfg_t *cfg,
                  int *hip_err);
void reasm_destroy(Reasm *r);
int  reasm_run(Reasm *r, hipStream_t st, const udpdk_rx_batch_t *bt, const uint32_t *meta_dev,
                uint64_t tms, udpdk_reasm_out_t *o, int *hip_err, bool inplace);

__global__ void tx_build(TxArgs a);

} // namespace udpdk
