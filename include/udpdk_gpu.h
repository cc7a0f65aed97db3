/*
 * udpdk_gpu.h — C ABI of the MI355X (gfx950) batch datapath.
 *
 * This is the drop-in boundary for UDPDK's per-packet hot path. The reference has no plugin
 * registry (udpdk/Makefile:72-81 localises every non-API symbol), so the replacement points are
 * the two function bodies the hot path lives in:
 *
 *   RX  udpdk_poller.c:516-545 (burst loop) + :316-413 reassemble() + :274-298 enqueue/flush
 *       -> udpdk_gpu_rx(): one launch sequence over N frames instead of N reassemble() calls,
 *          producing a verdict word per frame and stable per-socket output lanes (the
 *          equivalent of exch_slots[s].rx_buffer flushed into exch_slots[s].rx_q).
 *   TX  udpdk_syscall.c:314-356 (udpdk_sendto header build + rte_ipv4_cksum)
 *       -> udpdk_gpu_tx_build(): header build + IPv4 checksum + payload copy for N datagrams.
 *
 * The bind table walked by reassemble() (udpdk_bind_table.c:152 btable_get_bindings + the list
 * iterator, list_iterator.c:19-55) is replaced by an immutable flattened snapshot uploaded with
 * udpdk_gpu_bind_snapshot_upload(); the host bind table (see udpdk_api.h) builds it in list order.
 *
 * Conventions
 *   - Plain C types only; no HIP/torch types cross the boundary. Streams are opaque (void*).
 *   - Every entry point returns 0 on success or a negative errno (-EINVAL bad arguments,
 *     -ENOMEM allocation failure, -ENOSPC output capacity exceeded, -EIO HIP failure; the HIP
 *     error code of the last failure is kept in the context, see udpdk_gpu_last_hip_error()).
 *     Nothing aborts. (Reference convention: API calls return -1 + errno, udpdk_syscall.c:23-520;
 *     the datapath itself never reports errors, it logs and drops.)
 *   - Ports and IPv4 addresses are "raw": the 2/4 wire bytes read as a little-endian host
 *     integer, exactly how the reference compares and indexes them (udpdk_poller.c:372-373,
 *     udpdk_bind_table.c:152, udpdk_syscall.c:230).
 *   - Buffers named *_dev are device pointers (from udpdk_gpu_alloc or any hipMalloc on the
 *     context's device); buffers named *_host are host pointers.
 *   - Calls on one context are asynchronous on that context's stream unless stated otherwise.
 *     One host thread per context; contexts on different devices are independent.
 */
#ifndef UDPDK_GPU_H
#define UDPDK_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: udpdk_reasm_out_t stats grew to UDPDK_RS_N = 11 (RS_SERIAL, RS_SORTED);
 *    udpdk_gpu_rx_gather_packed; TX payloads need UDPDK_GPU_FRAMES_TAILROOM readable bytes
 * 3: udpdk_frag_table_cfg_t grew max_entries (the table's LRU limit) and flags (32 bytes) */
#define UDPDK_GPU_ABI_VERSION 3

/* ---------------------------------------------------------------------------------------------
 * Per-frame verdict word (one uint32 per frame, written by udpdk_gpu_rx)
 *
 *   bits  0..3   verdict (enum udpdk_verdict)
 *   bit   4      IPv4 header checksum verifies (RFC 1071 over the fixed 20 B at frame offset 14)
 *   bits  5..6   UDP checksum state (enum udpdk_udp_csum)
 *   bit   7      UDP length bad: dgram_len < 8 or 34 + dgram_len > frame length
 *   bit   8      IHL != 5 (the reference parses at fixed offsets regardless, poller.c:336,:372)
 *   bits  9..15  number of deliveries (fan-out), saturating at 127
 *   bits 16..31  sockfd of the first delivery (the original mbuf's socket; clones follow it)
 * ------------------------------------------------------------------------------------------- */
enum udpdk_verdict {
    UDPDK_V_DELIVERED = 0, /* >= 1 socket matched (poller.c:391-403)                            */
    UDPDK_V_NOT_IPV4  = 1, /* !RTE_ETH_IS_IPV4_HDR(ptype) (poller.c:334, :362-366)               */
    UDPDK_V_FRAG      = 2, /* rte_ipv4_frag_pkt_is_fragmented (poller.c:338); host slow path      */
    UDPDK_V_NOT_UDP   = 3, /* next_proto_id != 17 (poller.c:368-371)                             */
    UDPDK_V_NO_BIND   = 4, /* empty bind list for the raw dst port (poller.c:376-380)            */
    UDPDK_V_NO_MATCH  = 5, /* bind list present, no IP matched (poller.c:406-411)                */
    UDPDK_V_TRUNC     = 6, /* IPv4 by ptype but shorter than the 42 B Eth/IPv4/UDP header, and
                              not a fragment of >= 34 B (those are FRAG: a fragment needs only
                              its IPv4 header); the reference would read past data_len        */
    UDPDK_V_BAD_DESC  = 7  /* offset + length beyond frames_bytes: nothing was read              */
};
#define UDPDK_N_VERDICTS 8

enum udpdk_udp_csum {
    UDPDK_UDP_CSUM_NONE = 0, /* dgram_cksum == 0 (RFC 768 "no checksum") or not a UDP verdict */
    UDPDK_UDP_CSUM_OK   = 1,
    UDPDK_UDP_CSUM_BAD  = 2
};

#define UDPDK_META_VERDICT(m)  ((unsigned)(m) & 0xFu)
#define UDPDK_META_IP_OK(m)    (((unsigned)(m) >> 4) & 1u)
#define UDPDK_META_UDP_CSUM(m) (((unsigned)(m) >> 5) & 3u)
#define UDPDK_META_LEN_BAD(m)  (((unsigned)(m) >> 7) & 1u)
#define UDPDK_META_IHL_NE5(m)  (((unsigned)(m) >> 8) & 1u)
#define UDPDK_META_FANOUT(m)   (((unsigned)(m) >> 9) & 0x7Fu)
#define UDPDK_META_SOCKFD(m)   ((unsigned)(m) >> 16)

/* Counters reduced over a whole udpdk_gpu_rx call (replace the per-drop RTE_LOG WARNINGs,
 * poller.c:363, :369, :378, :410). */
enum udpdk_rx_counter {
    UDPDK_C_VERDICT0   = 0,  /* 0..7: frames per verdict                                     */
    UDPDK_C_DELIVERIES = 8,  /* total (frame, socket) deliveries = lane entries               */
    UDPDK_C_IP_BAD     = 9,  /* IPv4-gated frames whose header checksum fails                 */
    UDPDK_C_UDP_OK     = 10,
    UDPDK_C_UDP_BAD    = 11,
    UDPDK_C_UDP_NONE   = 12, /* UDP-verdict frames carrying dgram_cksum == 0                  */
    UDPDK_C_LEN_BAD    = 13,
    UDPDK_C_IHL_NE5    = 14,
    UDPDK_C_BYTES      = 15, /* sum of frame lengths                                         */
    UDPDK_N_COUNTERS   = 16
};

/* Limits of the GPU path. NUM_SOCKETS_MAX is 1024 in the reference (udpdk_constants.h:12); the
 * lane count is widened here and bounded by the per-workgroup LDS histogram. */
#define UDPDK_GPU_MAX_LANES        16384u
#define UDPDK_GPU_MAX_BINDS        (1u << 20)
#define UDPDK_GPU_MAX_PORT_BINDS   4095u
#define UDPDK_UDP_PORTS            65536u     /* UDP_MAX_PORT, udpdk_constants.h:13 */
/* Readable bytes the RX kernels need after frames_bytes (byte-aligned dword loads of a batch's
 * last frame may end up to 3 bytes past it). */
#define UDPDK_GPU_FRAMES_TAILROOM  16u

/* ---------------------------------------------------------------------------------------------
 * Context
 * ------------------------------------------------------------------------------------------- */
typedef struct udpdk_gpu_ctx udpdk_gpu_ctx;

/* Create a context on `device` with its own stream and workspace sized for batches of up to
 * max_frames frames and up to max_lanes per-socket lanes. Called from udpdk_init(). */
int  udpdk_gpu_ctx_create(int device, uint32_t max_frames, uint32_t max_lanes,
                          udpdk_gpu_ctx **out);
/* Synchronise and free everything. Called from udpdk_cleanup(). NULL is a no-op. */
int  udpdk_gpu_ctx_destroy(udpdk_gpu_ctx *ctx);
int  udpdk_gpu_sync(udpdk_gpu_ctx *ctx);
int  udpdk_gpu_last_hip_error(const udpdk_gpu_ctx *ctx);
int  udpdk_gpu_device_count(int *count);
int  udpdk_gpu_abi_version(void);
/* The context's HIP stream (hipStream_t) as an opaque pointer. */
void *udpdk_gpu_stream(udpdk_gpu_ctx *ctx);

/* Device / pinned-host memory helpers on the context's device (so callers need no HIP). */
int  udpdk_gpu_alloc(udpdk_gpu_ctx *ctx, size_t bytes, void **dev);
int  udpdk_gpu_free(udpdk_gpu_ctx *ctx, void *dev);
int  udpdk_gpu_host_alloc(udpdk_gpu_ctx *ctx, size_t bytes, void **host); /* pinned */
int  udpdk_gpu_host_free(udpdk_gpu_ctx *ctx, void *host);
int  udpdk_gpu_memset(udpdk_gpu_ctx *ctx, void *dev, int value, size_t bytes);       /* async */
int  udpdk_gpu_h2d(udpdk_gpu_ctx *ctx, void *dev, const void *host, size_t bytes);   /* async */
int  udpdk_gpu_d2h(udpdk_gpu_ctx *ctx, void *host, const void *dev, size_t bytes);   /* async */

/* ---------------------------------------------------------------------------------------------
 * Bind snapshot (replaces sock_bind_table[65536] of list<bind_info>, udpdk_bind_table.c:17-18,
 * walked at poller.c:376-405). Bindings of one raw port are contiguous and in list order
 * (head -> tail: ANY bindings lpush'ed, specific ones rpush'ed, udpdk_bind_table.c:119-124).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t ip;      /* raw IPv4 (bind_info.ip_addr.s_addr, udpdk_types.h:33); 0 = INADDR_ANY */
    int32_t  sockfd;  /* bind_info.sockfd (udpdk_types.h:32), 0..65535                         */
    uint32_t reuse;   /* bind_info.reuse_addr || bind_info.reuse_port (poller.c:396)            */
} udpdk_binding_t;

/* Socket slot state needed by TX header build (exch_slot_info, udpdk_types.h:40-47). */
typedef struct {
    uint32_t ip;       /* raw bound IPv4, 0 = ANY                                              */
    uint32_t udp_port; /* raw bound UDP port (low 16 bits)                                     */
    uint32_t bound;    /* slot did bind (explicitly or by sendto auto-bind)                    */
} udpdk_slot_t;

typedef struct {
    const uint32_t        *port_first;  /* [65536] index of the port's first binding          */
    const uint16_t        *port_count;  /* [65536] bindings on the port (0 = none)            */
    const udpdk_binding_t *binds;       /* [n_binds]                                          */
    uint32_t               n_binds;
    uint32_t               n_lanes;     /* > max(sockfd & lane_mask) over all bindings        */
    uint32_t               lane_mask;   /* 0xFFFFFFFF: lanes keyed by full sockfd;
                                           0xFF: compat mode, the reference's (uint8_t) slot
                                           index (poller.c:294, :393)           */
    const udpdk_slot_t    *slots;       /* [n_slots] for TX, may be NULL                      */
    uint32_t               n_slots;
    uint64_t               version;     /* bumped by every bind/close on the host             */
} udpdk_bind_snapshot_t;

/* Upload (host arrays -> device, synchronous on the context stream). */
int udpdk_gpu_bind_snapshot_upload(udpdk_gpu_ctx *ctx, const udpdk_bind_snapshot_t *snap);

/* ---------------------------------------------------------------------------------------------
 * RX: parse + validate + checksum + port demux + per-socket lanes
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    const uint8_t  *frames_dev;   /* frame bytes (rte_pktmbuf_mtod, Ethernet first, no FCS),
                                     16-byte aligned base, readable for frames_bytes +
                                     UDPDK_GPU_FRAMES_TAILROOM bytes (tailroom, as every DPDK
                                     mbuf data room has); bytes past frames_bytes never
                                     affect a result                                          */
    uint64_t        frames_bytes; /* < 2^32                                                    */
    const uint32_t *offset_dev;   /* [n] byte offset of each frame in frames_dev               */
    const uint16_t *length_dev;   /* [n] data_len of each frame                                */
    const uint32_t *ptype_dev;    /* [n] mbuf packet_type, or NULL: derived from ether_type
                                     (0x0800 -> L2_ETHER|L3_IPV4|L4_UDP, else L2_ETHER)        */
    uint32_t        n;
} udpdk_rx_batch_t;

typedef struct {
    uint32_t *meta_dev;      /* [n] verdict words                                             */
    uint32_t *lane_off_dev;  /* [n_lanes + 1] exclusive prefix of per-lane delivery counts    */
    uint32_t *lane_pkt_dev;  /* [lane_cap] frame indices grouped by lane, arrival order kept  */
    uint32_t  lane_cap;
} udpdk_rx_out_t;

typedef struct {
    uint64_t counters[UDPDK_N_COUNTERS];
    uint32_t deliveries;     /* == lane_off[n_lanes]                                           */
    uint32_t overflow;       /* deliveries > lane_cap: lane_pkt holds only the first lane_cap  */
} udpdk_rx_stats_t;

/* Enqueue the RX pipeline for one batch on the context stream (async): rx_classify, then, with
 * one lane and no fan-out in the snapshot, nothing more (the last classify workgroup completes
 * the lane) or rx_compact1, else rx_scan + rx_scatter. meta, lane_off and lane_pkt are complete
 * when the stream reaches the end of the sequence. Which single-lane form runs (and how many
 * tail chunk groups classify keeps in flight) follows hints the kernels leave in pinned host
 * memory about the context's recent calls; every form gives the same results for any batch.
 * A fresh context starts on the two-launch form.
 *
 * Tailroom contract: batch->frames_dev must be readable for frames_bytes +
 * UDPDK_GPU_FRAMES_TAILROOM bytes. The kernels read frame bytes with byte-aligned dword loads
 * that are range-checked against frames_bytes rounded up to a dword, so the last frame of a batch
 * whose frames_bytes % 4 != 0 may be read up to 3 bytes past frames_bytes (never used in a
 * result). The library cannot check the allocation size behind a device pointer: a buffer that
 * ends exactly at frames_bytes may fault (tests/test_gpu_rx.py::test_tailroom_exact_allocation). */
int udpdk_gpu_rx(udpdk_gpu_ctx *ctx, const udpdk_rx_batch_t *batch, const udpdk_rx_out_t *out);
/* Pipelining: with depth d in 2..4, consecutive udpdk_gpu_rx calls rotate over d internal
 * streams with their own workspaces, so one batch's launch, prologue and compaction overlap the
 * other batches' streaming (3 is fastest for 1 M x 64 B batches). Calls must then not share
 * output buffers with the d - 1 previous calls still in flight. Depth 1 (default): every call in
 * order on the context stream. Synchronises. */
int udpdk_gpu_pipeline_depth(udpdk_gpu_ctx *ctx, int depth);
/* Make the context stream (udpdk_gpu_stream) wait, on the device, for all work enqueued so far on
 * the other pipes (no host wait). memset/h2d/d2h/tx_build/rx_host join implicitly. */
int udpdk_gpu_join(udpdk_gpu_ctx *ctx);
/* Counters of the last udpdk_gpu_rx (reduced from its per-tile counter rows by one small kernel
 * launched here, so batches nobody asks statistics for pay nothing), then wait for the stream.
 * Returns -ENOSPC on lane overflow. */
int udpdk_gpu_rx_stats(udpdk_gpu_ctx *ctx, udpdk_rx_stats_t *stats);

/* End-to-end variant for host-resident batches (the real poller's situation: frames arrive in
 * host mbufs): pinned staging, H2D, the RX pipeline, D2H of meta and lanes (lane_pkt: only the
 * min(deliveries, lane_cap) entries made). Synchronous. frames_host etc. follow
 * udpdk_rx_batch_t; outputs are host arrays. */
int udpdk_gpu_rx_host(udpdk_gpu_ctx *ctx,
                      const uint8_t *frames_host, uint64_t frames_bytes,
                      const uint32_t *offset_host, const uint16_t *length_host,
                      const uint32_t *ptype_host, uint32_t n,
                      uint32_t *meta_host, uint32_t *lane_off_host,
                      uint32_t *lane_pkt_host, uint32_t lane_cap,
                      udpdk_rx_stats_t *stats);

/* Device view of the batch the last udpdk_gpu_rx_host call staged (frames, descriptors) and its
 * verdict words, valid until the next udpdk_gpu_rx_host[_async] call: for udpdk_gpu_rx_gather
 * and udpdk_gpu_rx_reassemble on frames already on the device (the socket layer's poller). */
int udpdk_gpu_rx_host_batch(udpdk_gpu_ctx *ctx, udpdk_rx_batch_t *batch, const uint32_t **meta_dev);

/* Asynchronous form of udpdk_gpu_rx_host for a stream of host-resident batches: the staging,
 * H2D, RX pipeline, counter reduction and D2H of meta, lane_off and lane_pkt[0, lane_cap) are
 * enqueued on the next pipe (udpdk_gpu_pipeline_depth) with its own staging buffers, and the
 * call returns; with depth 2 one batch's PCIe copies overlap the other's kernels and copies in
 * the opposite direction. At most `depth` calls are outstanding (a call first completes the one
 * that used its pipe). Host inputs must stay untouched, and outputs and *stats are valid, only
 * once udpdk_gpu_rx_host_wait returns (or a later call reuses the pipe). */
int udpdk_gpu_rx_host_async(udpdk_gpu_ctx *ctx,
                            const uint8_t *frames_host, uint64_t frames_bytes,
                            const uint32_t *offset_host, const uint16_t *length_host,
                            const uint32_t *ptype_host, uint32_t n,
                            uint32_t *meta_host, uint32_t *lane_off_host,
                            uint32_t *lane_pkt_host, uint32_t lane_cap,
                            udpdk_rx_stats_t *stats);
/* Complete every outstanding udpdk_gpu_rx_host_async call (oldest first). */
int udpdk_gpu_rx_host_wait(udpdk_gpu_ctx *ctx);

/* Poller internals, for udpdk_poll_rx's pipelined form (a large host batch cut into chunks at
 * burst boundaries, each chunk's RX, gather and payload copy on its own pipe): the same host RX
 * as udpdk_gpu_rx_host_async on an explicit pipe (1 .. 3), and the device view, gather and
 * copies of that chunk on that pipe's stream with no joins across pipes, so one chunk's payload
 * D2H overlaps the next chunk's frame H2D. udpdk_gpu_pipe_wait completes the pipe's stream and
 * the stats of its RX. offset_base: subtracted from every offset_host entry (a chunk of a larger
 * buffer whose frames_host points offset_base bytes into it). Not needed by an application;
 * reference: udpdk_poller.c:516-545 (the burst loop these chunks stand for). */
int udpdk_gpu_pipe_rx_host(udpdk_gpu_ctx *ctx, int pipe,
                           const uint8_t *frames_host, uint64_t frames_bytes,
                           const uint32_t *offset_host, uint32_t offset_base,
                           const uint16_t *length_host,
                           const uint32_t *ptype_host, uint32_t n,
                           uint32_t *meta_host, uint32_t *lane_off_host,
                           uint32_t *lane_pkt_host, uint32_t lane_cap,
                           udpdk_rx_stats_t *stats);
int udpdk_gpu_pipe_wait(udpdk_gpu_ctx *ctx, int pipe);
int udpdk_gpu_pipe_batch(udpdk_gpu_ctx *ctx, int pipe, udpdk_rx_batch_t *batch, const uint32_t **meta_dev);
int udpdk_gpu_pipe_h2d(udpdk_gpu_ctx *ctx, int pipe, void *dev, const void *host, size_t bytes);
int udpdk_gpu_pipe_d2h(udpdk_gpu_ctx *ctx, int pipe, void *host, const void *dev, size_t bytes);

/* ---------------------------------------------------------------------------------------------
 * RX payload delivery: the batch form of udpdk_recvfrom (udpdk_syscall.c:401-488) over the lane
 * entries [first, first + count) of an RX output (e.g. one socket's lane, lane_off[s] ..
 * lane_off[s + 1], or all of them). Entry k = frame lane_pkt[first + k]: its UDP payload, frame
 * bytes [42, 42 + min(data_len - 42, dgram_len - 8)) (Ethernet padding trimmed, :459-466),
 * truncated to slot_bytes (recvfrom's len), goes to payload_dev + k * slot_bytes; len_dev[k] =
 * bytes copied (recvfrom's return value); src_ip_dev[k] / src_port_dev[k] = ip_hdr->src_addr /
 * udp_hdr->src_port as raw network-order values (sin_addr / sin_port, :446-447). Slot bytes past
 * len_dev[k] are scratch. Async on the context stream; the batch must be the one lane_pkt_dev
 * was computed from.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    uint8_t  *payload_dev;    /* [count * slot_bytes], 16-byte aligned                         */
    uint32_t  slot_bytes;     /* per-datagram buffer (recvfrom len), multiple of 16, >= 16      */
    uint32_t *len_dev;        /* [count]                                                       */
    uint32_t *src_ip_dev;     /* [count]                                                       */
    uint16_t *src_port_dev;   /* [count]                                                       */
} udpdk_rx_gather_t;

int udpdk_gpu_rx_gather(udpdk_gpu_ctx *ctx, const udpdk_rx_batch_t *batch,
                        const uint32_t *lane_pkt_dev, uint32_t first, uint32_t count,
                        const udpdk_rx_gather_t *out);
/* The same with packed slots: entry k's buffer is payload_dev + slot_off_dev[k], of
 * slot_off_dev[k + 1] - slot_off_dev[k] bytes (multiples of 16, ascending, count + 1 offsets);
 * out->slot_bytes is not used. A poller sizing each slot to its frame (data_len - 42, rounded up
 * to 16) hands the application every payload with one copy of only the bytes that exist. */
int udpdk_gpu_rx_gather_packed(udpdk_gpu_ctx *ctx, const udpdk_rx_batch_t *batch,
                               const uint32_t *lane_pkt_dev, uint32_t first, uint32_t count,
                               const uint32_t *slot_off_dev, const udpdk_rx_gather_t *out);
/* The packed gather on pipe `pipe`'s stream (poller internals, above). */
int udpdk_gpu_pipe_gather_packed(udpdk_gpu_ctx *ctx, int pipe, const udpdk_rx_batch_t *batch,
                                 const uint32_t *lane_pkt_dev, uint32_t first, uint32_t count,
                                 const uint32_t *slot_off_dev, const udpdk_rx_gather_t *out);

/* ---------------------------------------------------------------------------------------------
 * RX reassembly of IPv4 fragments (udpdk_poller.c:338-361: FRAG frames go through
 * rte_ipv4_frag_reassemble_packet on the table of udpdk_poller.c:130, and a completed datagram
 * continues through the demux at the position of the fragment that completed it)
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    uint32_t bucket_num;      /* NUM_FLOWS_DEF = 0x1000 (udpdk_constants.h:32)                  */
    uint32_t bucket_entries;  /* IP_FRAG_TBL_BUCKET_ENTRIES = 16 (power of two, <= 32)          */
    uint64_t max_cycles;      /* flow lifetime in the unit of the tms argument (frag_cycles =
                                 MAX_FLOW_TTL = 1 s of TSC cycles in the reference)              */
    uint32_t max_dgram;       /* IPv4 payload bytes one flow can hold, <= 65515; device memory is
                                 about entries x (max_dgram + 34) bytes                           */
    uint32_t max_entries;     /* NUM_FLOWS_MAX = 65535 (udpdk_constants.h:34): ip_frag_find adds a
                                 flow to a free entry only while fewer than max_entries are in
                                 use; at the limit it deletes the least recently added (or reused)
                                 entry if that one has expired, else drops the fragment (no
                                 space). 0: the table's entry count (the limit never applies).  */
    uint32_t flags;           /* UDPDK_FRAG_CKSUM_DPDK                                          */
    uint32_t reserved;        /* 0                                                              */
} udpdk_frag_table_cfg_t;

/* A reassembled datagram's IPv4 header checksum is left 0, as DPDK 20.05's ipv4_frag_reassemble
 * writes it and the reference delivers it ("TODO must fix the IP header checksum",
 * udpdk_poller.c:355-360), instead of the RFC 1071 value. */
#define UDPDK_FRAG_CKSUM_DPDK 1u

enum udpdk_rs_stat {
    UDPDK_RS_FRAGS      = 0, /* FRAG-verdict frames of the batch                                */
    UDPDK_RS_DROP_LEN   = 1, /* total_length <= 20 (rte_ipv4_frag_reassemble_packet drops it)    */
    UDPDK_RS_DROP_SHORT = 2, /* IP data past the frame or past max_dgram (divergence) */
    UDPDK_RS_NO_SPACE   = 3, /* no free or expired entry in the key's two buckets                */
    UDPDK_RS_ERRORS     = 4, /* flows dropped: duplicate first/last, > 4 fragments, bad size     */
    UDPDK_RS_HOLES      = 5, /* flows dropped: size complete but the fragments do not chain      */
    UDPDK_RS_EXPIRED    = 6, /* flows freed on timeout                                           */
    UDPDK_RS_DONE       = 7, /* datagrams reassembled                                             */
    UDPDK_RS_STORED     = 8, /* fragments of this batch held by the table for later batches      */
    UDPDK_RS_SERIAL     = 9, /* diagnostic: fragments that went through the table one at a time
                                in arrival order (flows that share buckets with an overlapping
                                flow, stay pending, or meet an existing or expired entry)       */
    UDPDK_RS_SORTED     = 10, /* diagnostic: 1 if the batch's flow keys needed the sorts (a key
                                 with fragments in several runs of the batch), 0 if every key's
                                 fragments were already one run in arrival order                */
    UDPDK_RS_N          = 11
};

typedef struct {
    udpdk_rx_batch_t batch;   /* reassembled frames (context-owned, valid until the next call):
                                 first fragment's Ethernet/IPv4 header with total length, DF-only
                                 fragment field and a valid checksum, then the IPv4 payload;
                                 ptype 0x211. Feed it to udpdk_gpu_rx for the demux.           */
    const uint32_t *origin_dev; /* [batch.n] index (in the input batch) of the fragment that
                                 completed each datagram; the datagrams are in this order       */
    uint64_t stats[UDPDK_RS_N];
} udpdk_reasm_out_t;

/* rte_ip_frag_table_create (udpdk_poller.c:130) on the device; replaces an existing table. */
int udpdk_gpu_frag_table_create(udpdk_gpu_ctx *ctx, const udpdk_frag_table_cfg_t *cfg);
/* Reassembly step for one batch whose udpdk_gpu_rx verdicts are in meta_dev (FRAG frames are
 * consumed; state persists across calls). tms is the batch's timestamp (the poller's cur_tsc).
 * Synchronous. Every output, count and table entry equals one-fragment-at-a-time processing in
 * arrival order (rte_ipv4_frag_reassemble_packet per fragment, udpdk_poller.c:338-361): flows
 * that cannot meet another flow in the table run in parallel, the rest in arrival order. */
int udpdk_gpu_rx_reassemble(udpdk_gpu_ctx *ctx, const udpdk_rx_batch_t *batch,
                            const uint32_t *meta_dev, uint64_t tms, udpdk_reasm_out_t *out);
/* As udpdk_gpu_rx_reassemble, consuming the FRAG frames' bytes the way DPDK chains the fragment
 * mbufs instead of copying them: when every datagram the call completes has its fragments back
 * to back in batch->frames_dev, in data order, each exactly 34 header bytes + its data (a
 * fragmenting sender's frames received in order), the first fragment's frame is extended over its
 * followers (each later fragment's data moves back over the headers before it, the header is
 * patched) and out->batch.frames_dev is batch->frames_dev, with the datagrams at their first
 * fragment's offset. Otherwise the call copies, exactly as udpdk_gpu_rx_reassemble. The frame
 * buffer must be writable and its frames must not overlap; other frames are not touched. */
int udpdk_gpu_rx_reassemble_inplace(udpdk_gpu_ctx *ctx, udpdk_rx_batch_t *batch,
                                    const uint32_t *meta_dev, uint64_t tms, udpdk_reasm_out_t *out);

/* ---------------------------------------------------------------------------------------------
 * Receive-side scaling: the reference configures ETH_MQ_RX_RSS with a single
 * RX ring ("TODO add RSS support", udpdk_init.c:112-137) and polls queue 0 (udpdk_poller.c:516).
 * udpdk_gpu_rss computes, per frame, the Toeplitz hash a NIC computes for rss_hf = IPv4 |
 * non-fragmented IPv4 UDP and the redirection-table queue, and lists each queue's frames in
 * arrival order: the split of one ingress batch over several pollers or GPUs by flow.
 * ------------------------------------------------------------------------------------------- */
#define UDPDK_RSS_KEY_BYTES   40u
#define UDPDK_RSS_RETA_MAX    512u
#define UDPDK_RSS_MAX_QUEUES  64u
enum udpdk_rss_type {
    UDPDK_RSS_IPV4            = 1u, /* 2-tuple (src, dst address) for IPv4 frames              */
    UDPDK_RSS_NONFRAG_IPV4_UDP = 2u /* 4-tuple (+ src, dst port) for unfragmented UDP          */
};
typedef struct {
    uint8_t  key[UDPDK_RSS_KEY_BYTES];  /* rss_key, byte 0 first                                */
    uint32_t hash_types;                /* udpdk_rss_type bits                                   */
    uint32_t n_queues;                  /* RX queues, 1..UDPDK_RSS_MAX_QUEUES                    */
    uint32_t reta_size;                 /* power of two, 1..UDPDK_RSS_RETA_MAX                   */
    uint16_t reta[UDPDK_RSS_RETA_MAX];  /* queue of entry hash & (reta_size - 1)                 */
} udpdk_rss_conf_t;

typedef struct {
    uint32_t *hash_dev;       /* [n] the frame's RSS hash (mbuf hash.rss); 0 when no type applies */
    uint32_t *queue_off_dev;  /* [n_queues + 1] exclusive prefix of per-queue frame counts        */
    uint32_t *queue_pkt_dev;  /* [n] frame indices grouped by queue, arrival order kept           */
} udpdk_rss_out_t;

/* The widely used 40-byte Toeplitz key (the RSS verification suite's), both hash types, and a
 * 128-entry redirection table spreading entries round-robin over n_queues. Host only. */
int udpdk_gpu_rss_default_conf(udpdk_rss_conf_t *conf, uint32_t n_queues);
/* rte_eth_dev_rss_hash_update + rte_eth_dev_rss_reta_update: the context's RSS configuration. */
int udpdk_gpu_rss_config(udpdk_gpu_ctx *ctx, const udpdk_rss_conf_t *conf);
/* Hash, queue and per-queue lists for one batch (async on the context stream). Frames the IPv4
 * gate rejects (the rx_classify ptype rule) or with descriptors past frames_bytes get hash 0. */
int udpdk_gpu_rss(udpdk_gpu_ctx *ctx, const udpdk_rx_batch_t *batch, const udpdk_rss_out_t *out);

/* ---------------------------------------------------------------------------------------------
 * TX: Eth/IPv4/UDP header build + rte_ipv4_cksum + payload copy (udpdk_syscall.c:314-356)
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    uint8_t  src_mac[6];     /* config.src_mac_addr ([port0] mac_addr, udpdk_args.c:21-49)     */
    uint8_t  dst_mac[6];     /* config.dst_mac_addr ([port0_dst] mac_addr)                     */
    uint32_t src_ip;         /* config.src_ip_addr, raw                                        */
} udpdk_tx_config_t;

typedef struct {
    const uint8_t  *payload_dev;     /* payload bytes, followed by UDPDK_GPU_FRAMES_TAILROOM
                                        readable bytes (a payload ending at payload_bytes is
                                        read with dword loads up to 3 bytes past it)           */
    uint64_t        payload_bytes;
    const uint32_t *payload_off_dev; /* [n]                                                    */
    const uint16_t *payload_len_dev; /* [n] sendto len, <= 65507                               */
    const int32_t  *sockfd_dev;      /* [n] sending socket (slot table from the snapshot)      */
    const uint32_t *dst_ip_dev;      /* [n] raw dest_addr->sin_addr                            */
    const uint16_t *dst_port_dev;    /* [n] raw dest_addr->sin_port                            */
    uint32_t        n;
} udpdk_tx_batch_t;

typedef struct {
    uint8_t        *frames_dev;      /* output frames                                          */
    uint64_t        frames_bytes;    /* capacity                                               */
    const uint32_t *frame_off_dev;   /* [n] where datagram i's frame(s) start (len_i + 42
                                        bytes, or udpdk_gpu_tx_span() with fragmentation)    */
} udpdk_tx_out_t;

int udpdk_gpu_tx_build(udpdk_gpu_ctx *ctx, const udpdk_tx_config_t *cfg,
                       const udpdk_tx_batch_t *batch, const udpdk_tx_out_t *out);

/* TX with the poller's IPv4 fragmentation (udpdk_poller.c:461-501: a frame of pkt_len =
 * len + 42 > IPV4_MTU_DEFAULT goes through rte_ipv4_fragment_packet(pkt, ..., mtu) and gets its
 * Ethernet header back per fragment). mtu = 1500 reproduces the reference (IPV4_MTU_DEFAULT =
 * RTE_ETHER_MTU, udpdk_constants.h:37); mtu = 0 is udpdk_gpu_tx_build. (mtu - 20) must be a
 * multiple of 8 and mtu >= 68. Every fragment carries mtu - 20 bytes of the IPv4 payload (the
 * UDP header + data), the last the remainder; fragment k of datagram i starts at
 * frame_off[i] + k * (mtu + 14), so datagram i occupies udpdk_gpu_tx_span(len_i, mtu) bytes.
 * Fragment headers: total length 20 + fragment payload, fragment offset (8-byte units) + MF on
 * all but the last, id 0 (as sent), and the IPv4 checksum a NIC fills for PKT_TX_IP_CKSUM
 * (~RFC 1071 sum; DPDK leaves 0 in the mbuf). Unfragmented frames are exactly tx_build's. */
int udpdk_gpu_tx_build_mtu(udpdk_gpu_ctx *ctx, const udpdk_tx_config_t *cfg,
                           const udpdk_tx_batch_t *batch, const udpdk_tx_out_t *out,
                           uint32_t mtu);
/* Output bytes of one datagram of `len` payload bytes and its frame count (host helper). */
uint64_t udpdk_gpu_tx_span(uint32_t len, uint32_t mtu, uint32_t *n_frames);

/* ---------------------------------------------------------------------------------------------
 * Timing (for bench.py / the roofline): on every `enable`-th udpdk_gpu_rx call (0 = off, 1 =
 * every call) each kernel is launched with start/stop events carried by its own dispatch
 * (hipExtLaunchKernelGGL), so no marker packet separates back-to-back kernels; sampling keeps the
 * host cost of the events (~10 us per timed call) off most calls. Read back the accumulated
 * device milliseconds and the number of timed launches per kernel id.
 * ------------------------------------------------------------------------------------------- */
enum udpdk_gpu_kernel_id {
    UDPDK_K_RX_CLASSIFY = 0,   /* parse + checksums + demux + tile histograms (dominant)      */
    UDPDK_K_RX_SCAN     = 1,   /* lane offsets (one or three launches)                         */
    UDPDK_K_RX_SCATTER  = 2,   /* stable per-lane compaction (rx_scatter, or rx_compact1)      */
    UDPDK_K_TX_BUILD    = 3,
    UDPDK_K_RX_GATHER   = 4,   /* payload delivery (udpdk_gpu_rx_gather)                       */
    UDPDK_N_KERNEL_IDS  = 5
};
int udpdk_gpu_timing_enable(udpdk_gpu_ctx *ctx, int enable);
/* Synchronises; ms[k] = accumulated device ms, launches[k] = number of timed calls. Resets. */
int udpdk_gpu_timing_read(udpdk_gpu_ctx *ctx, double ms[UDPDK_N_KERNEL_IDS],
                          uint32_t launches[UDPDK_N_KERNEL_IDS]);

/* Tile geometry the RX pipeline will use for (n, n_lanes): frames per tile and tile count. */
int udpdk_gpu_rx_geometry(uint32_t n, uint32_t n_lanes, uint32_t *tile_frames,
                          uint32_t *n_tiles);

#ifdef __cplusplus
}
#endif

#endif /* UDPDK_GPU_H */
