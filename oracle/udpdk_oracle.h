/*
 * udpdk_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU-only restatement of the reference UDPDK hot path (leoll2/UDPDK @ v1) used as the
 * parity checker for the HIP datapath and as bench.py's cpu_baseline ("port"). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product library
 * (udpdk_amd/libudpdk_amd.so) never links or calls it.
 *
 * Pinning: the reference itself is unbuildable here (it needs DPDK 20.05; deps/dpdk is an empty
 * submodule) so this restatement is pinned by the TX golden vectors and RX behaviour probes that
 * SURVEY.md §8.G / §8(a) recorded from the reference's own code, and by published RFC 1071
 * checksum examples (tests/golden/). See DESIGN.md "Oracle and parity".
 */
#ifndef UDPDK_ORACLE_H
#define UDPDK_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_btable oracle_btable;

/* Bind table: sock_bind_table[65536] of lists (udpdk_bind_table.c:17-30). */
oracle_btable *oracle_btable_new(void);
void           oracle_btable_free(oracle_btable *bt);
/* btable_add_binding (udpdk_bind_table.c:92-126): 0 ok, -1 if btable_can_bind refuses. */
int            oracle_btable_add(oracle_btable *bt, int sockfd, uint32_t ip_raw, uint32_t port_raw,
                                 int opts);
/* btable_del_binding (udpdk_bind_table.c:129-149). */
void           oracle_btable_del(oracle_btable *bt, int sockfd, uint32_t port_raw);
/* btable_get_free_port (udpdk_bind_table.c:33-42). */
int            oracle_btable_free_port(const oracle_btable *bt);
/* Number of bindings on a raw port, and the i-th in list order (head -> tail). */
int            oracle_btable_port_len(const oracle_btable *bt, uint32_t port_raw);
int            oracle_btable_port_at(const oracle_btable *bt, uint32_t port_raw, int i,
                                     int *sockfd, uint32_t *ip_raw, int *reuse);

/* RX over a batch, in the reference's structure: 128-frame bursts (poller.c:517, BURST_SIZE),
 * reassemble() per frame (poller.c:316-413), per-slot rx_buffer appends (poller.c:294-298) and a
 * per-burst flush of every slot in index order (poller.c:537-541, :274-292).
 * Lanes are keyed by (sockfd & lane_mask). Writes meta[n] in the udpdk_gpu.h word format,
 * lane_off[n_lanes+1], lane_pkt[<= lane_cap], counters[16].
 * do_csum = 0 skips the (new, non-reference) checksum verification for the baseline timing.
 * Returns the number of deliveries, or -1 if lane_cap was too small / a key >= n_lanes. */
int64_t oracle_rx(const oracle_btable *bt, const uint8_t *frames, uint64_t frames_bytes,
                  const uint32_t *offset, const uint16_t *length, const uint32_t *ptype,
                  uint32_t n, uint32_t lane_mask, uint32_t n_lanes, int do_csum,
                  uint32_t *meta, uint32_t *lane_off, uint32_t *lane_pkt, uint32_t lane_cap,
                  uint64_t counters[16]);

/* CPU baseline: nthreads pinned threads, each runs the poller `reps` times over its own full,
 * NUMA-local copy of the batch with preallocated poller state (one independent shard per thread:
 * nthreads x n frames per rep in all). Returns the wall seconds of the timed passes, or -1. */
double  oracle_rx_parallel(const oracle_btable *bt, const uint8_t *frames, uint64_t frames_bytes,
                           const uint32_t *offset, const uint16_t *length, uint32_t n,
                           uint32_t lane_mask, uint32_t n_lanes, int do_csum, int nthreads,
                           int reps);

/* DPDK 20.05 rte_raw_cksum + rte_ipv4_cksum over a 20-byte header (called udpdk_syscall.c:337). */
uint16_t oracle_rte_ipv4_cksum(const uint8_t hdr[20]);

/* udpdk_sendto header build + payload (udpdk_syscall.c:314-356). Writes len + 42 bytes.
 * slot_bound/slot_ip/slot_port: exch_zone_desc->slots[sockfd] after any auto-bind. */
void oracle_tx_frame(const uint8_t src_mac[6], const uint8_t dst_mac[6], uint32_t cfg_src_ip,
                     int slot_bound, uint32_t slot_ip, uint32_t slot_port,
                     uint32_t dst_ip, uint32_t dst_port, const uint8_t *payload, uint32_t len,
                     uint8_t *out);

/* recvfrom payload delivery (udpdk_syscall.c:401-488) for lane entries [first, first + count):
 * payload k into out_payload + k * len (len = recvfrom's len), out_len[k] = bytes copied,
 * out_src_ip / out_src_port = raw ip src_addr / udp src_port. */
/* The poller's TX fragmentation of one sendto frame (udpdk_poller.c:461-501 +
 * rte_ipv4_fragment_packet): fragments back to back into out; returns the frame count. */
uint32_t oracle_tx_fragment(const uint8_t *frame, uint32_t pkt_len, uint32_t mtu, uint8_t *out);

/* RX reassembly (udpdk_oracle_frag.c): DPDK 20.05 rte_ipv4_frag_reassemble_packet restated. */
typedef struct oracle_ftable oracle_ftable;
enum oracle_rs_stat {
    ORACLE_RS_FRAGS = 0,      /* FRAG-verdict frames seen                                      */
    ORACLE_RS_DROP_LEN,       /* total_length <= 20 (rte_ipv4_frag_reassemble_packet)          */
    ORACLE_RS_DROP_SHORT,     /* IP data past the frame or past the datagram capacity          */
    ORACLE_RS_NO_SPACE,       /* ip_frag_find found no entry                                    */
    ORACLE_RS_ERRORS,         /* flows dropped: duplicate first/last, > 4 fragments, size      */
    ORACLE_RS_HOLES,          /* flows dropped: complete size but the chain walk found a hole  */
    ORACLE_RS_EXPIRED,        /* flows freed on timeout (own reuse or stale slot)              */
    ORACLE_RS_DONE,           /* datagrams reassembled                                          */
    ORACLE_RS_STORED,         /* fragments of this call still held by the table at its end      */
    ORACLE_RS_N
};
/* max_entries: rte_ip_frag_table_create's max_entries (0: the entry count); flags bit 0: the
 * reassembled header checksum left 0 as DPDK writes it (UDPDK_FRAG_CKSUM_DPDK). */
oracle_ftable *oracle_ftable_new(uint32_t bucket_num, uint32_t bucket_entries, uint64_t max_cycles,
                                 uint32_t max_dgram, uint32_t max_entries, uint32_t flags);
void           oracle_ftable_free(oracle_ftable *t);
uint32_t       oracle_frag_hash(uint32_t src, uint32_t dst, uint32_t id, uint32_t *sig2);
/* FRAG-verdict frames of one batch in arrival order; reassembled frames 16-byte aligned into
 * out, with their offset/length and the index of the completing fragment. Returns the count or
 * -1 if out/out_max is too small. stats accumulate. */
int64_t oracle_reassemble(oracle_ftable *t, const uint8_t *frames, uint64_t frames_bytes,
                          const uint32_t *offset, const uint16_t *length, const uint32_t *meta,
                          uint32_t n, uint64_t tms, uint8_t *out, uint64_t out_cap,
                          uint32_t *out_off, uint16_t *out_len, uint32_t *out_origin,
                          uint32_t out_max, uint64_t stats[ORACLE_RS_N]);

/* Receive-side scaling (udpdk_oracle_rss.c): Toeplitz hash and redirection-table queues. */
uint32_t oracle_toeplitz(const uint8_t key[40], const uint8_t *data, uint32_t len);
int oracle_rss(const uint8_t key[40], uint32_t hash_types, const uint16_t *reta, uint32_t reta_size,
               uint32_t n_queues, const uint8_t *frames, uint64_t frames_bytes,
               const uint32_t *offset, const uint16_t *length, const uint32_t *ptype, uint32_t n,
               uint32_t *hash_out, uint32_t *queue_off, uint32_t *queue_pkt);

void oracle_recv_gather(const uint8_t *frames, const uint32_t *offset, const uint16_t *length,
                        const uint32_t *lane_pkt, uint32_t first, uint32_t count, uint32_t len,
                        uint8_t *out_payload, uint32_t *out_len, uint32_t *out_src_ip,
                        uint16_t *out_src_port);

#ifdef __cplusplus
}
#endif

#endif
