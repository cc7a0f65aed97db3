/*
 * host_state.h — process-wide state of the host layer behind udpdk_api.h (internal).
 *
 * The reference keeps this state in DPDK memzones shared by the app and the forked poller
 * (exch_zone_desc, exch_slots, sock_bind_table: udpdk_globals.c:9-37, udpdk_init.c:226-279).
 * Here the application and the poller are threads of one process: plain static memory, one lock
 * for the bind table / socket slots (taken by socket, bind, close and by the poller while it
 * reads the table and fills rings), one for the TX queues, and lock-free single-producer /
 * single-consumer RX rings between the poller and recvfrom (rte_ring SP/SC, init.c:270-272).
 */
#ifndef UDPDK_HOST_STATE_H
#define UDPDK_HOST_STATE_H

#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <sys/types.h>

#include "udpdk_api.h"

/* Linux values the reference relies on (udpdk_syscall.c:102-105, :167, :174). */
#define H_SO_REUSEADDR 2
#define H_SO_REUSEPORT 15

#define H_BURST_SIZE     128     /* BURST_SIZE, udpdk_constants.h:41 */
#define H_MAX_WORKERS    31      /* poll worker threads beyond the caller's ([gpu] poll_threads) */
#define H_POLL_THREADS_DEFAULT 8
#define H_UDP_MAX_PAYLOAD 65507  /* 65535 - 20 - 8: the largest datagram fragmentation can carry */

/* A pinned host slab of gathered payloads: one per rx_gather of a poll. Ring entries point into
 * it; the last recvfrom of its datagrams returns it to the pool (the mbuf pool's role). */
struct h_arena {
    uint8_t  *payload;           /* cap_bytes: the datagrams' packed slots (16-byte aligned)     */
    uint32_t *len;               /* [cap_n] payload bytes                                        */
    uint32_t *src_ip;            /* [cap_n] raw                                                  */
    uint16_t *src_port;          /* [cap_n] raw                                                  */
    uint64_t  cap_bytes;
    uint32_t  cap_n;
    atomic_uint refs;            /* queued datagrams still pointing into this slab               */
    struct h_arena *next;        /* free list                                                    */
};

struct h_dgram {                 /* one queued datagram (the mbuf a ring entry would point to)   */
    const uint8_t *data;
    uint32_t len;                /* payload bytes after Ethernet-padding trim                    */
    uint32_t src_ip;             /* raw */
    uint32_t src_port;           /* raw */
    struct h_arena *arena;
};

struct h_ring {                  /* SP/SC ring of EXCH_RING_SIZE entries (udpdk_init.c:268-277)  */
    struct h_dgram *e;
    _Atomic uint32_t head;       /* consumer (recvfrom) */
    _Atomic uint32_t tail;       /* producer (the poller); tail - head = entries */
    /* consumer only: entries of one slab consumed and not yet released to it (one atomic release
     * per run of a slab's entries instead of one per recvfrom) */
    struct h_arena *rel_arena;
    uint32_t rel_n;
    /* close vs a recvfrom blocked on another thread: recvfrom counts itself in busy for its whole
     * call and leaves with EBADF once closing is set; close sets closing and waits for busy to
     * reach 0 before it clears the ring (both seq_cst, so one of the two sees the other). busy
     * is a count, so close also waits for every one of several callers; the ring itself stays
     * single-consumer like the reference's SP/SC rx_q (udpdk_init.c:270-272): one reading thread
     * per socket at a time. */
    atomic_int busy;
    atomic_int closing;
};

struct h_txd {                   /* one sendto waiting for the poller's TX half                  */
    uint64_t pay;                /* offset of its payload in g_udpdk.txp                         */
    uint32_t len;
    uint32_t dst_ip;             /* raw */
    uint32_t dst_port;           /* raw */
};

struct h_txq {                   /* per-socket TX ring (exch_slots[s].tx_q, EXCH_RING_SIZE)      */
    struct h_txd *e;
    uint32_t head, tail;         /* under tx_lock */
};

struct h_slot {                  /* exch_slot_info (udpdk_types.h:40-47) + bind list links        */
    int      used;
    int      bound;
    uint32_t udp_port;           /* raw */
    uint32_t ip;                 /* raw */
    int      so_options;
    /* binding (at most one per socket): node of its port's list */
    int32_t  prev, next;
    uint8_t  reuse_addr, reuse_port;
    struct h_ring rx;
    struct h_txq  tx;
};

/* Device buffers of one context's payload gather (the gather list + the kernel's outputs). */
struct h_gbuf {
    void     *acc, *pay, *len, *sip, *spt;
    uint64_t  acc_cap, pay_cap, len_cap, sip_cap, spt_cap;
};

#define H_MAX_DEVS 16            /* [gpu] devices: RX shard contexts */

/* One RX shard of a multi-device poll ([gpu] devices = 0-7): a contiguous range of the poll's
 * frames processed by its own GPU context (one pool thread drives each). */
struct h_shard {
    udpdk_gpu_ctx *g;
    int       device;
    uint32_t  i0, n;             /* frames [i0, i0 + n) of the poll (contiguous dispatch)        */
    /* RSS dispatch ([gpu] dispatch = rss): the poll indices of the shard's frames (arrival
     * order) and their bytes packed back to back, with their lengths and ptypes */
    uint32_t *idx;  uint64_t idx_cap;
    uint8_t  *pack; uint64_t pack_cap;
    uint16_t *plen; uint64_t plen_cap;
    uint32_t *ppt;  uint64_t ppt_cap;
    uint64_t  lo, bytes;         /* the frame bytes they span (lo 16-byte aligned)              */
    uint32_t *off;  uint64_t off_cap;                 /* offsets rebased to lo                  */
    uint32_t *meta, *loff, *lpkt;
    uint64_t  meta_cap, loff_cap, lpkt_cap;
    udpdk_rx_stats_t st;
    int       err;               /* errno of a failed step, 0 = fine                             */
    /* payload gather of the accepted entries that are this shard's frames */
    uint32_t  nacc;
    uint64_t  acc_bytes;
    uint32_t *acc, *acco;  uint64_t acc_cap, acco_cap;  /* local frame index, packed slot offset */
    struct h_gbuf gb;
    struct h_arena *arena;
};

struct h_state {
    struct h_slot slots[UDPDK_MAX_SOCKETS];
    int32_t  port_head[65536], port_tail[65536];
    uint16_t port_len[65536];
    uint64_t n_active;
    uint64_t version;
    atomic_int interrupted;
    pthread_mutex_t lock;        /* bind table + socket slots + the poller's use of them        */
    pthread_mutex_t tx_lock;     /* TX rings + payload store                                    */
    pthread_mutex_t arena_lock;  /* arena free list                                             */
    uint8_t  src_mac[6], dst_mac[6];
    uint32_t src_ip;
    uint32_t mtu;                /* IPV4_MTU_DEFAULT = RTE_ETHER_MTU (udpdk_constants.h:37)      */
    udpdk_gpu_ctx *gpu;
    int      gpu_device;
    uint32_t gpu_max_frames, gpu_max_lanes;
    /* bind snapshot as uploaded to the GPU: rebuilt only when the table's version moves */
    uint64_t snap_version;       /* version uploaded (UINT64_MAX = none)                        */
    int      snap_compat;
    uint32_t snap_lanes, snap_maxfan;
    /* fragments (udpdk_poller.c:338-361): the device reassembly table, created on the first
     * FRAG frame; geometry from the [gpu] frag_* ini keys (defaults: the poller's table) */
    int      frag_ready;
    uint32_t frag_buckets, frag_entries, frag_max_dgram;
    uint32_t frag_max_entries, frag_flags;    /* 0: NUM_FLOWS_MAX; [gpu] reasm_cksum = dpdk */
    uint64_t frag_ttl_ms;
    uint32_t poll_threads;       /* [gpu] poll_threads: threads of udpdk_poll_rx's socket loops  */
    uint32_t host_copy_min;      /* [gpu] host_copy_min: mean payload bytes from which a poll copies
                                  * its payloads on the host instead of gathering them on the GPU
                                  * (0: always the GPU gather)                                     */
    /* RX work buffers (poller thread only), grow-only */
    uint32_t *rx_meta, *rx_loff, *rx_lpkt;
    uint64_t  rx_meta_cap, rx_loff_cap, rx_lpkt_cap;
    uint32_t *fr_loff, *fr_lpkt, *fr_org;        /* reassembled datagrams: lanes, origins     */
    uint16_t *fr_len;
    uint64_t  fr_loff_cap, fr_lpkt_cap, fr_org_cap, fr_len_cap;
    uint32_t *acc_d, *acc_f;                     /* accepted entries: frame / datagram index   */
    uint32_t *acc_do, *acc_fo;                   /* their packed slot offsets (+ the total)    */
    uint32_t *acc_sock;                          /* per accepted entry: socket | from-frag<<31 */
    uint64_t  acc_d_cap, acc_f_cap, acc_do_cap, acc_fo_cap, acc_sock_cap;
    struct h_gbuf gb;                            /* device: gather list + outputs (context 0)  */
    /* udpdk_poll_rx's pipelined form (h_poll_chunked): pinned verdict words, per-chunk lanes and
     * the gather lists of the chunk in flight; [gpu] poll_chunk_mb = chunk size (0: one piece) */
    uint32_t *pc_meta, *pc_loff, *pc_lpkt, *pc_acc;
    uint64_t  pc_meta_cap, pc_loff_cap, pc_lpkt_cap, pc_acc_cap;
    uint32_t  poll_chunk_mb;
    uint32_t  poll_chunk_min_avg;                /* ... for batches of at least this mean frame size */
    /* multi-device RX ([gpu] devices): n_shards > 1 splits every poll into contiguous shards over
     * the shard contexts; the context above (g_udpdk.gpu) keeps TX and the reassembly table */
    uint32_t  n_shards;
    int       shard_dev[H_MAX_DEVS];
    /* [gpu] dispatch = rss: frames go to shard reta[Toeplitz hash] (the NIC's RSS queue, one
     * queue per device, udpdk_gpu_rss's hash and default key/RETA) instead of contiguous ranges;
     * lanes are merged back in arrival order */
    int       dispatch_rss;
    uint32_t  rss_tab[12][256];
    uint16_t  rss_reta[UDPDK_RSS_RETA_MAX];
    uint32_t  rss_reta_size, rss_types, rss_ready;
    uint8_t  *rss_sh;  uint64_t rss_sh_cap;      /* per poll frame: its shard                   */
    uint32_t *rss_loc; uint64_t rss_loc_cap;     /* ... and its index in that shard             */
    struct h_shard shard[H_MAX_DEVS];
    uint8_t  *acc_dk;                            /* per accepted direct entry: its shard        */
    uint32_t *acc_di;                            /* ... and its index in that shard's slab      */
    uint64_t  acc_dk_cap, acc_di_cap;
    uint8_t  *fb_frames;                         /* FRAG frames of a sharded poll, host copy    */
    uint32_t *fb_off, *fb_idx, *fb_meta, *fb_loff, *fb_lpkt, *fb_pt;
    uint16_t *fb_len;
    uint64_t  fb_frames_cap, fb_off_cap, fb_idx_cap, fb_meta_cap, fb_loff_cap, fb_lpkt_cap, fb_pt_cap,
              fb_len_cap;
    void     *dv_meta2, *dv_loff2, *dv_lpkt2;              /* device: RX of reassembled batch */
    uint64_t  dv_meta2_cap, dv_loff2_cap, dv_lpkt2_cap;
    struct h_arena *arena_free;
    /* pinned slab budget (the mbuf pool's fixed size, udpdk_init.c:78-79): bytes and slabs held
     * by live + free slabs, capped by [gpu] slab_bytes_max / slab_count_max; a poll whose payloads
     * find no slab within the budget drops its bursts (rx_nobufs), as rte_eth_rx_burst does when
     * the mempool is exhausted */
    uint64_t  arena_bytes, arena_bytes_max, rx_nobufs;
    uint32_t  arena_count, arena_count_max, arena_free_n;
    /* TX: per-socket rings of struct h_txd + the payload store they point into */
    uint8_t  *txp;
    uint64_t  txp_bytes, txp_cap;
    uint64_t  tx_queued;                         /* datagrams in all TX rings                   */
    uint64_t  tx_dropped;                        /* too large for the drain's limits (tx_drain)  */
    /* TX work buffers (tx_drain), grow-only: host pinned staging + device */
    void     *tx_h, *tx_d, *tx_fr_d;
    uint64_t  tx_h_cap, tx_d_cap, tx_fr_d_cap;
    struct h_txsel { int32_t s; uint32_t nf; uint64_t foff; } *tx_sel;
    uint64_t  tx_sel_cap;
    /* poller thread (udpdk_port_attach) */
    pthread_t poller;
    atomic_int poller_run;
    int       poller_started;
    udpdk_port_ops_t port;
    /* [gpu] port / port_peer: the port udpdk_init attaches the poller thread to (port_udp.c) */
    char      port_spec[128], port_peer[128];
};

extern struct h_state g_udpdk;

/* port_table.c */
void h_btable_reset(void);
int  h_btable_add(int sockfd, uint32_t ip, uint32_t port, int opts);
void h_btable_del(int sockfd, uint32_t port);
int  h_btable_free_port(void);

/* tx_drain.c: grow-only pinned host buffer (g_udpdk.gpu's allocator) */
int  h_grow_pinned(void **p, uint64_t *cap, uint64_t need);

/* sock_api.c */
void h_sockets_reset(void);
uint32_t h_ring_free(const struct h_ring *r);
int  h_ring_push_bulk(struct h_ring *r, const struct h_dgram *d, uint32_t n);
struct h_arena *h_arena_get(uint32_t n, uint64_t bytes);
void h_arena_put(struct h_arena *a);
void h_arena_release(struct h_arena *a, uint32_t refs);
void h_arenas_free_all(void);
void h_tx_reset(void);

/* h_pool.c: fork-join workers; h_pool_run calls fn(ctx, part, parts) for every part < parts
 * (part 0 on the caller) and returns when all have returned */
typedef void (*h_job_fn)(void *ctx, uint32_t part, uint32_t parts);
uint32_t h_pool_parts(void);
void h_pool_run(h_job_fn fn, void *ctx);
void h_pool_stop(void);

/* rx_poll.c */
int  h_snapshot_refresh(void);            /* under g_udpdk.lock */
void h_rx_buffers_free(void);
void h_shards_destroy(void);
void udpdk_poll_profile_dump(void);   /* -DUDPDK_POLL_PROFILE builds: phase times to stderr */
int  h_grow_dev(void **p, uint64_t *cap, uint64_t need);
int  h_grow_dev_on(udpdk_gpu_ctx *g, void **p, uint64_t *cap, uint64_t need);
int  h_rss_setup(void);
int  h_grow_host(void **p, uint64_t *cap, uint64_t need);

/* port_udp.c: the UDP test wire */
int  h_wire_open(const char *local, const char *peer, udpdk_port_ops_t *ops);
void h_wire_close(void);

/* tx_drain.c */
void h_tx_buffers_free(void);

#endif
