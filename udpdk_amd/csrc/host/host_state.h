/*
 * host_state.h — process-wide state of the host layer behind udpdk_api.h (internal).
 *
 * The reference keeps this state in DPDK memzones shared by the app and the forked poller
 * (exch_zone_desc, exch_slots, sock_bind_table: udpdk_globals.c:9-37, udpdk_init.c:226-279).
 * Here app and poller are the same process, so it is plain static memory.
 */
#ifndef UDPDK_HOST_STATE_H
#define UDPDK_HOST_STATE_H

#include <stdint.h>
#include <sys/types.h>

#include "udpdk_api.h"

/* Linux values the reference relies on (udpdk_syscall.c:102-105, :167, :174). */
#define H_SO_REUSEADDR 2
#define H_SO_REUSEPORT 15

struct h_dgram {             /* one queued datagram (the mbuf a ring entry would point to)   */
    uint8_t *data;
    uint32_t len;            /* payload bytes after Ethernet-padding trim                     */
    uint32_t src_ip;         /* raw */
    uint32_t src_port;       /* raw */
};

struct h_ring {              /* SP/SC ring of EXCH_RING_SIZE entries (udpdk_init.c:268-277)   */
    struct h_dgram *e;
    uint32_t head, tail;     /* tail - head = entries */
};

struct h_slot {              /* exch_slot_info (udpdk_types.h:40-47) + bind list links        */
    int      used;
    int      bound;
    uint32_t udp_port;       /* raw */
    uint32_t ip;             /* raw */
    int      so_options;
    /* binding (at most one per socket): node of its port's list */
    int32_t  prev, next;
    uint8_t  reuse_addr, reuse_port;
    struct h_ring rx;
};

struct h_state {
    struct h_slot slots[UDPDK_MAX_SOCKETS];
    int32_t  port_head[65536], port_tail[65536];
    uint16_t port_len[65536];
    uint64_t n_active;
    uint64_t version;
    volatile int interrupted;
    uint8_t  src_mac[6], dst_mac[6];
    uint32_t src_ip;
    udpdk_gpu_ctx *gpu;
    int      gpu_device;
    uint32_t gpu_max_frames, gpu_max_lanes;
    uint64_t snap_version;   /* version uploaded to the GPU (UINT64_MAX = none) */
    int      snap_compat;
    /* fragments (udpdk_poller.c:338-361): the device reassembly table, created on the first
     * FRAG frame; geometry from the [gpu] frag_* ini keys (defaults: the poller's table) */
    int      frag_ready;
    uint32_t frag_buckets, frag_entries, frag_max_dgram;
    uint64_t frag_ttl_ms;
    void    *fd_frames, *fd_offset, *fd_length, *fd_meta;      /* device copies, grow-only */
    uint64_t fd_frames_cap;
    uint32_t fd_n_cap;
    void    *fd_meta2, *fd_loff2, *fd_lpkt2;
    uint32_t fd_out_cap;
    /* TX queue of built frames (the tx_q rings + TX half of the poller, poller.c:452-514) */
    uint8_t *txq;
    uint64_t txq_bytes, txq_cap;
    uint32_t *txq_len;
    uint32_t txq_n, txq_ncap;
};

extern struct h_state g_udpdk;

/* port_table.c */
void h_btable_reset(void);
int  h_btable_add(int sockfd, uint32_t ip, uint32_t port, int opts);
void h_btable_del(int sockfd, uint32_t port);
int  h_btable_free_port(void);

/* sock_api.c */
void h_sockets_reset(void);
ssize_t h_build_frame(int sockfd, const void *buf, size_t len, uint32_t dst_ip,
                      uint32_t dst_port, uint8_t *out);
int  h_ring_push_bulk(struct h_ring *r, struct h_dgram *d, uint32_t n);

#endif
