/*
 * udpdk_oracle.c — TEST INFRASTRUCTURE ONLY (see udpdk_oracle.h).
 *
 * CPU restatement of the reference hot path. Every function cites the reference file:line it
 * follows (paths relative to leoll2/UDPDK udpdk/). Written from the reference's behaviour, not
 * its text: the list is an index-linked node pool instead of clib list + shmalloc, and the
 * mbuf/ring plumbing is reduced to per-slot buffers and per-lane queues.
 */
#define _GNU_SOURCE
#include "udpdk_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define O_PORTS          65536           /* UDP_MAX_PORT, udpdk_constants.h:13 */
#define O_MAX_BINDS      (1 << 20)
#define O_BURST          128             /* BURST_SIZE, udpdk_constants.h:41 */
#define O_SO_REUSEADDR   2               /* Linux SOL_SOCKET values used by udpdk_syscall.c:167,174 */
#define O_SO_REUSEPORT   15
#define O_INADDR_ANY     0u

/* ---------------------------------------------------------------------------------------------
 * Bind table: per raw port a doubly linked list of bind_info (udpdk_types.h:31-37) nodes.
 * ------------------------------------------------------------------------------------------- */
struct o_node {
    int32_t  sockfd;
    uint32_t ip;
    uint8_t  reuse_addr, reuse_port;
    int32_t  prev, next;       /* node indices, -1 = none */
};

struct oracle_btable {
    int32_t       head[O_PORTS], tail[O_PORTS];
    int32_t       len[O_PORTS];
    struct o_node *nodes;
    int32_t       n_nodes, cap;
    int32_t       free_list;
};

oracle_btable *oracle_btable_new(void)
{
    /* btable_init, udpdk_bind_table.c:21-30: every port starts unbound */
    oracle_btable *bt = calloc(1, sizeof(*bt));
    if (!bt) return NULL;
    for (int i = 0; i < O_PORTS; i++) { bt->head[i] = bt->tail[i] = -1; }
    bt->free_list = -1;
    return bt;
}

void oracle_btable_free(oracle_btable *bt)
{
    if (!bt) return;
    free(bt->nodes);
    free(bt);
}

static int32_t o_node_alloc(oracle_btable *bt)
{
    if (bt->free_list >= 0) {
        int32_t i = bt->free_list;
        bt->free_list = bt->nodes[i].next;
        return i;
    }
    if (bt->n_nodes == bt->cap) {
        int32_t nc = bt->cap ? bt->cap * 2 : 1024;
        if (nc > O_MAX_BINDS) return -1;
        struct o_node *nn = realloc(bt->nodes, (size_t)nc * sizeof(*nn));
        if (!nn) return -1;
        bt->nodes = nn;
        bt->cap = nc;
    }
    return bt->n_nodes++;
}

/* btable_can_bind, udpdk_bind_table.c:47-89 */
static int o_can_bind(const oracle_btable *bt, uint32_t ip_new, uint32_t port, int opts)
{
    if (bt->head[port] < 0) return 1;
    for (int32_t i = bt->head[port]; i >= 0; i = bt->nodes[i].next) {
        uint32_t ip_oth = bt->nodes[i].ip;
        int oth_reuseport = bt->nodes[i].reuse_port;
        if (ip_oth != ip_new && ip_oth != O_INADDR_ANY && ip_new != O_INADDR_ANY)
            continue;                                                     /* :70-72 */
        if (ip_oth != ip_new && (ip_oth == O_INADDR_ANY || ip_new != O_INADDR_ANY) &&
            ((opts & O_SO_REUSEADDR) || (opts & O_SO_REUSEPORT)))
            continue;                                                     /* :74-77 */
        if (ip_oth == ip_new && ip_new != O_INADDR_ANY && (opts & O_SO_REUSEPORT) &&
            oth_reuseport)
            continue;                                                     /* :79-82 */
        return 0;                                                         /* :83-84 */
    }
    return 1;
}

/* btable_add_binding, udpdk_bind_table.c:92-126 */
int oracle_btable_add(oracle_btable *bt, int sockfd, uint32_t ip_raw, uint32_t port_raw, int opts)
{
    uint32_t port = port_raw & 0xFFFFu;
    if (!o_can_bind(bt, ip_raw, port, opts)) return -1;
    int32_t i = o_node_alloc(bt);
    if (i < 0) return -1;
    struct o_node *nd = &bt->nodes[i];
    nd->sockfd = sockfd;
    nd->ip = ip_raw;
    nd->reuse_addr = (opts & O_SO_REUSEADDR) != 0;                        /* :114 */
    nd->reuse_port = (opts & O_SO_REUSEPORT) != 0;                        /* :115 */
    if (ip_raw == O_INADDR_ANY) {                                         /* :120-121 list_lpush */
        nd->prev = -1;
        nd->next = bt->head[port];
        if (bt->head[port] >= 0) bt->nodes[bt->head[port]].prev = i; else bt->tail[port] = i;
        bt->head[port] = i;
    } else {                                                              /* :122-123 list_rpush */
        nd->next = -1;
        nd->prev = bt->tail[port];
        if (bt->tail[port] >= 0) bt->nodes[bt->tail[port]].next = i; else bt->head[port] = i;
        bt->tail[port] = i;
    }
    bt->len[port]++;
    return 0;
}

/* btable_del_binding, udpdk_bind_table.c:129-149 (first node with that sockfd, head first) */
void oracle_btable_del(oracle_btable *bt, int sockfd, uint32_t port_raw)
{
    uint32_t port = port_raw & 0xFFFFu;
    for (int32_t i = bt->head[port]; i >= 0; i = bt->nodes[i].next) {
        if (bt->nodes[i].sockfd != sockfd) continue;
        struct o_node *nd = &bt->nodes[i];                                /* list_remove, list.c:215-229 */
        if (nd->prev >= 0) bt->nodes[nd->prev].next = nd->next; else bt->head[port] = nd->next;
        if (nd->next >= 0) bt->nodes[nd->next].prev = nd->prev; else bt->tail[port] = nd->prev;
        nd->next = bt->free_list;
        bt->free_list = i;
        bt->len[port]--;
        break;
    }
}

/* btable_get_free_port, udpdk_bind_table.c:33-42: lowest raw index with no list */
int oracle_btable_free_port(const oracle_btable *bt)
{
    for (int i = 0; i < O_PORTS; i++)
        if (bt->head[i] < 0) return i;
    return -1;
}

int oracle_btable_port_len(const oracle_btable *bt, uint32_t port_raw)
{
    return bt->len[port_raw & 0xFFFFu];
}

int oracle_btable_port_at(const oracle_btable *bt, uint32_t port_raw, int k, int *sockfd,
                          uint32_t *ip_raw, int *reuse)
{
    int32_t i = bt->head[port_raw & 0xFFFFu];
    while (i >= 0 && k > 0) { i = bt->nodes[i].next; k--; }
    if (i < 0) return -1;
    *sockfd = bt->nodes[i].sockfd;
    *ip_raw = bt->nodes[i].ip;
    *reuse = bt->nodes[i].reuse_addr || bt->nodes[i].reuse_port;
    return 0;
}

/* ---------------------------------------------------------------------------------------------
 * Checksums. RFC 1071 one's-complement sum of 16-bit words taken in host (little-endian) order,
 * the way DPDK's __rte_raw_cksum sums them; an odd trailing byte is zero-padded.
 * ------------------------------------------------------------------------------------------- */
static uint64_t o_sum16(const uint8_t *p, uint32_t nbytes)
{
    uint64_t s = 0;
    uint32_t i = 0;
    for (; i + 1 < nbytes; i += 2) s += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
    if (i < nbytes) s += p[i];
    return s;
}

static uint16_t o_fold(uint64_t s)
{
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)s;
}

/* DPDK 20.05 lib/librte_net/rte_ip.h: rte_raw_cksum reduces the 32-bit word sum twice and
 * rte_ipv4_cksum returns the raw value unchanged when it is 0xffff, else its complement
 * (SURVEY.md §8 a11, quirk Q7). */
uint16_t oracle_rte_ipv4_cksum(const uint8_t hdr[20])
{
    uint32_t sum = 0;
    for (int i = 0; i < 20; i += 2) sum += (uint32_t)hdr[i] | ((uint32_t)hdr[i + 1] << 8);
    sum = ((sum & 0xFFFF0000u) >> 16) + (sum & 0xFFFFu);
    sum = ((sum & 0xFFFF0000u) >> 16) + (sum & 0xFFFFu);
    uint16_t raw = (uint16_t)sum;
    return raw == 0xFFFFu ? raw : (uint16_t)~raw;
}

static inline uint16_t o_rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t o_rd32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

enum { V_DELIVERED, V_NOT_IPV4, V_FRAG, V_NOT_UDP, V_NO_BIND, V_NO_MATCH, V_TRUNC, V_BAD_DESC };

/* ---------------------------------------------------------------------------------------------
 * RX
 * ------------------------------------------------------------------------------------------- */
struct o_lane {            /* one per lane: the per-socket ring the poller flushes into */
    uint32_t *v;
    uint32_t  n, cap;
};

static int o_lane_push(struct o_lane *q, uint32_t x)
{
    if (q->n == q->cap) {
        uint32_t nc = q->cap ? q->cap * 2 : 64;
        uint32_t *nv = realloc(q->v, (size_t)nc * sizeof(uint32_t));
        if (!nv) return -1;
        q->v = nv;
        q->cap = nc;
    }
    q->v[q->n++] = x;
    return 0;
}

struct o_slot_buf {        /* exch_slot.rx_buffer + rx_count (udpdk_types.h:56-61) */
    uint32_t *pkt;
    uint32_t  count, cap;
};

struct o_rx_state {
    struct o_slot_buf *slots;    /* [n_lanes] */
    uint32_t          *touched;  /* slots with count > 0 in this burst */
    uint32_t           n_touched;
    int                err;
};

/* enqueue_rx_packet, poller.c:294-298: the slot index is the (masked) sockfd */
static void o_enqueue(struct o_rx_state *st, uint32_t key, uint32_t pkt)
{
    struct o_slot_buf *b = &st->slots[key];
    if (b->count == b->cap) {
        uint32_t nc = b->cap ? b->cap * 2 : 8;
        uint32_t *np = realloc(b->pkt, (size_t)nc * sizeof(uint32_t));
        if (!np) { st->err = 1; return; }
        b->pkt = np;
        b->cap = nc;
    }
    if (b->count == 0) st->touched[st->n_touched++] = key;
    b->pkt[b->count++] = pkt;
}

/* reassemble(), poller.c:316-413, for frame i. Returns the verdict word. */
static uint32_t o_reassemble(const oracle_btable *bt, const uint8_t *frames,
                             uint64_t frames_bytes, uint32_t off, uint32_t len,
                             const uint32_t *ptype, uint32_t i, uint32_t lane_mask,
                             uint32_t n_lanes, int do_csum, struct o_rx_state *st,
                             uint64_t *cnt)
{
    if ((uint64_t)off + len > frames_bytes) {
        cnt[V_BAD_DESC]++;
        return V_BAD_DESC;
    }
    const uint8_t *f = frames + off;
    cnt[15] += len;

    /* RTE_ETH_IS_IPV4_HDR(m->packet_type), poller.c:334. Without a NIC the ptype is derived
     * from the ether_type the way a PMD would report an untagged frame. */
    uint32_t pt;
    if (ptype) pt = ptype[i];
    else pt = len >= 14 ? ((f[12] == 0x08 && f[13] == 0x00) ? 0x211u : 0x1u) : 0u;
    if (!(pt & 0x10u)) { cnt[V_NOT_IPV4]++; return V_NOT_IPV4; }          /* :362-366 */
    /* a fragment needs only its IPv4 header to go to rte_ipv4_frag_reassemble_packet
     * (poller.c:338-361): an unpadded frame of 34-41 B (a last fragment of 1-7 data bytes) is
     * reassembled; any other frame shorter than the 42-byte Eth/IPv4/UDP header is TRUNC */
    if (len < 34) { cnt[V_TRUNC]++; return V_TRUNC; }
    /* rte_ipv4_frag_pkt_is_fragmented, poller.c:338 (MF flag or fragment offset) */
    const uint16_t fo = (uint16_t)((f[20] << 8) | f[21]);
    const int fragd = (fo & 0x2000u) || (fo & 0x1FFFu);
    if (len < 42 && !fragd) { cnt[V_TRUNC]++; return V_TRUNC; }

    uint32_t w = 0;
    /* ip = (eth_hdr + 1): fixed 14 B offset, IHL never read (poller.c:336) */
    if ((f[14] & 0x0F) != 5) { w |= 1u << 8; cnt[14]++; }
    if (do_csum) {
        if (o_fold(o_sum16(f + 14, 20)) == 0xFFFFu) w |= 1u << 4;
        else cnt[9]++;
    }
    if (fragd) { cnt[V_FRAG]++; return w | V_FRAG; }
    /* is_udp_pkt, poller.c:300-303, :368-371 */
    if (f[23] != 17) { cnt[V_NOT_UDP]++; return w | V_NOT_UDP; }

    /* UDP checksum (new output; the reference never verifies) */
    uint32_t udp_len = (uint32_t)((f[38] << 8) | f[39]);
    int len_bad = udp_len < 8 || 34 + udp_len > len;
    if (len_bad) { w |= 1u << 7; cnt[13]++; }
    if (do_csum) {
        uint32_t state;
        if (o_rd16(f + 40) == 0) state = 0;
        else if (len_bad) state = 2;
        else {
            uint32_t src = o_rd32(f + 26), dst = o_rd32(f + 30);
            uint64_t s = o_sum16(f + 34, udp_len);
            s += (src & 0xFFFFu) + (src >> 16) + (dst & 0xFFFFu) + (dst >> 16);
            s += 0x1100u;                               /* zero + protocol 17, network order */
            s += o_rd16(f + 38);                        /* UDP length, network order */
            state = o_fold(s) == 0xFFFFu ? 1 : 2;
        }
        w |= state << 5;
        cnt[state == 0 ? 12 : (state == 1 ? 10 : 11)]++;
    }

    /* get_udp_dst_port / get_ipv4_dst_addr: raw BE values at fixed offsets, poller.c:305-313 */
    uint32_t dport = o_rd16(f + 36);
    uint32_t dip = o_rd32(f + 30);
    if (bt->head[dport] < 0) { cnt[V_NO_BIND]++; return w | V_NO_BIND; } /* :376-380 */

    uint32_t fan = 0, first = 0;
    for (int32_t k = bt->head[dport]; k >= 0; k = bt->nodes[k].next) {    /* :381-405 */
        const struct o_node *b = &bt->nodes[k];
        if (dip == b->ip || b->ip == O_INADDR_ANY) {                       /* :391 */
            uint32_t key = (uint32_t)b->sockfd & lane_mask;
            if (key >= n_lanes) { st->err = 1; break; }
            o_enqueue(st, key, i);                                          /* :393 */
            if (fan == 0) first = (uint32_t)b->sockfd;
            fan++;
            if (b->reuse_addr || b->reuse_port) continue;                   /* :396-399 clone */
            break;                                                          /* :400-403 */
        }
    }
    if (fan == 0) { cnt[V_NO_MATCH]++; return w | V_NO_MATCH; }            /* :406-411 */
    cnt[V_DELIVERED]++;
    cnt[8] += fan;
    return w | V_DELIVERED | ((fan > 127 ? 127u : fan) << 9) | ((first & 0xFFFFu) << 16);
}

/* The per-socket state the poller keeps between bursts (exch_slots + rings): allocated once and
 * reused across calls, so a timed loop of oracle_rx_ws calls measures the poller's work, not the
 * allocator (the reference's rings and slot buffers are preallocated too, udpdk_init.c:252-279). */
struct o_rx_ws {
    struct o_lane     *lanes;
    struct o_rx_state  st;
    uint32_t           n_lanes;
};

static void o_ws_free(struct o_rx_ws *w)
{
    if (w->lanes) for (uint32_t k = 0; k < w->n_lanes; k++) free(w->lanes[k].v);
    if (w->st.slots) for (uint32_t k = 0; k < w->n_lanes; k++) free(w->st.slots[k].pkt);
    free(w->lanes);
    free(w->st.slots);
    free(w->st.touched);
    memset(w, 0, sizeof(*w));
}

static int o_ws_init(struct o_rx_ws *w, uint32_t n_lanes)
{
    memset(w, 0, sizeof(*w));
    w->n_lanes = n_lanes ? n_lanes : 1;
    w->lanes = calloc(w->n_lanes, sizeof(*w->lanes));
    w->st.slots = calloc(w->n_lanes, sizeof(*w->st.slots));
    w->st.touched = calloc(w->n_lanes, sizeof(uint32_t));
    if (!w->lanes || !w->st.slots || !w->st.touched) { o_ws_free(w); return -1; }
    return 0;
}

static int64_t o_rx_run(struct o_rx_ws *w, const oracle_btable *bt, const uint8_t *frames,
                        uint64_t frames_bytes, const uint32_t *offset, const uint16_t *length,
                        const uint32_t *ptype, uint32_t n, uint32_t lane_mask, uint32_t n_lanes,
                        int do_csum, uint32_t *meta, uint32_t *lane_off, uint32_t *lane_pkt,
                        uint32_t lane_cap, uint64_t counters[16])
{
    struct o_rx_state *st = &w->st;
    struct o_lane *lanes = w->lanes;
    uint64_t cnt[16] = {0};
    st->err = 0;
    st->n_touched = 0;
    for (uint32_t k = 0; k < n_lanes; k++) lanes[k].n = 0;

    /* poller_body RX half, poller.c:516-545: bursts of BURST_SIZE frames */
    for (uint32_t b0 = 0; b0 < n; b0 += O_BURST) {
        uint32_t b1 = b0 + O_BURST < n ? b0 + O_BURST : n;
        for (uint32_t i = b0; i < b1; i++)                                  /* :526-534 */
            meta[i] = o_reassemble(bt, frames, frames_bytes, offset[i], length[i], ptype, i,
                                   lane_mask, n_lanes, do_csum, st, cnt);
        if (st->err) return -1;
        /* flush every slot holding frames (:537-541 scans all slots in index order; the order
         * across slots cannot change any lane's contents) via flush_rx_queue (:274-292).
         * A full ring would drop the whole batch (:287-290); lanes here are unbounded. */
        for (uint32_t t = 0; t < st->n_touched; t++) {
            struct o_slot_buf *sb = &st->slots[st->touched[t]];
            for (uint32_t j = 0; j < sb->count; j++)
                if (o_lane_push(&lanes[st->touched[t]], sb->pkt[j])) return -1;
            sb->count = 0;                                                  /* :291 */
        }
        st->n_touched = 0;
    }

    uint64_t d = 0;
    for (uint32_t k = 0; k < n_lanes; k++) {
        lane_off[k] = (uint32_t)d;
        if (d + lanes[k].n > lane_cap) return -1;
        memcpy(lane_pkt + d, lanes[k].v, (size_t)lanes[k].n * sizeof(uint32_t));
        d += lanes[k].n;
    }
    lane_off[n_lanes] = (uint32_t)d;
    if (counters) memcpy(counters, cnt, sizeof(cnt));
    return (int64_t)d;
}

int64_t oracle_rx(const oracle_btable *bt, const uint8_t *frames, uint64_t frames_bytes,
                  const uint32_t *offset, const uint16_t *length, const uint32_t *ptype,
                  uint32_t n, uint32_t lane_mask, uint32_t n_lanes, int do_csum,
                  uint32_t *meta, uint32_t *lane_off, uint32_t *lane_pkt, uint32_t lane_cap,
                  uint64_t counters[16])
{
    struct o_rx_ws w;
    if (o_ws_init(&w, n_lanes)) return -1;
    const int64_t r = o_rx_run(&w, bt, frames, frames_bytes, offset, length, ptype, n, lane_mask,
                               n_lanes, do_csum, meta, lane_off, lane_pkt, lane_cap, counters);
    o_ws_free(&w);
    return r;
}

/* ---------------------------------------------------------------------------------------------
 * CPU baseline harness: every pinned thread runs the poller over its own full copy of the batch
 * (one independent shard per thread). The copy, the poller state and the
 * outputs are allocated and first touched by the thread itself after pinning (NUMA-local), and
 * one untimed pass grows the per-socket vectors to size before the timed passes.
 * ------------------------------------------------------------------------------------------- */
struct o_job {
    const oracle_btable *bt;
    const uint8_t *frames;
    uint64_t frames_bytes;
    const uint32_t *offset;
    const uint16_t *length;
    uint32_t n, lane_mask, n_lanes;
    int do_csum, reps, cpu, err;
    pthread_barrier_t *bar;
};

static void *o_job_run(void *arg)
{
    struct o_job *j = arg;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(j->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    const uint32_t cap = j->n * 2u + 64u;     /* fan-out <= 2 in the bench workloads */
    uint8_t *fr = malloc(j->frames_bytes + 64);
    uint32_t *off = malloc((size_t)j->n * 4 + 4), *meta = malloc((size_t)j->n * 4 + 4);
    uint16_t *len = malloc((size_t)j->n * 2 + 2);
    uint32_t *loff = malloc(((size_t)j->n_lanes + 1) * 4), *pkt = malloc((size_t)cap * 4);
    struct o_rx_ws w;
    const int ok = fr && off && meta && len && loff && pkt && o_ws_init(&w, j->n_lanes) == 0;
    if (ok) {
        memcpy(fr, j->frames, j->frames_bytes);
        memset(fr + j->frames_bytes, 0, 64);
        memcpy(off, j->offset, (size_t)j->n * 4);
        memcpy(len, j->length, (size_t)j->n * 2);
        memset(meta, 0, (size_t)j->n * 4);
        memset(pkt, 0, (size_t)cap * 4);
        if (o_rx_run(&w, j->bt, fr, j->frames_bytes, off, len, NULL, j->n, j->lane_mask, j->n_lanes,
                     j->do_csum, meta, loff, pkt, cap, NULL) < 0)
            j->err = 1;
    } else {
        j->err = 1;
    }
    pthread_barrier_wait(j->bar);
    for (int r = 0; ok && r < j->reps; r++)
        o_rx_run(&w, j->bt, fr, j->frames_bytes, off, len, NULL, j->n, j->lane_mask, j->n_lanes,
                 j->do_csum, meta, loff, pkt, cap, NULL);
    pthread_barrier_wait(j->bar);
    if (ok) o_ws_free(&w);
    free(fr); free(off); free(meta); free(len); free(loff); free(pkt);
    return NULL;
}

double oracle_rx_parallel(const oracle_btable *bt, const uint8_t *frames, uint64_t frames_bytes,
                          const uint32_t *offset, const uint16_t *length, uint32_t n,
                          uint32_t lane_mask, uint32_t n_lanes, int do_csum, int nthreads,
                          int reps)
{
    if (nthreads < 1) nthreads = 1;
    struct o_job *jobs = calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
    /* thread t pinned to the t-th CPU this process may run on (its affinity mask: on a
     * partitioned host that is the share the process was given, not every online CPU) */
    int cpus[CPU_SETSIZE], ncpu = 0;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
    for (int t = 0; t < nthreads; t++) {
        struct o_job *j = &jobs[t];
        j->bt = bt; j->frames = frames; j->frames_bytes = frames_bytes;
        j->offset = offset; j->length = length; j->n = n;
        j->lane_mask = lane_mask; j->n_lanes = n_lanes; j->do_csum = do_csum; j->reps = reps;
        j->cpu = ncpu > 0 ? cpus[t % ncpu] : 0;
        j->bar = &bar;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, o_job_run, &jobs[t]);
    struct timespec t0, t1;
    pthread_barrier_wait(&bar);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_barrier_wait(&bar);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
    }
    const double secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    pthread_barrier_destroy(&bar);
    free(jobs);
    free(th);
    return err ? -1.0 : secs;
}

/* ---------------------------------------------------------------------------------------------
 * TX: udpdk_sendto header build, udpdk_syscall.c:314-356
 * ------------------------------------------------------------------------------------------- */
void oracle_tx_frame(const uint8_t src_mac[6], const uint8_t dst_mac[6], uint32_t cfg_src_ip,
                     int slot_bound, uint32_t slot_ip, uint32_t slot_port,
                     uint32_t dst_ip, uint32_t dst_port, const uint8_t *payload, uint32_t len,
                     uint8_t *out)
{
    memcpy(out + 0, dst_mac, 6);                                          /* :317 d_addr */
    memcpy(out + 6, src_mac, 6);                                          /* :316 s_addr */
    out[12] = 0x08; out[13] = 0x00;                                       /* :318 */
    uint8_t *ip = out + 14;
    memset(ip, 0, 20);                                                    /* :322 */
    ip[0] = 0x45;                                                         /* :323 IP_VHL_DEF */
    ip[8] = 64;                                                           /* :326 IP_DEFTTL */
    ip[9] = 17;                                                           /* :327 */
    uint32_t src = (slot_bound && slot_ip != O_INADDR_ANY) ? slot_ip : cfg_src_ip; /* :329-334 */
    memcpy(ip + 12, &src, 4);
    memcpy(ip + 16, &dst_ip, 4);                                          /* :335 */
    uint32_t tl = len + 28;                                               /* :336 */
    ip[2] = (uint8_t)(tl >> 8); ip[3] = (uint8_t)tl;
    uint16_t ck = oracle_rte_ipv4_cksum(ip);                              /* :337 */
    memcpy(ip + 10, &ck, 2);                                              /* host u16 store */
    uint8_t *udp = out + 34;
    udp[0] = (uint8_t)slot_port; udp[1] = (uint8_t)(slot_port >> 8);       /* :341 raw */
    udp[2] = (uint8_t)dst_port; udp[3] = (uint8_t)(dst_port >> 8);         /* :342 raw */
    uint32_t ul = len + 8;                                                /* :344 */
    udp[4] = (uint8_t)(ul >> 8); udp[5] = (uint8_t)ul;
    udp[6] = 0; udp[7] = 0;                                               /* :343 */
    if (len) memcpy(out + 42, payload, len);                              /* :355-356 */
}

/* ---------------------------------------------------------------------------------------------
 * The poller's TX fragmentation, udpdk_poller.c:461-501: a frame of pkt_len > IPV4_MTU_DEFAULT
 * (udpdk_constants.h:37, RTE_ETHER_MTU = 1500) loses its Ethernet header (rte_pktmbuf_adj), is
 * cut by rte_ipv4_fragment_packet(pkt, out, n, IPV4_MTU_DEFAULT, ...) and every fragment gets the
 * saved Ethernet header back (rte_pktmbuf_prepend + copies of ether_type, s_addr, d_addr).
 *
 * rte_ipv4_fragment_packet (DPDK 20.05 lib/librte_ip_frag/rte_ipv4_fragmentation.c, not in the
 * container; restated from its published source): frag_size = mtu - 20 (a multiple of 8); the
 * input's IP payload is cut into runs of frag_size bytes, the last the remainder; each fragment
 * header is the input header (__fill_ipv4hdr_frag) with fragment_offset = input flags/offset +
 * (data offset >> 3), MF set unless it is the last, total_length = 20 + its payload and
 * hdr_checksum = 0 (the poller sets PKT_TX_IP_CKSUM: the NIC computes it). Here the checksum is
 * written as the NIC would: ~(RFC 1071 sum), i.e. 0 when the sum folds to 0xffff.
 *
 * `frame` is one udpdk_sendto frame of len + 42 bytes (oracle_tx_frame); the fragments are
 * written back to back into `out`; returns the number of frames. mtu = 0 or pkt_len <= mtu:
 * the frame is copied unchanged.
 * ------------------------------------------------------------------------------------------- */
uint32_t oracle_tx_fragment(const uint8_t *frame, uint32_t pkt_len, uint32_t mtu, uint8_t *out)
{
    if (!mtu || pkt_len <= mtu) {                                         /* poller.c:466 */
        memcpy(out, frame, pkt_len);
        return 1;
    }
    const uint8_t *ip = frame + 14;                                       /* :471 adj */
    const uint32_t ip_payload = pkt_len - 14 - 20;
    const uint32_t frag_size = mtu - 20;
    const uint16_t in_fo = (uint16_t)((ip[6] << 8) | ip[7]);
    uint32_t n = 0, pos = 0;
    uint8_t *o = out;
    while (pos < ip_payload) {
        const uint32_t len = ip_payload - pos < frag_size ? ip_payload - pos : frag_size;
        const int more = pos + len < ip_payload;
        memcpy(o, frame, 14);                                             /* :484-490 */
        uint8_t *h = o + 14;
        memcpy(h, ip, 20);                                                /* __fill_ipv4hdr_frag */
        uint16_t fo = (uint16_t)(in_fo + (pos >> 3));
        fo = (uint16_t)(fo | (more ? 0x2000u : 0u));
        h[6] = (uint8_t)(fo >> 8); h[7] = (uint8_t)fo;
        const uint32_t tl = 20 + len;
        h[2] = (uint8_t)(tl >> 8); h[3] = (uint8_t)tl;
        h[10] = 0; h[11] = 0;
        uint32_t sum = 0;
        for (int i = 0; i < 20; i += 2) sum += (uint32_t)h[i] | ((uint32_t)h[i + 1] << 8);
        sum = (sum >> 16) + (sum & 0xFFFFu);
        sum = (sum >> 16) + (sum & 0xFFFFu);
        const uint16_t ck = (uint16_t)~sum;                               /* NIC IP checksum */
        memcpy(h + 10, &ck, 2);
        memcpy(o + 34, ip + 20 + pos, len);
        o += 34 + len;
        pos += len;
        n++;
    }
    return n;
}

/* ---------------------------------------------------------------------------------------------
 * recvfrom payload delivery, udpdk_syscall.c:401-488 (single-segment mbufs), for lane entries
 * [first, first + count): entry k's payload into out_payload + k * len (len = recvfrom's len),
 * bytes copied into out_len[k], ip_hdr->src_addr / udp_hdr->src_port raw into out_src_*.
 * ------------------------------------------------------------------------------------------- */
void oracle_recv_gather(const uint8_t *frames, const uint32_t *offset, const uint16_t *length,
                        const uint32_t *lane_pkt, uint32_t first, uint32_t count, uint32_t len,
                        uint8_t *out_payload, uint32_t *out_len, uint32_t *out_src_ip,
                        uint16_t *out_src_port)
{
    for (uint32_t k = 0; k < count; k++) {
        const uint8_t *f = frames + offset[lane_pkt[first + k]];
        const uint32_t data_len = length[lane_pkt[first + k]];
        const uint16_t dgram_len = (uint16_t)(((uint32_t)f[38] << 8) | f[39]);
        const uint16_t dgram_payl_len = (uint16_t)(dgram_len - 8u);                 /* :436 */
        memcpy(&out_src_ip[k], f + 26, 4);                                          /* :447 */
        out_src_port[k] = (uint16_t)((uint32_t)f[34] | ((uint32_t)f[35] << 8));      /* :446 */
        uint32_t seg_len = data_len - 42u;                                          /* :458 */
        if (seg_len > dgram_payl_len) seg_len = dgram_payl_len;                     /* :459-462 */
        const uint32_t eff = seg_len < len ? seg_len : len;                         /* :464-468 */
        memcpy(out_payload + (size_t)k * len, f + 42, eff);                         /* :470 */
        out_len[k] = eff;                                                           /* :487 */
    }
}
