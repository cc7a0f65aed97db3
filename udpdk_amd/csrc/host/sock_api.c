/*
 * sock_api.c — the socket calls of udpdk_api.h, the RX rings and payload slabs, the TX rings.
 *
 * Argument validation, errno values and slot state transitions follow udpdk_syscall.c
 * (socket :23-81, get/setsockopt :83-192, bind :194-245, sendto :247-368, recvfrom :370-488,
 * close :490-521). Deliberate fixes: close decrements the active count (the reference
 * increments it, :519), and sendto accepts payloads up to 65507 bytes, which
 * the poller's TX fragmentation carries (the reference writes past its 2048-byte mbuf above
 * 2006 bytes, §8 Q14); larger ones get EMSGSIZE.
 *
 * sendto does what the reference's sendto does short of building the frame: validate, auto-bind,
 * queue the datagram on the socket's TX ring (ENOBUFS when full, :356-365). The frame is built
 * on the GPU by the poller's TX half (udpdk_tx_drain). recvfrom pops the socket's RX ring and
 * copies the payload out of the pinned slab the poller gathered it into on the GPU.
 */
#include <errno.h>
#include <netinet/in.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

#include "host_state.h"

#ifndef UDPDK_RECV_PREFETCH
#define UDPDK_RECV_PREFETCH 4096u      /* bytes of the next datagram prefetched by recvfrom */
#endif

struct h_state g_udpdk;

static int h_valid_fd(int s) { return s >= 0 && s < UDPDK_MAX_SOCKETS; }

/* ---- RX rings: single producer (the poller), single consumer (recvfrom) ------------------- */
static void h_ring_clear(struct h_ring *r)
{
    h_arena_release(r->rel_arena, r->rel_n);
    r->rel_arena = NULL;
    r->rel_n = 0;
    if (r->e) {
        const uint32_t t = atomic_load_explicit(&r->tail, memory_order_acquire);
        for (uint32_t i = atomic_load_explicit(&r->head, memory_order_relaxed); i != t; i++)
            h_arena_release(r->e[i % UDPDK_RX_RING_SIZE].arena, 1);
        free(r->e);
    }
    r->e = NULL;
    atomic_store_explicit(&r->head, 0, memory_order_relaxed);
    atomic_store_explicit(&r->tail, 0, memory_order_relaxed);
}

/* Entries the producer may still add (usable size = size - 1, as rte_ring). */
uint32_t h_ring_free(const struct h_ring *r)
{
    const uint32_t h = atomic_load_explicit(&r->head, memory_order_acquire);
    const uint32_t t = atomic_load_explicit(&r->tail, memory_order_relaxed);
    return (UDPDK_RX_RING_SIZE - 1) - (t - h);
}

/* All-or-nothing append of n datagrams (rte_ring_enqueue_bulk, poller.c:287-290): the entries
 * are written first, then published by a release store of tail that recvfrom acquires. */
int h_ring_push_bulk(struct h_ring *r, const struct h_dgram *d, uint32_t n)
{
    if (!r->e) {
        r->e = calloc(UDPDK_RX_RING_SIZE, sizeof(*r->e));
        if (!r->e) return -1;
    }
    if (n > h_ring_free(r)) return -1;
    const uint32_t t = atomic_load_explicit(&r->tail, memory_order_relaxed);
    for (uint32_t i = 0; i < n; i++) r->e[(t + i) % UDPDK_RX_RING_SIZE] = d[i];
    atomic_store_explicit(&r->tail, t + n, memory_order_release);
    return 0;
}

/* ---- payload slabs ------------------------------------------------------------------------ */
#define H_ARENA_FREE_KEEP 32     /* free slabs kept for reuse; the rest go back to the runtime
                                  * (a pipelined poll makes a slab per chunk: with 8 kept, every
                                  * 1 M x 1500 B poll freed and re-pinned three 140 MB slabs) */

/* frees a slab's memory; the budget accounting is the caller's */
static void h_arena_destroy(struct h_arena *a)
{
    if (!a) return;
    void *p[] = {a->payload, a->len, a->src_ip, a->src_port};
    for (unsigned k = 0; k < 4; k++)
        if (p[k] && g_udpdk.gpu) udpdk_gpu_host_free(g_udpdk.gpu, p[k]);
    free(a);
}

static uint64_t h_arena_footprint(uint64_t cb, uint32_t cn) { return cb + 10ull * cn; }

/* A slab for n datagrams in `need` bytes of packed slots: the first free one that is large
 * enough, else a new one (pinned, so the gather's D2H is a straight DMA) if the slab budget
 * allows it after the free slabs that do not fit have been released. NULL + ENOBUFS when the
 * budget is exhausted by slabs that queued datagrams still hold (the reference's mbuf pool
 * exhausted: the burst is not received). */
struct h_arena *h_arena_get(uint32_t n, uint64_t need)
{
    pthread_mutex_lock(&g_udpdk.arena_lock);
    /* the smallest free slab that fits (a pipelined poll asks for one slab per chunk, of
     * similar sizes: first fit handed a chunk a larger one that a later chunk then missed) */
    struct h_arena **best = NULL, *a = NULL;
    for (struct h_arena **pp = &g_udpdk.arena_free; *pp; pp = &(*pp)->next)
        if ((*pp)->cap_bytes >= need && (*pp)->cap_n >= n && (!best || (*pp)->cap_bytes < (*best)->cap_bytes))
            best = pp;
    if (best) {
        a = *best;
        *best = a->next;
        g_udpdk.arena_free_n--;
    }
    /* a new slab's capacity rounded up to 1/8 of its power of two (<= 12.5 % more), so the next
     * poll's slightly larger chunk still fits it */
    const uint32_t cn0 = n < 4096 ? 4096 : n;
    const uint32_t cn = cn0 > (1u << 16) ? (cn0 + 8191u) & ~8191u : cn0;
    uint64_t cb = need < ((uint64_t)cn * 64) ? (uint64_t)cn * 64 : need;
    if (cb > (1ull << 20)) {
        uint64_t p2 = 1ull << 20;
        while (p2 <= cb / 2) p2 <<= 1;
        const uint64_t g = p2 / 8;
        cb = (cb + g - 1) / g * g;
    }
    if (!a) {
        const uint64_t fp = h_arena_footprint(cb, cn);
        /* release free slabs (none fits) until the new one fits the budget */
        while ((g_udpdk.arena_bytes + fp > g_udpdk.arena_bytes_max ||
                g_udpdk.arena_count + 1 > g_udpdk.arena_count_max) && g_udpdk.arena_free) {
            struct h_arena *f = g_udpdk.arena_free;
            g_udpdk.arena_free = f->next;
            g_udpdk.arena_free_n--;
            g_udpdk.arena_bytes -= h_arena_footprint(f->cap_bytes, f->cap_n);
            g_udpdk.arena_count--;
            h_arena_destroy(f);
        }
        if (g_udpdk.arena_bytes + fp > g_udpdk.arena_bytes_max ||
            g_udpdk.arena_count + 1 > g_udpdk.arena_count_max) {
            pthread_mutex_unlock(&g_udpdk.arena_lock);
            errno = ENOBUFS;
            return NULL;
        }
        g_udpdk.arena_bytes += fp;         /* reserved before the allocation */
        g_udpdk.arena_count++;
    }
    pthread_mutex_unlock(&g_udpdk.arena_lock);
    if (!a) {
        a = calloc(1, sizeof(*a));
        if (a && (udpdk_gpu_host_alloc(g_udpdk.gpu, cb, (void **)&a->payload) ||
                  udpdk_gpu_host_alloc(g_udpdk.gpu, 4ull * cn, (void **)&a->len) ||
                  udpdk_gpu_host_alloc(g_udpdk.gpu, 4ull * cn, (void **)&a->src_ip) ||
                  udpdk_gpu_host_alloc(g_udpdk.gpu, 2ull * cn, (void **)&a->src_port))) {
            h_arena_destroy(a);
            a = NULL;
        }
        if (!a) {
            pthread_mutex_lock(&g_udpdk.arena_lock);
            g_udpdk.arena_bytes -= h_arena_footprint(cb, cn);
            g_udpdk.arena_count--;
            pthread_mutex_unlock(&g_udpdk.arena_lock);
            errno = ENOMEM;
            return NULL;
        }
        a->cap_bytes = cb;
        a->cap_n = cn;
    }
    a->next = NULL;
    atomic_store_explicit(&a->refs, 0, memory_order_relaxed);
    return a;
}

/* Back to the pool; beyond H_ARENA_FREE_KEEP free slabs the largest goes back to the runtime,
 * so one burst of huge polls does not keep its slabs pinned forever. */
void h_arena_put(struct h_arena *a)
{
    pthread_mutex_lock(&g_udpdk.arena_lock);
    a->next = g_udpdk.arena_free;
    g_udpdk.arena_free = a;
    g_udpdk.arena_free_n++;
    struct h_arena *victim = NULL;
    if (g_udpdk.arena_free_n > H_ARENA_FREE_KEEP) {
        struct h_arena **vp = &g_udpdk.arena_free;
        for (struct h_arena **pp = &g_udpdk.arena_free; *pp; pp = &(*pp)->next)
            if ((*pp)->cap_bytes > (*vp)->cap_bytes) vp = pp;
        victim = *vp;
        *vp = victim->next;
        g_udpdk.arena_free_n--;
        g_udpdk.arena_bytes -= h_arena_footprint(victim->cap_bytes, victim->cap_n);
        g_udpdk.arena_count--;
    }
    pthread_mutex_unlock(&g_udpdk.arena_lock);
    h_arena_destroy(victim);
}

/* Drop refs references (recvfrom of one datagram, or a ring cleared by close); the last one
 * returns the slab to the pool. */
void h_arena_release(struct h_arena *a, uint32_t refs)
{
    if (a && refs && atomic_fetch_sub_explicit(&a->refs, refs, memory_order_acq_rel) == refs)
        h_arena_put(a);
}

void h_arenas_free_all(void)
{
    pthread_mutex_lock(&g_udpdk.arena_lock);
    struct h_arena *a = g_udpdk.arena_free;
    g_udpdk.arena_free = NULL;
    g_udpdk.arena_free_n = 0;
    while (a) {
        struct h_arena *n = a->next;
        g_udpdk.arena_bytes -= h_arena_footprint(a->cap_bytes, a->cap_n);
        g_udpdk.arena_count--;
        h_arena_destroy(a);
        a = n;
    }
    pthread_mutex_unlock(&g_udpdk.arena_lock);
}

uint64_t udpdk_rx_nobufs(void) { return __atomic_load_n(&g_udpdk.rx_nobufs, __ATOMIC_RELAXED); }

/* ---- TX rings ----------------------------------------------------------------------------- */
void h_tx_reset(void)
{
    pthread_mutex_lock(&g_udpdk.tx_lock);
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {
        free(g_udpdk.slots[s].tx.e);
        g_udpdk.slots[s].tx.e = NULL;
        g_udpdk.slots[s].tx.head = g_udpdk.slots[s].tx.tail = 0;
    }
    free(g_udpdk.txp);
    g_udpdk.txp = NULL;
    g_udpdk.txp_bytes = g_udpdk.txp_cap = 0;
    g_udpdk.tx_queued = 0;
    g_udpdk.tx_dropped = 0;
    pthread_mutex_unlock(&g_udpdk.tx_lock);
}

uint64_t udpdk_tx_pending(void)
{
    pthread_mutex_lock(&g_udpdk.tx_lock);
    const uint64_t q = g_udpdk.tx_queued;
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    return q;
}

uint64_t udpdk_tx_dropped(void)
{
    pthread_mutex_lock(&g_udpdk.tx_lock);
    const uint64_t q = g_udpdk.tx_dropped;
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    return q;
}

void h_sockets_reset(void)
{
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {
        h_ring_clear(&g_udpdk.slots[s].rx);
        free(g_udpdk.slots[s].tx.e);
        memset(&g_udpdk.slots[s], 0, sizeof(g_udpdk.slots[s]));
        g_udpdk.slots[s].prev = g_udpdk.slots[s].next = -1;
    }
    g_udpdk.n_active = 0;
    free(g_udpdk.txp);
    g_udpdk.txp = NULL;
    g_udpdk.txp_bytes = g_udpdk.txp_cap = 0;
    g_udpdk.tx_queued = 0;
    g_udpdk.tx_dropped = 0;
    __atomic_store_n(&g_udpdk.rx_nobufs, 0, __ATOMIC_RELAXED);   /* per library session */
    g_udpdk.version++;
}

/* ---- socket calls ------------------------------------------------------------------------- */
int udpdk_socket(int domain, int type, int protocol)
{
    if (domain != AF_INET) { errno = EAFNOSUPPORT; return -1; }
    if (type != SOCK_DGRAM) { errno = EPROTONOSUPPORT; return -1; }
    if (protocol != 0 && protocol != IPPROTO_UDP) { errno = EINVAL; return -1; }
    pthread_mutex_lock(&g_udpdk.lock);
    int ret = -1;
    if (g_udpdk.n_active >= UDPDK_MAX_SOCKETS) {
        errno = ENOBUFS;
    } else {
        for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {   /* lowest free slot */
            struct h_slot *sl = &g_udpdk.slots[s];
            if (sl->used) continue;
            sl->used = 1;
            sl->bound = 0;
            sl->so_options = 0;
            sl->ip = 0;
            sl->udp_port = 0;
            sl->prev = sl->next = -1;
            g_udpdk.n_active++;
            ret = s;
            break;
        }
        if (ret < 0) errno = ENOBUFS;
    }
    pthread_mutex_unlock(&g_udpdk.lock);
    return ret;
}

static int h_sockopt_check(int s, int level, int optname, const void *optval, const void *optlen)
{
    if (!h_valid_fd(s) || !g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (level != SOL_SOCKET) { errno = EINVAL; return -1; }
    if (optname != SO_REUSEADDR && optname != SO_REUSEPORT) { errno = ENOPROTOOPT; return -1; }
    if (!optval || !optlen) { errno = EFAULT; return -1; }
    return 0;
}

int udpdk_getsockopt(int s, int level, int optname, void *optval, socklen_t *optlen)
{
    if (h_sockopt_check(s, level, optname, optval, optlen)) return -1;
    /* bitwise test of the option value: SO_REUSEPORT (15) contains SO_REUSEADDR (2), so
     * setting REUSEPORT reads back REUSEADDR = 1 as in the reference */
    *(int *)optval = (g_udpdk.slots[s].so_options & optname) != 0;
    return 0;
}

int udpdk_setsockopt(int s, int level, int optname, const void *optval, socklen_t optlen)
{
    if (h_sockopt_check(s, level, optname, optval, &optlen)) return -1;
    struct h_slot *sl = &g_udpdk.slots[s];
    const int was = sl->so_options & optname;
    const int want = *(const int *)optval != 0;
    if (want && !was) sl->so_options |= optname;
    else if (!want && was) sl->so_options &= ~optname;
    return 0;
}

static int h_bind_locked(int s, const struct sockaddr *addr, socklen_t addrlen)
{
    if (!h_valid_fd(s) || !g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (g_udpdk.slots[s].bound) { errno = EINVAL; return -1; }
    if (!addr || addr->sa_family != AF_INET) { errno = EINVAL; return -1; }
    if (addrlen != sizeof(struct sockaddr_in)) { errno = EINVAL; return -1; }
    const struct sockaddr_in *in = (const struct sockaddr_in *)addr;
    const uint32_t port = in->sin_port;            /* raw network-order value */
    const uint32_t ip = in->sin_addr.s_addr;
    if (h_btable_add(s, ip, port, g_udpdk.slots[s].so_options) < 0) { errno = EADDRINUSE; return -1; }
    g_udpdk.slots[s].bound = 1;
    g_udpdk.slots[s].udp_port = port;
    g_udpdk.slots[s].ip = ip;
    return 0;
}

int udpdk_bind(int s, const struct sockaddr *addr, socklen_t addrlen)
{
    pthread_mutex_lock(&g_udpdk.lock);
    const int rc = h_bind_locked(s, addr, addrlen);
    pthread_mutex_unlock(&g_udpdk.lock);
    return rc;
}

int udpdk_close(int s)
{
    pthread_mutex_lock(&g_udpdk.lock);
    if (!h_valid_fd(s) || !g_udpdk.slots[s].used) {
        pthread_mutex_unlock(&g_udpdk.lock);
        errno = EBADF;
        return -1;
    }
    struct h_slot *sl = &g_udpdk.slots[s];
    /* a recvfrom blocked on this socket in another thread leaves with EBADF before the ring's
     * entries and storage go (it would otherwise read freed entries) */
    atomic_store(&sl->rx.closing, 1);
    while (atomic_load(&sl->rx.busy)) sched_yield();
    if (sl->bound) h_btable_del(s, sl->udp_port);
    h_ring_clear(&sl->rx);
    pthread_mutex_lock(&g_udpdk.tx_lock);
    if (sl->tx.e) {
        g_udpdk.tx_queued -= sl->tx.tail - sl->tx.head;   /* queued sends die with the socket */
        free(sl->tx.e);
    }
    sl->tx.e = NULL;
    sl->tx.head = sl->tx.tail = 0;
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    sl->bound = 0;
    sl->used = 0;
    sl->so_options = 0;
    g_udpdk.n_active--;
    g_udpdk.version++;
    atomic_store(&sl->rx.closing, 0);          /* later calls see used == 0 */
    pthread_mutex_unlock(&g_udpdk.lock);
    return 0;
}

/* Auto-bind an unbound socket to ANY on the lowest free raw port (udpdk_syscall.c:294-304). */
static int h_autobind_locked(int s)
{
    if (g_udpdk.slots[s].bound) return 0;
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    const int p = h_btable_free_port();
    if (p < 0) { errno = EADDRINUSE; return -1; }
    a.sin_port = (uint16_t)p;
    return h_bind_locked(s, (const struct sockaddr *)&a, sizeof(a));
}

ssize_t udpdk_sendto(int s, const void *buf, size_t len, int flags,
                     const struct sockaddr *dest, socklen_t addrlen)
{
    if (s < 0 || s >= UDPDK_MAX_SOCKETS) { errno = ENOTSOCK; return -1; }
    if (!g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (flags != 0) { errno = EINVAL; return -1; }
    if (!dest || addrlen == 0) { errno = EINVAL; return -1; }
    if (len > H_UDP_MAX_PAYLOAD) { errno = EMSGSIZE; return -1; }
    if (len && !buf) { errno = EFAULT; return -1; }
    pthread_mutex_lock(&g_udpdk.lock);
    const int rc = h_autobind_locked(s);
    pthread_mutex_unlock(&g_udpdk.lock);
    if (rc) return -1;
    const struct sockaddr_in *d = (const struct sockaddr_in *)dest;
    pthread_mutex_lock(&g_udpdk.tx_lock);
    struct h_txq *q = &g_udpdk.slots[s].tx;
    ssize_t ret = -1;
    if (!q->e && !(q->e = malloc(UDPDK_RX_RING_SIZE * sizeof(*q->e)))) {
        errno = ENOMEM;
    } else if (q->tail - q->head >= UDPDK_RX_RING_SIZE - 1) {
        errno = ENOBUFS;                           /* rte_ring_enqueue failed (:356-365) */
    } else {
        const uint64_t need = g_udpdk.txp_bytes + len;
        if (need > g_udpdk.txp_cap) {
            uint64_t nc = g_udpdk.txp_cap ? g_udpdk.txp_cap * 2 : (1u << 20);
            while (nc < need) nc *= 2;
            uint8_t *np = realloc(g_udpdk.txp, nc);
            if (!np) { errno = ENOMEM; goto out; }
            g_udpdk.txp = np;
            g_udpdk.txp_cap = nc;
        }
        struct h_txd *t = &q->e[q->tail % UDPDK_RX_RING_SIZE];
        t->pay = g_udpdk.txp_bytes;
        t->len = (uint32_t)len;
        t->dst_ip = d->sin_addr.s_addr;
        t->dst_port = d->sin_port;
        if (len) memcpy(g_udpdk.txp + g_udpdk.txp_bytes, buf, len);
        g_udpdk.txp_bytes += len;
        q->tail++;
        g_udpdk.tx_queued++;
        ret = (ssize_t)len;
    }
out:
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    return ret;
}

ssize_t udpdk_recvfrom(int s, void *buf, size_t len, int flags,
                       struct sockaddr *src_addr, socklen_t *addrlen)
{
    if (s < 0 || s >= UDPDK_MAX_SOCKETS) { errno = ENOTSOCK; return -1; }
    if (!g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (flags != 0) { errno = EINVAL; return -1; }
    if (buf == NULL && addrlen != NULL) { errno = EINVAL; return -1; }
    struct h_ring *r = &g_udpdk.slots[s].rx;
    atomic_fetch_add(&r->busy, 1);             /* seq_cst: see udpdk_close */
    if (atomic_load(&r->closing) || !g_udpdk.slots[s].used) {
        atomic_fetch_sub_explicit(&r->busy, 1, memory_order_release);
        errno = EBADF;
        return -1;
    }
    const uint32_t h = atomic_load_explicit(&r->head, memory_order_relaxed);
    /* busy wait like udpdk_syscall.c:424-426; datagrams arrive from the poller (udpdk_poll_rx) */
    while (atomic_load_explicit(&r->tail, memory_order_acquire) == h) {
        const int intr = atomic_load_explicit(&g_udpdk.interrupted, memory_order_relaxed);
        if (intr || atomic_load_explicit(&r->closing, memory_order_relaxed)) {
            atomic_fetch_sub_explicit(&r->busy, 1, memory_order_release);
            errno = intr ? EINTR : EBADF;
            return -1;
        }
        sched_yield();
    }
    const struct h_dgram d = r->e[h % UDPDK_RX_RING_SIZE];
    if (src_addr && addrlen) {
        struct sockaddr_in a;
        memset(&a, 0, sizeof(a));
        a.sin_family = AF_INET;
        a.sin_port = (uint16_t)d.src_port;
        a.sin_addr.s_addr = d.src_ip;
        const socklen_t n = sizeof(a) <= *addrlen ? (socklen_t)sizeof(a) : *addrlen;
        memcpy(src_addr, &a, n);
        *addrlen = n;
    }
    const uint32_t t = atomic_load_explicit(&r->tail, memory_order_acquire);
    if (t != h + 1) {
        /* the next datagram's bytes are fetched while this one is copied: recvfrom at 1500 B is
         * one memcpy out of host memory per call, bound by the core's cache misses (two entries
         * ahead measured even at 1500 B and 8 % slower at IMIX). Only the first
         * UDPDK_RECV_PREFETCH bytes: a 64 KiB datagram would otherwise issue 1024 prefetches
         * competing with this call's own copy (the hardware prefetcher follows the memcpy's
         * stream past them) */
        const struct h_dgram *nx = &r->e[(h + 1) % UDPDK_RX_RING_SIZE];
        const char *np = (const char *)nx->data;
        const uint32_t pf = nx->len < UDPDK_RECV_PREFETCH ? nx->len : UDPDK_RECV_PREFETCH;
        for (uint32_t o = 0; o < pf; o += 64) __builtin_prefetch(np + o);
    }
    const size_t n = d.len < len ? d.len : len;
    if (n) memcpy(buf, d.data, n);
    /* the slab reference goes back once per run of one slab's entries: when the next entry is
     * another slab's or the ring is drained (a consumed entry never holds its slab longer than an
     * unconsumed one would) */
    if (d.arena != r->rel_arena) {
        h_arena_release(r->rel_arena, r->rel_n);
        r->rel_arena = d.arena;
        r->rel_n = 0;
    }
    r->rel_n++;
    const bool run_ends = t == h + 1 || r->e[(h + 1) % UDPDK_RX_RING_SIZE].arena != d.arena;
    atomic_store_explicit(&r->head, h + 1, memory_order_release);
    if (run_ends) {
        h_arena_release(r->rel_arena, r->rel_n);
        r->rel_arena = NULL;
        r->rel_n = 0;
    }
    atomic_fetch_sub_explicit(&r->busy, 1, memory_order_release);
    return (ssize_t)n;
}

int udpdk_slot_table(udpdk_slot_t *slots, uint32_t n_slots)
{
    if (!slots) { errno = EINVAL; return -1; }
    for (uint32_t s = 0; s < n_slots; s++) {
        const struct h_slot *sl = s < UDPDK_MAX_SOCKETS ? &g_udpdk.slots[s] : NULL;
        slots[s].ip = sl ? sl->ip : 0u;
        slots[s].udp_port = sl ? sl->udp_port : 0u;
        slots[s].bound = sl ? (uint32_t)sl->bound : 0u;
    }
    return 0;
}
