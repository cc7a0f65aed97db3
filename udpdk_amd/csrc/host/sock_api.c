/*
 * sock_api.c — the socket calls of udpdk_api.h.
 *
 * Argument validation, errno values and slot state transitions follow udpdk_syscall.c
 * (socket :23-81, get/setsockopt :83-192, bind :194-245, sendto :247-368, recvfrom :370-488,
 * close :490-521). Deliberate fixes: close decrements the active count (the reference
 * increments it, :519) and sendto refuses payloads that would not fit the
 * reference's 2048-byte mbuf data room unfragmented (EMSGSIZE, §8 Q14).
 */
#include <errno.h>
#include <netinet/in.h>
#include <stdlib.h>
#include <string.h>

#include "host_state.h"

struct h_state g_udpdk;

#define H_MAX_PAYLOAD 1458   /* largest datagram sent unfragmented: 1500 - 42 (poller.c:461) */

static int h_valid_fd(int s) { return s >= 0 && s < UDPDK_MAX_SOCKETS; }

static void h_ring_clear(struct h_ring *r)
{
    if (r->e) {
        for (uint32_t i = r->head; i != r->tail; i++) free(r->e[i % UDPDK_RX_RING_SIZE].data);
        free(r->e);
    }
    r->e = NULL;
    r->head = r->tail = 0;
}

void h_sockets_reset(void)
{
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {
        h_ring_clear(&g_udpdk.slots[s].rx);
        memset(&g_udpdk.slots[s], 0, sizeof(g_udpdk.slots[s]));
        g_udpdk.slots[s].prev = g_udpdk.slots[s].next = -1;
    }
    g_udpdk.n_active = 0;
    g_udpdk.version++;
}

/* All-or-nothing append of n datagrams (rte_ring_enqueue_bulk semantics, poller.c:287-290).
 * On refusal the caller frees the datagrams. */
int h_ring_push_bulk(struct h_ring *r, struct h_dgram *d, uint32_t n)
{
    if (!r->e) {
        r->e = calloc(UDPDK_RX_RING_SIZE, sizeof(*r->e));
        if (!r->e) return -1;
    }
    if (r->tail - r->head + n > UDPDK_RX_RING_SIZE - 1) return -1;   /* usable size = size - 1 */
    for (uint32_t i = 0; i < n; i++) r->e[(r->tail + i) % UDPDK_RX_RING_SIZE] = d[i];
    r->tail += n;
    return 0;
}

int udpdk_socket(int domain, int type, int protocol)
{
    if (domain != AF_INET) { errno = EAFNOSUPPORT; return -1; }
    if (type != SOCK_DGRAM) { errno = EPROTONOSUPPORT; return -1; }
    if (protocol != 0 && protocol != IPPROTO_UDP) { errno = EINVAL; return -1; }
    if (g_udpdk.n_active >= UDPDK_MAX_SOCKETS) { errno = ENOBUFS; return -1; }
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
        return s;
    }
    errno = ENOBUFS;
    return -1;
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

int udpdk_bind(int s, const struct sockaddr *addr, socklen_t addrlen)
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

int udpdk_close(int s)
{
    if (!h_valid_fd(s) || !g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    struct h_slot *sl = &g_udpdk.slots[s];
    if (sl->bound) h_btable_del(s, sl->udp_port);
    h_ring_clear(&sl->rx);
    sl->bound = 0;
    sl->used = 0;
    sl->so_options = 0;
    g_udpdk.n_active--;
    return 0;
}

/* Auto-bind an unbound socket to ANY on the lowest free raw port (udpdk_syscall.c:294-304). */
static int h_autobind(int s)
{
    if (g_udpdk.slots[s].bound) return 0;
    struct sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    const int p = h_btable_free_port();
    if (p < 0) { errno = EADDRINUSE; return -1; }
    a.sin_port = (uint16_t)p;
    return udpdk_bind(s, (const struct sockaddr *)&a, sizeof(a));
}

static uint16_t h_ipv4_cksum(const uint8_t *ip)
{
    /* rte_raw_cksum + rte_ipv4_cksum, DPDK 20.05: raw 0xffff kept as is */
    uint32_t s = 0;
    for (int i = 0; i < 20; i += 2) s += (uint32_t)ip[i] | ((uint32_t)ip[i + 1] << 8);
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    const uint16_t raw = (uint16_t)s;
    return raw == 0xFFFFu ? raw : (uint16_t)~raw;
}

ssize_t h_build_frame(int s, const void *buf, size_t len, uint32_t dst_ip, uint32_t dst_port,
                      uint8_t *f)
{
    const struct h_slot *sl = &g_udpdk.slots[s];
    memcpy(f, g_udpdk.dst_mac, 6);
    memcpy(f + 6, g_udpdk.src_mac, 6);
    f[12] = 0x08; f[13] = 0x00;
    uint8_t *ip = f + 14;
    memset(ip, 0, 20);
    ip[0] = 0x45;
    ip[8] = 64;
    ip[9] = 17;
    const uint32_t src = (sl->bound && sl->ip != 0) ? sl->ip : g_udpdk.src_ip;
    memcpy(ip + 12, &src, 4);
    memcpy(ip + 16, &dst_ip, 4);
    const uint32_t tl = (uint32_t)len + 28;
    ip[2] = (uint8_t)(tl >> 8); ip[3] = (uint8_t)tl;
    const uint16_t ck = h_ipv4_cksum(ip);
    memcpy(ip + 10, &ck, 2);
    uint8_t *u = f + 34;
    u[0] = (uint8_t)sl->udp_port; u[1] = (uint8_t)(sl->udp_port >> 8);
    u[2] = (uint8_t)dst_port; u[3] = (uint8_t)(dst_port >> 8);
    const uint32_t ul = (uint32_t)len + 8;
    u[4] = (uint8_t)(ul >> 8); u[5] = (uint8_t)ul;
    u[6] = u[7] = 0;
    if (len) memcpy(f + 42, buf, len);
    return (ssize_t)len + 42;
}

static int h_sendto_check(int s, size_t len, int flags, const struct sockaddr *dest, socklen_t addrlen)
{
    if (s < 0 || s >= UDPDK_MAX_SOCKETS) { errno = ENOTSOCK; return -1; }
    if (!g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (flags != 0) { errno = EINVAL; return -1; }
    if (!dest || addrlen == 0) { errno = EINVAL; return -1; }
    if (len > H_MAX_PAYLOAD) { errno = EMSGSIZE; return -1; }
    return 0;
}

ssize_t udpdk_build_frame(int s, const void *buf, size_t len, const struct sockaddr *dest,
                          socklen_t addrlen, uint8_t *out)
{
    if (h_sendto_check(s, len, 0, dest, addrlen)) return -1;
    if (h_autobind(s)) return -1;
    const struct sockaddr_in *d = (const struct sockaddr_in *)dest;
    return h_build_frame(s, buf, len, d->sin_addr.s_addr, d->sin_port, out);
}

ssize_t udpdk_sendto(int s, const void *buf, size_t len, int flags,
                     const struct sockaddr *dest, socklen_t addrlen)
{
    if (h_sendto_check(s, len, flags, dest, addrlen)) return -1;
    if (h_autobind(s)) return -1;
    const uint64_t need = g_udpdk.txq_bytes + len + 42;
    if (need > g_udpdk.txq_cap) {
        uint64_t nc = g_udpdk.txq_cap ? g_udpdk.txq_cap * 2 : (1u << 20);
        while (nc < need) nc *= 2;
        uint8_t *nq = realloc(g_udpdk.txq, nc);
        if (!nq) { errno = ENOMEM; return -1; }
        g_udpdk.txq = nq;
        g_udpdk.txq_cap = nc;
    }
    if (g_udpdk.txq_n == g_udpdk.txq_ncap) {
        uint32_t nc = g_udpdk.txq_ncap ? g_udpdk.txq_ncap * 2 : 1024;
        uint32_t *nl = realloc(g_udpdk.txq_len, (size_t)nc * sizeof(uint32_t));
        if (!nl) { errno = ENOMEM; return -1; }
        g_udpdk.txq_len = nl;
        g_udpdk.txq_ncap = nc;
    }
    const struct sockaddr_in *d = (const struct sockaddr_in *)dest;
    const ssize_t fl = h_build_frame(s, buf, len, d->sin_addr.s_addr, d->sin_port,
                                     g_udpdk.txq + g_udpdk.txq_bytes);
    g_udpdk.txq_len[g_udpdk.txq_n++] = (uint32_t)fl;
    g_udpdk.txq_bytes += (uint64_t)fl;
    return (ssize_t)len;
}

int udpdk_tx_drain(uint8_t *out, uint64_t out_cap, uint32_t *out_off, uint16_t *out_len,
                   uint32_t max, uint32_t *n_out)
{
    if (!n_out || (max && (!out || !out_off || !out_len))) { errno = EINVAL; return -1; }
    uint32_t k = 0;
    uint64_t pos = 0;
    while (k < max && k < g_udpdk.txq_n && pos + g_udpdk.txq_len[k] <= out_cap) {
        out_off[k] = (uint32_t)pos;
        out_len[k] = (uint16_t)g_udpdk.txq_len[k];
        pos += g_udpdk.txq_len[k];
        k++;
    }
    if (pos) memcpy(out, g_udpdk.txq, pos);
    memmove(g_udpdk.txq, g_udpdk.txq + pos, g_udpdk.txq_bytes - pos);
    memmove(g_udpdk.txq_len, g_udpdk.txq_len + k, (size_t)(g_udpdk.txq_n - k) * sizeof(uint32_t));
    g_udpdk.txq_bytes -= pos;
    g_udpdk.txq_n -= k;
    *n_out = k;
    return 0;
}

ssize_t udpdk_recvfrom(int s, void *buf, size_t len, int flags,
                       struct sockaddr *src_addr, socklen_t *addrlen)
{
    if (s < 0 || s >= UDPDK_MAX_SOCKETS) { errno = ENOTSOCK; return -1; }
    if (!g_udpdk.slots[s].used) { errno = EBADF; return -1; }
    if (flags != 0) { errno = EINVAL; return -1; }
    if (buf == NULL && addrlen != NULL) { errno = EINVAL; return -1; }
    struct h_ring *r = &g_udpdk.slots[s].rx;
    while (r->head == r->tail && !g_udpdk.interrupted) {
        /* busy wait like udpdk_syscall.c:424-426; datagrams arrive via udpdk_poll_rx */
    }
    if (g_udpdk.interrupted) { errno = EINTR; return -1; }
    struct h_dgram d = r->e[r->head % UDPDK_RX_RING_SIZE];
    r->head++;
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
    const size_t n = d.len < len ? d.len : len;
    if (n) memcpy(buf, d.data, n);
    free(d.data);
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
