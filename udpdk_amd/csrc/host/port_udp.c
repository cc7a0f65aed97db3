/*
 * port_udp.c — a test wire for the poller thread: Ethernet frames carried one per datagram over a
 * kernel UDP socket ("[gpu] port = udp:<ip>:<port>" + "port_peer = <ip>:<port>" in the .ini).
 *
 * The reference forks a poller that busy-polls NIC port 0 (udpdk_init.c:293, :362-368), so an
 * unmodified application's udpdk_sendto / udpdk_recvfrom move packets without any further call
 * (apps/pingpong/main.c:87-91, :138-140; apps/pktgen/main.c:156, :197). With this port,
 * udpdk_init does the same: it starts the poller thread (udpdk_port_attach) on the wire, so two
 * processes running the reference's apps exchange datagrams through the GPU datapath (TX frames
 * built by tx_build on one side, classified and demultiplexed by rx_classify on the other).
 * "[gpu] port = loopback" attaches the built-in loopback port instead.
 *
 * Not a datapath: one recvmmsg / sendmmsg per burst, frames at a fixed 2 KiB stride (the
 * reference's mbuf data room, udpdk_init.c:78-79).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "host_state.h"

#define H_WIRE_STRIDE 2048u
#define H_WIRE_BURST  64u

static int g_wire_fd = -1;

static int h_parse_ep(const char *v, struct sockaddr_in *a)
{
    char ip[64];
    unsigned port;
    const char *c = strrchr(v, ':');
    if (!c || (size_t)(c - v) >= sizeof(ip)) return -1;
    memcpy(ip, v, (size_t)(c - v));
    ip[c - v] = 0;
    if (sscanf(c + 1, "%u", &port) != 1 || port > 65535) return -1;
    memset(a, 0, sizeof(*a));
    a->sin_family = AF_INET;
    a->sin_port = htons((uint16_t)port);
    return inet_pton(AF_INET, ip, &a->sin_addr) == 1 ? 0 : -1;
}

static uint32_t h_wire_rx(void *user, uint8_t *frames, uint64_t cap, uint32_t *off, uint16_t *len, uint32_t max)
{
    (void)user;
    struct mmsghdr m[H_WIRE_BURST];
    struct iovec v[H_WIRE_BURST];
    uint32_t k = (uint32_t)(cap / H_WIRE_STRIDE);
    if (k > max) k = max;
    if (k > H_WIRE_BURST) k = H_WIRE_BURST;
    if (!k) return 0;
    memset(m, 0, sizeof(m));
    for (uint32_t i = 0; i < k; i++) {
        v[i].iov_base = frames + (uint64_t)i * H_WIRE_STRIDE;
        v[i].iov_len = H_WIRE_STRIDE;
        m[i].msg_hdr.msg_iov = &v[i];
        m[i].msg_hdr.msg_iovlen = 1;
    }
    const int r = recvmmsg(g_wire_fd, m, k, MSG_DONTWAIT, NULL);
    if (r <= 0) return 0;
    uint32_t n = 0;
    for (int i = 0; i < r; i++) {
        if (m[i].msg_hdr.msg_flags & MSG_TRUNC) continue;       /* longer than an mbuf: dropped */
        off[n] = (uint32_t)i * H_WIRE_STRIDE;
        len[n] = (uint16_t)m[i].msg_len;
        n++;
    }
    return n;
}

static void h_wire_tx(void *user, const uint8_t *frames, const uint32_t *off, const uint16_t *len, uint32_t n)
{
    (void)user;
    struct mmsghdr m[H_WIRE_BURST];
    struct iovec v[H_WIRE_BURST];
    for (uint32_t b = 0; b < n; b += H_WIRE_BURST) {
        const uint32_t k = n - b < H_WIRE_BURST ? n - b : H_WIRE_BURST;
        memset(m, 0, sizeof(m));
        for (uint32_t i = 0; i < k; i++) {
            v[i].iov_base = (void *)(frames + off[b + i]);
            v[i].iov_len = len[b + i];
            m[i].msg_hdr.msg_iov = &v[i];
            m[i].msg_hdr.msg_iovlen = 1;
        }
        /* a peer that is not up yet refuses (ECONNREFUSED): the frames are lost, like frames
         * sent on a link whose other end is down */
        (void)sendmmsg(g_wire_fd, m, k, 0);
    }
}

int h_wire_open(const char *local, const char *peer, udpdk_port_ops_t *ops)
{
    struct sockaddr_in la, pa;
    if (h_parse_ep(local, &la) || h_parse_ep(peer, &pa)) { errno = EINVAL; return -1; }
    const int fd = socket(AF_INET, SOCK_DGRAM, 0);
    if (fd < 0) return -1;
    const int buf = 8 << 20;
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
    if (bind(fd, (struct sockaddr *)&la, sizeof(la)) || connect(fd, (struct sockaddr *)&pa, sizeof(pa))) {
        const int e = errno;
        close(fd);
        errno = e;
        return -1;
    }
    g_wire_fd = fd;
    memset(ops, 0, sizeof(*ops));
    ops->rx_burst = h_wire_rx;
    ops->tx_burst = h_wire_tx;
    ops->batch_frames = 256;
    return 0;
}

void h_wire_close(void)
{
    if (g_wire_fd >= 0) close(g_wire_fd);
    g_wire_fd = -1;
}
