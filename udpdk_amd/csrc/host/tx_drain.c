/*
 * tx_drain.c — udpdk_tx_drain: the poller's TX half (udpdk_poller.c:453-514) on the GPU.
 *
 * Selection follows the poller loop: sockets in index order, each socket's TX ring dequeued
 * while the burst holds fewer than BURST_SIZE frames (a datagram longer than the MTU counts as
 * its fragments, :461-501), the burst flushed when it reaches BURST_SIZE, and the loop repeated
 * until the rings are empty or the caller's frame / byte limits stop it. The selected
 * datagrams' payloads go to the GPU in one pinned H2D, udpdk_gpu_tx_build_mtu builds every frame
 * (Ethernet/IPv4/UDP headers from the slot table of the uploaded bind snapshot, rte_ipv4_cksum,
 * payload copy, fragmentation at the MTU) and one D2H returns them.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "host_state.h"

void h_tx_buffers_free(void)
{
    if (g_udpdk.tx_h && g_udpdk.gpu) udpdk_gpu_host_free(g_udpdk.gpu, g_udpdk.tx_h);
    if (g_udpdk.tx_d && g_udpdk.gpu) udpdk_gpu_free(g_udpdk.gpu, g_udpdk.tx_d);
    if (g_udpdk.tx_fr_d && g_udpdk.gpu) udpdk_gpu_free(g_udpdk.gpu, g_udpdk.tx_fr_d);
    g_udpdk.tx_h = g_udpdk.tx_d = g_udpdk.tx_fr_d = NULL;
    g_udpdk.tx_h_cap = g_udpdk.tx_d_cap = g_udpdk.tx_fr_d_cap = 0;
    free(g_udpdk.tx_sel);
    g_udpdk.tx_sel = NULL;
    g_udpdk.tx_sel_cap = 0;
}

int h_grow_pinned(void **p, uint64_t *cap, uint64_t need)
{
    if (*p && *cap >= need) return 0;
    if (*p) udpdk_gpu_host_free(g_udpdk.gpu, *p);
    *p = NULL;
    *cap = 0;
    const uint64_t nc = need < (1u << 16) ? (1u << 16) : need + need / 4;
    const int rc = udpdk_gpu_host_alloc(g_udpdk.gpu, nc, p);
    if (rc) { errno = -rc; return -1; }
    *cap = nc;
    return 0;
}

static inline uint64_t a16(uint64_t x) { return (x + 15u) & ~(uint64_t)15u; }

int udpdk_tx_drain(uint8_t *out, uint64_t out_cap, uint32_t *out_off, uint16_t *out_len,
                   uint32_t max, uint32_t *n_out)
{
    if (!n_out || (max && (!out || !out_off || !out_len))) { errno = EINVAL; return -1; }
    *n_out = 0;
    if (!g_udpdk.gpu) { errno = ENODEV; return -1; }
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    const uint32_t mtu = g_udpdk.mtu;
    /* the slot table the TX kernel reads (source port and address per socket). tx_lock is taken
     * before the table lock is dropped (the order udpdk_close uses): a sendto that auto-binds, or
     * a close + socket + bind, either lands before the refresh (and is in the uploaded table) or
     * queues its datagram only after this drain has released tx_lock, so no datagram selected
     * below is built from a slot row older than its socket's binding. */
    pthread_mutex_lock(&g_udpdk.lock);
    const int src = h_snapshot_refresh();
    if (src) {
        pthread_mutex_unlock(&g_udpdk.lock);
        return -1;
    }
    pthread_mutex_lock(&g_udpdk.tx_lock);
    pthread_mutex_unlock(&g_udpdk.lock);
    int ret = -1, rc;
    /* 1. selection in the poller's order */
    uint32_t nsel = 0, nframes = 0, burst = 0;
    uint64_t bytes = 0, pay = 0;
    int progress = 1, full = 0;
    uint32_t taken[UDPDK_MAX_SOCKETS];
    memset(taken, 0, sizeof(taken));
    while (progress && !full) {
        progress = 0;
        for (int s = 0; s < UDPDK_MAX_SOCKETS && !full; s++) {
            struct h_txq *q = &g_udpdk.slots[s].tx;
            if (!g_udpdk.slots[s].used || !q->e) continue;
            while (burst < H_BURST_SIZE && q->head + taken[s] != q->tail) {
                const struct h_txd *t = &q->e[(q->head + taken[s]) % UDPDK_RX_RING_SIZE];
                uint32_t nf = 1;
                const uint64_t span = udpdk_gpu_tx_span(t->len, mtu, &nf);
                if (nframes + nf > max || bytes + span > out_cap) {
                    if (nframes == 0 && taken[s] == 0 && (nf > max || span > out_cap)) {
                        /* larger than any drain with these limits can carry: it would block
                         * the ring's head forever. Dropped and counted (udpdk_tx_dropped), as
                         * the reference's poller drops a burst it cannot send. */
                        q->head++;
                        g_udpdk.tx_queued--;
                        g_udpdk.tx_dropped++;
                        continue;
                    }
                    full = 1;
                    break;
                }
                if (nsel + 1 > g_udpdk.tx_sel_cap) {
                    const uint64_t nc = g_udpdk.tx_sel_cap ? 2 * g_udpdk.tx_sel_cap : 4096;
                    void *ns = realloc(g_udpdk.tx_sel, nc * sizeof(*g_udpdk.tx_sel));
                    if (!ns) { errno = ENOMEM; goto out; }
                    g_udpdk.tx_sel = ns;
                    g_udpdk.tx_sel_cap = nc;
                }
                g_udpdk.tx_sel[nsel].s = s;
                g_udpdk.tx_sel[nsel].nf = nf;
                g_udpdk.tx_sel[nsel].foff = bytes;
                nsel++;
                taken[s]++;
                nframes += nf;
                bytes += span;
                pay += t->len;
                burst += nf;
                progress = 1;
            }
            if (burst >= H_BURST_SIZE) burst = 0;           /* flush_tx_table */
        }
        burst = 0;                                           /* end of the loop's TX half */
    }
    if (!nsel) {
        if (!g_udpdk.tx_queued) g_udpdk.txp_bytes = 0;   /* only dropped ones were left */
        ret = 0;
        goto out;
    }
    /* 2. host staging (pinned): payloads packed, then the per-datagram arrays */
    const uint64_t o_pay = 0, o_poff = a16(pay), o_len = o_poff + a16(4ull * nsel),
                   o_sock = o_len + a16(2ull * nsel), o_ip = o_sock + a16(4ull * nsel),
                   o_port = o_ip + a16(4ull * nsel), o_foff = o_port + a16(2ull * nsel),
                   tot = o_foff + a16(4ull * nsel);
    if (h_grow_pinned(&g_udpdk.tx_h, &g_udpdk.tx_h_cap, tot) ||
        h_grow_dev(&g_udpdk.tx_d, &g_udpdk.tx_d_cap, tot + 64) ||
        h_grow_dev(&g_udpdk.tx_fr_d, &g_udpdk.tx_fr_d_cap, bytes + 64))
        goto out;
    uint8_t *h = g_udpdk.tx_h;
    uint32_t *poff = (uint32_t *)(h + o_poff), *sock = (uint32_t *)(h + o_sock);
    uint32_t *ip = (uint32_t *)(h + o_ip), *foff = (uint32_t *)(h + o_foff);
    uint16_t *len = (uint16_t *)(h + o_len), *port = (uint16_t *)(h + o_port);
    memset(taken, 0, sizeof(taken));
    uint64_t pp = 0;
    for (uint32_t i = 0; i < nsel; i++) {
        const int s = g_udpdk.tx_sel[i].s;
        const struct h_txq *q = &g_udpdk.slots[s].tx;
        const struct h_txd *t = &q->e[(q->head + taken[s]++) % UDPDK_RX_RING_SIZE];
        memcpy(h + o_pay + pp, g_udpdk.txp + t->pay, t->len);
        poff[i] = (uint32_t)pp;
        len[i] = (uint16_t)t->len;
        sock[i] = (uint32_t)s;
        ip[i] = t->dst_ip;
        port[i] = (uint16_t)t->dst_port;
        foff[i] = (uint32_t)g_udpdk.tx_sel[i].foff;
        pp += t->len;
    }
    /* 3. GPU: one H2D, the build, one D2H */
    uint8_t *d = g_udpdk.tx_d;
    udpdk_tx_config_t cfg;
    memcpy(cfg.src_mac, g_udpdk.src_mac, 6);
    memcpy(cfg.dst_mac, g_udpdk.dst_mac, 6);
    cfg.src_ip = g_udpdk.src_ip;
    udpdk_tx_batch_t b = {d + o_pay, pay, (const uint32_t *)(d + o_poff), (const uint16_t *)(d + o_len),
                          (const int32_t *)(d + o_sock), (const uint32_t *)(d + o_ip),
                          (const uint16_t *)(d + o_port), nsel};
    udpdk_tx_out_t o = {g_udpdk.tx_fr_d, bytes + 64, (const uint32_t *)(d + o_foff)};
    if ((rc = udpdk_gpu_h2d(g, d, h, tot)) || (rc = udpdk_gpu_tx_build_mtu(g, &cfg, &b, &o, mtu)) ||
        (rc = udpdk_gpu_d2h(g, out, g_udpdk.tx_fr_d, bytes)) || (rc = udpdk_gpu_sync(g))) {
        errno = -rc;
        goto out;
    }
    /* 4. frame table, dequeue, payload store compaction */
    uint32_t k = 0;
    for (uint32_t i = 0; i < nsel; i++) {
        const uint32_t nf = g_udpdk.tx_sel[i].nf;
        const uint64_t span = udpdk_gpu_tx_span(len[i], mtu, NULL);
        for (uint32_t f = 0; f < nf; f++) {
            out_off[k] = foff[i] + f * (mtu + 14u);
            out_len[k] = (uint16_t)(f + 1 < nf ? mtu + 14u : span - (uint64_t)(nf - 1) * (mtu + 14u));
            k++;
        }
    }
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) g_udpdk.slots[s].tx.head += taken[s];
    g_udpdk.tx_queued -= nsel;
    if (!g_udpdk.tx_queued) {
        g_udpdk.txp_bytes = 0;
    } else if (g_udpdk.txp_bytes > (1u << 24)) {
        /* compact: the remaining datagrams' payloads to the front, in store order */
        uint64_t w = 0, lo = UINT64_MAX;
        for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {
            const struct h_txq *q = &g_udpdk.slots[s].tx;
            for (uint32_t j = q->head; q->e && j != q->tail; j++)
                if (q->e[j % UDPDK_RX_RING_SIZE].pay < lo) lo = q->e[j % UDPDK_RX_RING_SIZE].pay;
        }
        if (lo != UINT64_MAX && lo > 0) {
            w = g_udpdk.txp_bytes - lo;
            memmove(g_udpdk.txp, g_udpdk.txp + lo, w);
            for (int s = 0; s < UDPDK_MAX_SOCKETS; s++) {
                struct h_txq *q = &g_udpdk.slots[s].tx;
                for (uint32_t j = q->head; q->e && j != q->tail; j++) q->e[j % UDPDK_RX_RING_SIZE].pay -= lo;
            }
            g_udpdk.txp_bytes = w;
        }
    }
    *n_out = k;
    ret = 0;
out:
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    return ret;
}
