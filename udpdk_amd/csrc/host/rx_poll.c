/*
 * rx_poll.c — udpdk_poll_rx: the poller's RX half (udpdk_poller.c:516-545) over a host batch.
 *
 *   1. the frames go to the GPU once (udpdk_gpu_rx_host: pinned staging, H2D, classify + demux +
 *      lanes, D2H of verdict words and lanes); the staged batch stays resident;
 *   2. FRAG frames (poller.c:338-361) are reassembled on the device from that staged batch and
 *      the completed datagrams demultiplexed by a second udpdk_gpu_rx;
 *   3. per socket, direct and reassembled deliveries are merged in arrival order (a reassembled
 *      datagram at the index of the fragment that completed it) and admitted to the socket's
 *      ring per burst of BURST_SIZE frames, all-or-nothing like flush_rx_queue (:274-292);
 *   4. the admitted datagrams' payloads are gathered on the GPU (udpdk_gpu_rx_gather, the batch
 *      recvfrom) into pinned slabs with one D2H per source batch;
 *   5. the ring entries are published; recvfrom copies from the slab and releases it.
 * The bind snapshot is uploaded only when the bind table's version has moved since the last
 * upload (no per-call walk of the 65,536 ports).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "host_state.h"

int h_grow_dev(void **p, uint64_t *cap, uint64_t need)
{
    if (*p && *cap >= need) return 0;
    if (*p) udpdk_gpu_free(g_udpdk.gpu, *p);
    *p = NULL;
    *cap = 0;
    uint64_t nc = need < 4096 ? 4096 : need + need / 4;
    const int rc = udpdk_gpu_alloc(g_udpdk.gpu, nc, p);
    if (rc) { errno = -rc; return -1; }
    *cap = nc;
    return 0;
}

int h_grow_host(void **p, uint64_t *cap, uint64_t need)
{
    if (*p && *cap >= need) return 0;
    uint64_t nc = need < 4096 ? 4096 : need + need / 4;
    void *q = realloc(*p, nc);
    if (!q) { errno = ENOMEM; return -1; }
    *p = q;
    *cap = nc;
    return 0;
}

void h_rx_buffers_free(void)
{
    void **host[] = {(void **)&g_udpdk.rx_meta, (void **)&g_udpdk.rx_loff, (void **)&g_udpdk.rx_lpkt,
                     (void **)&g_udpdk.fr_loff, (void **)&g_udpdk.fr_lpkt, (void **)&g_udpdk.fr_org,
                     (void **)&g_udpdk.fr_len, (void **)&g_udpdk.acc_d, (void **)&g_udpdk.acc_f,
                     (void **)&g_udpdk.acc_sock};
    uint64_t *hcap[] = {&g_udpdk.rx_meta_cap, &g_udpdk.rx_loff_cap, &g_udpdk.rx_lpkt_cap,
                        &g_udpdk.fr_loff_cap, &g_udpdk.fr_lpkt_cap, &g_udpdk.fr_org_cap,
                        &g_udpdk.fr_len_cap, &g_udpdk.acc_d_cap, &g_udpdk.acc_f_cap,
                        &g_udpdk.acc_sock_cap};
    for (unsigned k = 0; k < sizeof(host) / sizeof(host[0]); k++) {
        free(*host[k]);
        *host[k] = NULL;
        *hcap[k] = 0;
    }
    void **dev[] = {&g_udpdk.dv_acc, &g_udpdk.dv_pay, &g_udpdk.dv_len, &g_udpdk.dv_sip,
                    &g_udpdk.dv_spt, &g_udpdk.dv_meta2, &g_udpdk.dv_loff2, &g_udpdk.dv_lpkt2};
    uint64_t *dcap[] = {&g_udpdk.dv_acc_cap, &g_udpdk.dv_pay_cap, &g_udpdk.dv_len_cap,
                        &g_udpdk.dv_sip_cap, &g_udpdk.dv_spt_cap, &g_udpdk.dv_meta2_cap,
                        &g_udpdk.dv_loff2_cap, &g_udpdk.dv_lpkt2_cap};
    for (unsigned k = 0; k < sizeof(dev) / sizeof(dev[0]); k++) {
        if (*dev[k] && g_udpdk.gpu) udpdk_gpu_free(g_udpdk.gpu, *dev[k]);
        *dev[k] = NULL;
        *dcap[k] = 0;
    }
}

/* Upload the bind snapshot when the table changed since the last upload; keep its lane count
 * and largest per-port fan-out (the lane capacity a batch can need) with it. g_udpdk.lock held. */
int h_snapshot_refresh(void)
{
    if (g_udpdk.snap_version == g_udpdk.version) return 0;
    udpdk_bind_snapshot_t snap;
    if (udpdk_btable_snapshot(&snap, 0)) return -1;
    const int rc = udpdk_gpu_bind_snapshot_upload(g_udpdk.gpu, &snap);
    if (rc) { errno = -rc; return -1; }
    uint32_t maxfan = 1;
    for (uint32_t p = 0; p < 65536; p++)
        if (snap.port_count[p] > maxfan) maxfan = snap.port_count[p];
    g_udpdk.snap_lanes = snap.n_lanes;
    g_udpdk.snap_maxfan = maxfan;
    g_udpdk.snap_version = snap.version;
    return 0;
}

static uint64_t h_now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u;
}

/* The FRAG frames of the staged batch through the device reassembly table, then the completed
 * datagrams through the demux. Out: *rb = the reassembled batch (device, valid until the next
 * reassembly call), fr_loff[lanes + 1] / fr_lpkt[] its lanes (host), fr_org[] each datagram's
 * completing fragment index, fr_len[] its frame length. *nf = 0 when nothing completed. */
static int h_frag_pass(const udpdk_rx_batch_t *staged, const uint32_t *meta_dev, const uint32_t *meta,
                       uint32_t n, uint32_t lanes, uint32_t maxfan, udpdk_rx_batch_t *rb, uint32_t *nd)
{
    *nd = 0;
    uint32_t nfrag = 0;
    for (uint32_t i = 0; i < n; i++) nfrag += (meta[i] & 0xFu) == UDPDK_V_FRAG;
    if (!nfrag) return 0;
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    int rc;
    if (!g_udpdk.frag_ready) {
        udpdk_frag_table_cfg_t fc = {g_udpdk.frag_buckets, g_udpdk.frag_entries, g_udpdk.frag_ttl_ms,
                                     g_udpdk.frag_max_dgram};
        if ((rc = udpdk_gpu_frag_table_create(g, &fc))) { errno = -rc; return -1; }
        g_udpdk.frag_ready = 1;
    }
    udpdk_reasm_out_t ro;
    if ((rc = udpdk_gpu_rx_reassemble(g, staged, meta_dev, h_now_ms(), &ro))) { errno = -rc; return -1; }
    const uint32_t C = ro.batch.n;
    if (!C) return 0;
    const uint64_t cap64 = (uint64_t)C * maxfan;
    const uint32_t cap = cap64 > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap64;
    if (h_grow_dev(&g_udpdk.dv_meta2, &g_udpdk.dv_meta2_cap, 4ull * C) ||
        h_grow_dev(&g_udpdk.dv_loff2, &g_udpdk.dv_loff2_cap, 4ull * (lanes + 1)) ||
        h_grow_dev(&g_udpdk.dv_lpkt2, &g_udpdk.dv_lpkt2_cap, 4ull * cap) ||
        h_grow_host((void **)&g_udpdk.fr_loff, &g_udpdk.fr_loff_cap, 4ull * (lanes + 1)) ||
        h_grow_host((void **)&g_udpdk.fr_org, &g_udpdk.fr_org_cap, 4ull * C) ||
        h_grow_host((void **)&g_udpdk.fr_len, &g_udpdk.fr_len_cap, 2ull * C))
        return -1;
    udpdk_rx_out_t o2 = {g_udpdk.dv_meta2, g_udpdk.dv_loff2, g_udpdk.dv_lpkt2, cap};
    udpdk_rx_stats_t st2;
    if ((rc = udpdk_gpu_rx(g, &ro.batch, &o2)) || (rc = udpdk_gpu_rx_stats(g, &st2))) { errno = -rc; return -1; }
    const uint32_t D = st2.deliveries;
    if (h_grow_host((void **)&g_udpdk.fr_lpkt, &g_udpdk.fr_lpkt_cap, 4ull * D + 4)) return -1;
    if ((rc = udpdk_gpu_d2h(g, g_udpdk.fr_loff, g_udpdk.dv_loff2, 4ull * (lanes + 1))) ||
        (rc = udpdk_gpu_d2h(g, g_udpdk.fr_lpkt, g_udpdk.dv_lpkt2, 4ull * D)) ||
        (rc = udpdk_gpu_d2h(g, g_udpdk.fr_org, ro.origin_dev, 4ull * C)) ||
        (rc = udpdk_gpu_d2h(g, g_udpdk.fr_len, ro.batch.length_dev, 2ull * C)) ||
        (rc = udpdk_gpu_sync(g))) {
        errno = -rc;
        return -1;
    }
    *rb = ro.batch;
    *nd = C;
    return 0;
}

/* Gather the payloads of the count entries listed in acc (frame indices of batch b) into a new
 * slab: one gather launch, one D2H of each output. slot_bytes covers the longest. */
static int h_gather(const udpdk_rx_batch_t *b, const uint32_t *acc, uint32_t count, uint32_t maxlen,
                    struct h_arena **out)
{
    *out = NULL;
    if (!count) return 0;
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    const uint32_t slot = ((maxlen ? maxlen : 1) + 15u) & ~15u;
    struct h_arena *a = h_arena_get(count, slot);
    if (!a) { errno = ENOMEM; return -1; }
    int rc;
    if (h_grow_dev(&g_udpdk.dv_acc, &g_udpdk.dv_acc_cap, 4ull * count) ||
        h_grow_dev(&g_udpdk.dv_pay, &g_udpdk.dv_pay_cap, (uint64_t)count * slot) ||
        h_grow_dev(&g_udpdk.dv_len, &g_udpdk.dv_len_cap, 4ull * count) ||
        h_grow_dev(&g_udpdk.dv_sip, &g_udpdk.dv_sip_cap, 4ull * count) ||
        h_grow_dev(&g_udpdk.dv_spt, &g_udpdk.dv_spt_cap, 2ull * count)) {
        h_arena_put(a);
        return -1;
    }
    udpdk_rx_gather_t go = {g_udpdk.dv_pay, slot, g_udpdk.dv_len, g_udpdk.dv_sip, g_udpdk.dv_spt};
    if ((rc = udpdk_gpu_h2d(g, g_udpdk.dv_acc, acc, 4ull * count)) ||
        (rc = udpdk_gpu_rx_gather(g, b, g_udpdk.dv_acc, 0, count, &go)) ||
        (rc = udpdk_gpu_d2h(g, a->payload, g_udpdk.dv_pay, (uint64_t)count * slot)) ||
        (rc = udpdk_gpu_d2h(g, a->len, g_udpdk.dv_len, 4ull * count)) ||
        (rc = udpdk_gpu_d2h(g, a->src_ip, g_udpdk.dv_sip, 4ull * count)) ||
        (rc = udpdk_gpu_d2h(g, a->src_port, g_udpdk.dv_spt, 2ull * count))) {
        h_arena_put(a);
        errno = -rc;
        return -1;
    }
    *out = a;
    return 0;
}

int udpdk_poll_rx(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                  const uint16_t *length, const uint32_t *ptype, uint32_t n,
                  udpdk_rx_stats_t *stats_out)
{
    if (!g_udpdk.gpu) { errno = ENODEV; return -1; }
    if (n && (!frames || !offset || !length)) { errno = EINVAL; return -1; }
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    pthread_mutex_lock(&g_udpdk.lock);
    int ret = -1, rc;
    struct h_arena *ad = NULL, *af = NULL;
    if (h_snapshot_refresh()) goto out;
    const uint32_t lanes = g_udpdk.snap_lanes, maxfan = g_udpdk.snap_maxfan;
    const uint64_t cap64 = (uint64_t)n * maxfan;
    const uint32_t cap = cap64 > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap64;
    if (h_grow_host((void **)&g_udpdk.rx_meta, &g_udpdk.rx_meta_cap, 4ull * n + 4) ||
        h_grow_host((void **)&g_udpdk.rx_loff, &g_udpdk.rx_loff_cap, 4ull * (lanes + 1)) ||
        h_grow_host((void **)&g_udpdk.rx_lpkt, &g_udpdk.rx_lpkt_cap, 4ull * cap + 4))
        goto out;
    uint32_t *meta = g_udpdk.rx_meta, *loff = g_udpdk.rx_loff, *lpkt = g_udpdk.rx_lpkt;
    udpdk_rx_stats_t st;
    if ((rc = udpdk_gpu_rx_host(g, frames, frames_bytes, offset, length, ptype, n, meta, loff, lpkt,
                                cap, &st))) { errno = -rc; goto out; }
    udpdk_rx_batch_t staged;
    const uint32_t *meta_dev = NULL;
    if ((rc = udpdk_gpu_rx_host_batch(g, &staged, &meta_dev))) { errno = -rc; goto out; }
    udpdk_rx_batch_t rb;
    uint32_t nd = 0;
    if (h_frag_pass(&staged, meta_dev, meta, n, lanes, maxfan, &rb, &nd)) goto out;
    const uint32_t *floff = nd ? g_udpdk.fr_loff : NULL, *flpkt = g_udpdk.fr_lpkt, *forg = g_udpdk.fr_org;

    /* admission: per socket, arrival-ordered merge, one all-or-nothing decision per burst */
    const uint32_t D = loff[lanes], DF = nd ? floff[lanes] : 0u;
    if (h_grow_host((void **)&g_udpdk.acc_d, &g_udpdk.acc_d_cap, 4ull * D + 4) ||
        h_grow_host((void **)&g_udpdk.acc_f, &g_udpdk.acc_f_cap, 4ull * DF + 4) ||
        h_grow_host((void **)&g_udpdk.acc_sock, &g_udpdk.acc_sock_cap, 4ull * (D + DF) + 4))
        goto out;
    uint32_t nad = 0, naf = 0, nacc = 0, maxd = 0, maxf = 0;
    for (uint32_t s = 0; s < lanes && s < UDPDK_MAX_SOCKETS; s++) {
        const uint32_t a0 = loff[s], a1 = loff[s + 1];
        const uint32_t b0 = nd ? floff[s] : 0u, b1 = nd ? floff[s + 1] : 0u;
        if (a0 == a1 && b0 == b1) continue;
        if (!g_udpdk.slots[s].used) continue;          /* closed since the snapshot: dropped */
        uint32_t room = h_ring_free(&g_udpdk.slots[s].rx);
        uint32_t e = a0, q = b0;
        while (e < a1 || q < b1) {
            /* the burst of the next delivery in arrival order, and its deliveries */
            const uint32_t ie = e < a1 ? lpkt[e] : UINT32_MAX, iq = q < b1 ? forg[flpkt[q]] : UINT32_MAX;
            const uint32_t burst = (ie < iq ? ie : iq) / H_BURST_SIZE;
            uint32_t ce = e, cq = q;
            while (ce < a1 && lpkt[ce] / H_BURST_SIZE == burst) ce++;
            while (cq < b1 && forg[flpkt[cq]] / H_BURST_SIZE == burst) cq++;
            const uint32_t k = (ce - e) + (cq - q);
            if (k <= room) {
                room -= k;
                while (e < ce || q < cq) {
                    if (q >= cq || (e < ce && lpkt[e] < forg[flpkt[q]])) {
                        const uint32_t fi = lpkt[e++];
                        const uint32_t pl = length[fi] > 42u ? length[fi] - 42u : 0u;
                        if (pl > maxd) maxd = pl;
                        g_udpdk.acc_d[nad++] = fi;
                        g_udpdk.acc_sock[nacc++] = s;
                    } else {
                        const uint32_t di = flpkt[q++];
                        const uint32_t pl = g_udpdk.fr_len[di] > 42u ? g_udpdk.fr_len[di] - 42u : 0u;
                        if (pl > maxf) maxf = pl;
                        g_udpdk.acc_f[naf++] = di;
                        g_udpdk.acc_sock[nacc++] = s | 0x80000000u;
                    }
                }
            } else {
                e = ce;                                /* ring full: the burst is dropped */
                q = cq;
            }
        }
    }
    /* payloads of the admitted datagrams, gathered on the GPU into pinned slabs */
    if (h_gather(&staged, g_udpdk.acc_d, nad, maxd, &ad)) goto out;
    if (naf && h_gather(&rb, g_udpdk.acc_f, naf, maxf, &af)) goto out;
    if ((rc = udpdk_gpu_sync(g))) { errno = -rc; goto out; }
    if (ad) atomic_store_explicit(&ad->refs, nad, memory_order_relaxed);
    if (af) atomic_store_explicit(&af->refs, naf, memory_order_relaxed);
    /* publish: consecutive entries of one socket go to its ring in one bulk enqueue */
    {
        struct h_dgram buf[H_BURST_SIZE];
        uint32_t kd = 0, kf = 0, k = 0;
        while (k < nacc) {
            const uint32_t s = g_udpdk.acc_sock[k] & 0x7FFFFFFFu;
            uint32_t nb = 0;
            while (k < nacc && (g_udpdk.acc_sock[k] & 0x7FFFFFFFu) == s && nb < H_BURST_SIZE) {
                struct h_dgram *d = &buf[nb++];
                if (g_udpdk.acc_sock[k] >> 31) {
                    d->arena = af;
                    d->data = af->payload + (uint64_t)kf * af->slot_bytes;
                    d->len = af->len[kf];
                    d->src_ip = af->src_ip[kf];
                    d->src_port = af->src_port[kf];
                    kf++;
                } else {
                    d->arena = ad;
                    d->data = ad->payload + (uint64_t)kd * ad->slot_bytes;
                    d->len = ad->len[kd];
                    d->src_ip = ad->src_ip[kd];
                    d->src_port = ad->src_port[kd];
                    kd++;
                }
                k++;
            }
            if (h_ring_push_bulk(&g_udpdk.slots[s].rx, buf, nb)) {   /* admitted: cannot fail */
                for (uint32_t z = 0; z < nb; z++) h_arena_release(buf[z].arena, 1);
            }
        }
    }
    ad = af = NULL;
    if (stats_out) *stats_out = st;
    ret = 0;
out:
    if (ad) h_arena_put(ad);
    if (af) h_arena_put(af);
    pthread_mutex_unlock(&g_udpdk.lock);
    return ret;
}
