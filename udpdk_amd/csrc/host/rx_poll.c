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

/* Diagnostic build (-DUDPDK_POLL_PROFILE): wall time per phase of udpdk_poll_rx, summed over the
 * calls and printed to stderr by udpdk_poll_profile_dump (called from udpdk_cleanup). */
#ifdef UDPDK_POLL_PROFILE
#include <stdio.h>
static double g_prof[8];
static const char *g_prof_name[8] = {"snapshot", "gpu_rx_host", "frag_pass", "admission", "gather",
                                     "gather_sync", "publish", "calls"};
static double h_prof_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}
#define PROF_T(v) const double v = h_prof_now()
#define PROF_ADD(k, a, b) (g_prof[k] += (b) - (a))
__attribute__((visibility("hidden"))) void udpdk_poll_profile_dump(void)
{
    if (!g_prof[7]) return;
    fprintf(stderr, "{\"udpdk_poll_profile_ms_per_call\": {");
    for (int k = 0; k < 7; k++) fprintf(stderr, "%s\"%s\": %.3f", k ? ", " : "", g_prof_name[k], g_prof[k] / g_prof[7]);
    fprintf(stderr, "}, \"calls\": %.0f}\n", g_prof[7]);
}
#else
#define PROF_T(v) do {} while (0)
#define PROF_ADD(k, a, b) do {} while (0)
void udpdk_poll_profile_dump(void) {}
#endif

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
                     (void **)&g_udpdk.acc_do, (void **)&g_udpdk.acc_fo, (void **)&g_udpdk.acc_sock};
    uint64_t *hcap[] = {&g_udpdk.rx_meta_cap, &g_udpdk.rx_loff_cap, &g_udpdk.rx_lpkt_cap,
                        &g_udpdk.fr_loff_cap, &g_udpdk.fr_lpkt_cap, &g_udpdk.fr_org_cap,
                        &g_udpdk.fr_len_cap, &g_udpdk.acc_d_cap, &g_udpdk.acc_f_cap,
                        &g_udpdk.acc_do_cap, &g_udpdk.acc_fo_cap, &g_udpdk.acc_sock_cap};
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
static int h_frag_pass(const udpdk_rx_batch_t *staged, const uint32_t *meta_dev, uint64_t nfrag,
                       uint32_t lanes, uint32_t maxfan, udpdk_rx_batch_t *rb, uint32_t *nd)
{
    *nd = 0;
    if (!nfrag) return 0;                   /* the batch's FRAG verdict count (RX counters) */
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
 * slab of packed slots (entry k at offs[k], offs[count] bytes in all, each slot its frame's
 * payload room rounded up to 16): one gather launch, one D2H of each output, and only the
 * bytes that exist cross PCIe (a slot per longest datagram moved 4.6x the IMIX payload). */
static int h_gather(const udpdk_rx_batch_t *b, const uint32_t *acc, const uint32_t *offs, uint32_t count,
                    struct h_arena **out)
{
    *out = NULL;
    if (!count) return 0;
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    const uint64_t bytes = offs[count] ? offs[count] : 16u;
    struct h_arena *a = h_arena_get(count, bytes);
    if (!a) { errno = ENOMEM; return -1; }
    int rc;
    if (h_grow_dev(&g_udpdk.dv_acc, &g_udpdk.dv_acc_cap, 8ull * count + 4) ||
        h_grow_dev(&g_udpdk.dv_pay, &g_udpdk.dv_pay_cap, bytes) ||
        h_grow_dev(&g_udpdk.dv_len, &g_udpdk.dv_len_cap, 4ull * count) ||
        h_grow_dev(&g_udpdk.dv_sip, &g_udpdk.dv_sip_cap, 4ull * count) ||
        h_grow_dev(&g_udpdk.dv_spt, &g_udpdk.dv_spt_cap, 2ull * count)) {
        h_arena_put(a);
        return -1;
    }
    udpdk_rx_gather_t go = {g_udpdk.dv_pay, 16u, g_udpdk.dv_len, g_udpdk.dv_sip, g_udpdk.dv_spt};
    uint32_t *dacc = g_udpdk.dv_acc, *doff = dacc + count;
    if ((rc = udpdk_gpu_h2d(g, dacc, acc, 4ull * count)) ||
        (rc = udpdk_gpu_h2d(g, doff, offs, 4ull * count + 4)) ||
        (rc = udpdk_gpu_rx_gather_packed(g, b, dacc, 0, count, doff, &go)) ||
        (rc = udpdk_gpu_d2h(g, a->payload, g_udpdk.dv_pay, bytes)) ||
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

/* Per-socket admission (two passes over the same sockets, split over the pool's parts): pass 1
 * records the ring room each socket had and what it admits (entries and slab bytes, direct and
 * reassembled); pass 2, after a prefix over the sockets, writes the accepted lists at those
 * bases. Both passes make the same decisions: they read the room once, in pass 1. */
static uint32_t s_room[UDPDK_MAX_SOCKETS], s_nd[UDPDK_MAX_SOCKETS], s_nf[UDPDK_MAX_SOCKETS];
static uint64_t s_bd[UDPDK_MAX_SOCKETS], s_bf[UDPDK_MAX_SOCKETS];
static uint32_t s_kd[UDPDK_MAX_SOCKETS], s_kf[UDPDK_MAX_SOCKETS];
static uint64_t s_od[UDPDK_MAX_SOCKETS], s_of[UDPDK_MAX_SOCKETS];

struct h_adm {
    const uint32_t *loff, *lpkt, *floff, *flpkt, *forg;
    const uint16_t *length;
    uint32_t lanes;
    int fill;
    uint32_t sb[H_MAX_WORKERS + 3];   /* part p takes sockets [sb[p], sb[p + 1]) */
};

/* socket ranges of about equal delivery counts */
static void h_adm_split(struct h_adm *A, uint32_t parts)
{
    const uint32_t L = A->lanes, D = A->loff[L] + (A->floff ? A->floff[L] : 0u);
    uint32_t s = 0;
    A->sb[0] = 0;
    for (uint32_t p = 1; p < parts; p++) {
        const uint64_t want = (uint64_t)D * p / parts;
        while (s < L && (uint64_t)A->loff[s] + (A->floff ? A->floff[s] : 0u) < want) s++;
        A->sb[p] = s;
    }
    A->sb[parts] = L;
}

static void h_adm_socket(const struct h_adm *A, uint32_t s)
{
    const uint32_t *lpkt = A->lpkt, *flpkt = A->flpkt, *forg = A->forg;
    const uint32_t a0 = A->loff[s], a1 = A->loff[s + 1];
    const uint32_t b0 = A->floff ? A->floff[s] : 0u, b1 = A->floff ? A->floff[s + 1] : 0u;
    if (!A->fill) {
        s_nd[s] = s_nf[s] = 0;
        s_bd[s] = s_bf[s] = 0;
        if ((a0 == a1 && b0 == b1) || !g_udpdk.slots[s].used) return;   /* closed: dropped */
        s_room[s] = h_ring_free(&g_udpdk.slots[s].rx);
    } else if (!s_nd[s] && !s_nf[s]) {
        return;
    }
    uint32_t room = s_room[s], nd = 0, nf = 0;
    uint64_t bd = 0, bf = 0;
    uint32_t kd = s_kd[s], kf = s_kf[s], ka = s_kd[s] + s_kf[s];
    uint64_t od = s_od[s], of = s_of[s];
    uint32_t e = a0, q = b0;
    while (e < a1 || q < b1) {
        /* the burst of the next delivery in arrival order, and its deliveries */
        const uint32_t ie = e < a1 ? lpkt[e] : UINT32_MAX, iq = q < b1 ? forg[flpkt[q]] : UINT32_MAX;
        const uint32_t burst = (ie < iq ? ie : iq) / H_BURST_SIZE;
        uint32_t ce = e, cq = q;
        while (ce < a1 && lpkt[ce] / H_BURST_SIZE == burst) ce++;
        while (cq < b1 && forg[flpkt[cq]] / H_BURST_SIZE == burst) cq++;
        const uint32_t k = (ce - e) + (cq - q);
        if (k > room) {                            /* ring full: the burst is dropped */
            e = ce;
            q = cq;
            continue;
        }
        room -= k;
        while (e < ce || q < cq) {
            if (q >= cq || (e < ce && lpkt[e] < forg[flpkt[q]])) {
                const uint32_t fi = lpkt[e++];
                const uint32_t pl = A->length[fi] > 42u ? A->length[fi] - 42u : 0u;
                const uint32_t sz = (pl + 15u) & ~15u;
                if (A->fill) {
                    g_udpdk.acc_do[kd] = (uint32_t)od;
                    g_udpdk.acc_d[kd++] = fi;
                    g_udpdk.acc_sock[ka++] = s;
                    od += sz;
                } else {
                    nd++;
                    bd += sz;
                }
            } else {
                const uint32_t di = flpkt[q++];
                const uint32_t pl = g_udpdk.fr_len[di] > 42u ? g_udpdk.fr_len[di] - 42u : 0u;
                const uint32_t sz = (pl + 15u) & ~15u;
                if (A->fill) {
                    g_udpdk.acc_fo[kf] = (uint32_t)of;
                    g_udpdk.acc_f[kf++] = di;
                    g_udpdk.acc_sock[ka++] = s | 0x80000000u;
                    of += sz;
                } else {
                    nf++;
                    bf += sz;
                }
            }
        }
    }
    if (!A->fill) {
        s_nd[s] = nd;
        s_nf[s] = nf;
        s_bd[s] = bd;
        s_bf[s] = bf;
    }
}

static void h_adm_job(void *ctx, uint32_t part, uint32_t parts)
{
    const struct h_adm *A = ctx;
    (void)parts;
    for (uint32_t s = A->sb[part]; s < A->sb[part + 1]; s++) h_adm_socket(A, s);
}

/* Ring publication of the admitted entries: socket s's are acc_sock[s_kd + s_kf ...] in arrival
 * order, its direct and reassembled ones consumed from acc_d / acc_f at s_kd[s] / s_kf[s]. */
struct h_pub {
    const struct h_adm *A;
    struct h_arena *ad, *af;
};

static void h_pub_job(void *ctx, uint32_t part, uint32_t parts)
{
    const struct h_pub *P = ctx;
    (void)parts;
    struct h_dgram buf[H_BURST_SIZE];
    for (uint32_t s = P->A->sb[part]; s < P->A->sb[part + 1]; s++) {
        const uint32_t n = s_nd[s] + s_nf[s];
        uint32_t kd = s_kd[s], kf = s_kf[s], k = s_kd[s] + s_kf[s];
        const uint32_t kend = k + n;
        while (k < kend) {
            uint32_t nb = 0;
            while (k < kend && nb < H_BURST_SIZE) {
                struct h_dgram *d = &buf[nb++];
                if (g_udpdk.acc_sock[k] >> 31) {
                    struct h_arena *af = P->af;
                    d->arena = af;
                    d->data = af->payload + g_udpdk.acc_fo[kf];
                    d->len = af->len[kf];
                    d->src_ip = af->src_ip[kf];
                    d->src_port = af->src_port[kf];
                    kf++;
                } else {
                    struct h_arena *ad = P->ad;
                    d->arena = ad;
                    d->data = ad->payload + g_udpdk.acc_do[kd];
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
    PROF_T(p0);
    if (h_snapshot_refresh()) goto out;
    PROF_T(p1);
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
    PROF_T(p2);
    udpdk_rx_batch_t staged;
    const uint32_t *meta_dev = NULL;
    if ((rc = udpdk_gpu_rx_host_batch(g, &staged, &meta_dev))) { errno = -rc; goto out; }
    udpdk_rx_batch_t rb;
    uint32_t nd = 0;
    if (h_frag_pass(&staged, meta_dev, st.counters[UDPDK_V_FRAG], lanes, maxfan, &rb, &nd)) goto out;
    PROF_T(p3);
    const uint32_t *floff = nd ? g_udpdk.fr_loff : NULL, *flpkt = g_udpdk.fr_lpkt, *forg = g_udpdk.fr_org;

    /* admission: per socket, arrival-ordered merge, one all-or-nothing decision per burst; the
     * sockets split over the pool's parts, counted first, then filled at their prefix bases */
    const uint32_t D = loff[lanes], DF = nd ? floff[lanes] : 0u;
    if (h_grow_host((void **)&g_udpdk.acc_d, &g_udpdk.acc_d_cap, 4ull * D + 4) ||
        h_grow_host((void **)&g_udpdk.acc_f, &g_udpdk.acc_f_cap, 4ull * DF + 4) ||
        h_grow_host((void **)&g_udpdk.acc_do, &g_udpdk.acc_do_cap, 4ull * D + 8) ||
        h_grow_host((void **)&g_udpdk.acc_fo, &g_udpdk.acc_fo_cap, 4ull * DF + 8) ||
        h_grow_host((void **)&g_udpdk.acc_sock, &g_udpdk.acc_sock_cap, 4ull * (D + DF) + 4))
        goto out;
    struct h_adm A = {loff, lpkt, floff, flpkt, forg, length, lanes < UDPDK_MAX_SOCKETS ? lanes : UDPDK_MAX_SOCKETS, 0, {0}};
    h_adm_split(&A, h_pool_parts());
    h_pool_run(h_adm_job, &A);                       /* pass 1: what each socket admits */
    uint32_t nad = 0, naf = 0;
    uint64_t offd = 0, offf = 0;                    /* packed slot offsets (payload room / 16) */
    for (uint32_t s = 0; s < A.lanes; s++) {
        s_kd[s] = nad;
        s_kf[s] = naf;
        s_od[s] = offd;
        s_of[s] = offf;
        nad += s_nd[s];
        naf += s_nf[s];
        offd += s_bd[s];
        offf += s_bf[s];
    }
    if (offd > 0xFFFFFFF0ull || offf > 0xFFFFFFF0ull) { errno = ENOBUFS; goto out; }
    A.fill = 1;
    h_pool_run(h_adm_job, &A);                       /* pass 2: the accepted lists */
    /* payloads of the admitted datagrams, gathered on the GPU into pinned slabs */
    PROF_T(p4);
    g_udpdk.acc_do[nad] = (uint32_t)offd;
    g_udpdk.acc_fo[naf] = (uint32_t)offf;
    if (h_gather(&staged, g_udpdk.acc_d, g_udpdk.acc_do, nad, &ad)) goto out;
    if (naf && h_gather(&rb, g_udpdk.acc_f, g_udpdk.acc_fo, naf, &af)) goto out;
    PROF_T(p5);
    if ((rc = udpdk_gpu_sync(g))) { errno = -rc; goto out; }
    PROF_T(p6);
    if (ad) atomic_store_explicit(&ad->refs, nad, memory_order_relaxed);
    if (af) atomic_store_explicit(&af->refs, naf, memory_order_relaxed);
    /* publish: each socket's entries go to its ring in bulk enqueues, sockets over the pool */
    {
        struct h_pub P = {&A, ad, af};
        h_pool_run(h_pub_job, &P);
    }
    ad = af = NULL;
    if (stats_out) *stats_out = st;
    ret = 0;
#ifdef UDPDK_POLL_PROFILE
    {   /* the first call (allocations, snapshot upload) is left out */
        static int first = 1;
        PROF_T(p7);
        if (!first) {
            PROF_ADD(0, p0, p1); PROF_ADD(1, p1, p2); PROF_ADD(2, p2, p3); PROF_ADD(3, p3, p4);
            PROF_ADD(4, p4, p5); PROF_ADD(5, p5, p6); PROF_ADD(6, p6, p7);
            g_prof[7] += 1;
        }
        first = 0;
    }
#endif
out:
    if (ad) h_arena_put(ad);
    if (af) h_arena_put(af);
    pthread_mutex_unlock(&g_udpdk.lock);
    return ret;
}
