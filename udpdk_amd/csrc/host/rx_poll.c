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
 *
 * Multi-device ([gpu] devices = 0-7): step 1 runs per contiguous
 * shard of the batch on its own context (one pool thread per shard: H2D, kernels, D2H on that
 * device), and the shards' per-socket lanes are concatenated in shard order, which is global
 * arrival order because each shard is contiguous and its lanes are stable. The FRAG frames of
 * all shards go, in arrival order, through the one reassembly table of the main context (a flow's
 * fragments may straddle shards). Step 4 gathers each shard's admitted payloads on its own device
 * into a slab of its own. Admission (3) and publication (5) are the single-device code on the
 * merged lanes, so the rings equal a single-context poll's.
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
/* the pipelined form's phases, summed over its chunks */
static double g_cprof[8];
static const char *g_cprof_name[8] = {"rx_issue", "rx_wait", "gather_wait", "publish", "frag_pass",
                                      "admission", "gather_issue", "calls"};
#define CPROF_T(v) v = h_prof_now()
#define CPROF_ADD(k, a, b) (g_cprof[k] += (b) - (a))
__attribute__((visibility("hidden"))) void udpdk_poll_profile_dump(void)
{
    if (g_prof[7]) {
        fprintf(stderr, "{\"udpdk_poll_profile_ms_per_call\": {");
        for (int k = 0; k < 7; k++) fprintf(stderr, "%s\"%s\": %.3f", k ? ", " : "", g_prof_name[k], g_prof[k] / g_prof[7]);
        fprintf(stderr, "}, \"calls\": %.0f}\n", g_prof[7]);
    }
    if (g_cprof[7]) {
        fprintf(stderr, "{\"udpdk_poll_chunked_profile_ms_per_call\": {");
        for (int k = 0; k < 7; k++) fprintf(stderr, "%s\"%s\": %.3f", k ? ", " : "", g_cprof_name[k], g_cprof[k] / g_cprof[7]);
        fprintf(stderr, "}, \"calls\": %.0f}\n", g_cprof[7]);
    }
}
#else
#define PROF_T(v) do {} while (0)
#define PROF_ADD(k, a, b) do {} while (0)
#define CPROF_T(v) (void)(v)
#define CPROF_ADD(k, a, b) do {} while (0)
void udpdk_poll_profile_dump(void) {}
#endif

int h_grow_dev_on(udpdk_gpu_ctx *g, void **p, uint64_t *cap, uint64_t need)
{
    if (*p && *cap >= need) return 0;
    if (*p) udpdk_gpu_free(g, *p);
    *p = NULL;
    *cap = 0;
    uint64_t nc = need < 4096 ? 4096 : need + need / 4;
    const int rc = udpdk_gpu_alloc(g, nc, p);
    if (rc) { errno = -rc; return -1; }
    *cap = nc;
    return 0;
}

int h_grow_dev(void **p, uint64_t *cap, uint64_t need) { return h_grow_dev_on(g_udpdk.gpu, p, cap, need); }

static void h_gbuf_free(udpdk_gpu_ctx *g, struct h_gbuf *b)
{
    void *d[] = {b->acc, b->pay, b->len, b->sip, b->spt};
    for (unsigned k = 0; k < 5; k++)
        if (d[k] && g) udpdk_gpu_free(g, d[k]);
    memset(b, 0, sizeof(*b));
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
                     (void **)&g_udpdk.acc_do, (void **)&g_udpdk.acc_fo, (void **)&g_udpdk.acc_sock,
                     (void **)&g_udpdk.acc_dk, (void **)&g_udpdk.acc_di, (void **)&g_udpdk.fb_frames,
                     (void **)&g_udpdk.fb_off, (void **)&g_udpdk.fb_idx, (void **)&g_udpdk.fb_meta,
                     (void **)&g_udpdk.fb_loff, (void **)&g_udpdk.fb_lpkt, (void **)&g_udpdk.fb_pt,
                     (void **)&g_udpdk.fb_len};
    uint64_t *hcap[] = {&g_udpdk.rx_meta_cap, &g_udpdk.rx_loff_cap, &g_udpdk.rx_lpkt_cap,
                        &g_udpdk.fr_loff_cap, &g_udpdk.fr_lpkt_cap, &g_udpdk.fr_org_cap,
                        &g_udpdk.fr_len_cap, &g_udpdk.acc_d_cap, &g_udpdk.acc_f_cap,
                        &g_udpdk.acc_do_cap, &g_udpdk.acc_fo_cap, &g_udpdk.acc_sock_cap,
                        &g_udpdk.acc_dk_cap, &g_udpdk.acc_di_cap, &g_udpdk.fb_frames_cap,
                        &g_udpdk.fb_off_cap, &g_udpdk.fb_idx_cap, &g_udpdk.fb_meta_cap,
                        &g_udpdk.fb_loff_cap, &g_udpdk.fb_lpkt_cap, &g_udpdk.fb_pt_cap,
                        &g_udpdk.fb_len_cap};
    for (unsigned k = 0; k < sizeof(host) / sizeof(host[0]); k++) {
        free(*host[k]);
        *host[k] = NULL;
        *hcap[k] = 0;
    }
    void **dev[] = {&g_udpdk.dv_meta2, &g_udpdk.dv_loff2, &g_udpdk.dv_lpkt2};
    uint64_t *dcap[] = {&g_udpdk.dv_meta2_cap, &g_udpdk.dv_loff2_cap, &g_udpdk.dv_lpkt2_cap};
    for (unsigned k = 0; k < sizeof(dev) / sizeof(dev[0]); k++) {
        if (*dev[k] && g_udpdk.gpu) udpdk_gpu_free(g_udpdk.gpu, *dev[k]);
        *dev[k] = NULL;
        *dcap[k] = 0;
    }
    h_gbuf_free(g_udpdk.gpu, &g_udpdk.gb);
    void **pin[] = {(void **)&g_udpdk.pc_meta, (void **)&g_udpdk.pc_loff, (void **)&g_udpdk.pc_lpkt,
                    (void **)&g_udpdk.pc_acc};
    uint64_t *pcap[] = {&g_udpdk.pc_meta_cap, &g_udpdk.pc_loff_cap, &g_udpdk.pc_lpkt_cap, &g_udpdk.pc_acc_cap};
    for (unsigned k = 0; k < sizeof(pin) / sizeof(pin[0]); k++) {
        if (*pin[k] && g_udpdk.gpu) udpdk_gpu_host_free(g_udpdk.gpu, *pin[k]);
        *pin[k] = NULL;
        *pcap[k] = 0;
    }
}

/* The shard contexts and their buffers (udpdk_cleanup). */
void h_shards_destroy(void)
{
    for (uint32_t k = 0; k < H_MAX_DEVS; k++) {
        struct h_shard *S = &g_udpdk.shard[k];
        h_gbuf_free(S->g, &S->gb);
        free(S->off); free(S->meta); free(S->loff); free(S->lpkt); free(S->acc); free(S->acco);
        free(S->idx); free(S->pack); free(S->plen); free(S->ppt);
        if (S->g) udpdk_gpu_ctx_destroy(S->g);
        memset(S, 0, sizeof(*S));
    }
    g_udpdk.n_shards = 0;
    free(g_udpdk.rss_sh); free(g_udpdk.rss_loc);
    g_udpdk.rss_sh = NULL; g_udpdk.rss_loc = NULL;
    g_udpdk.rss_sh_cap = g_udpdk.rss_loc_cap = 0;
    g_udpdk.rss_ready = 0;
}

/* Upload the bind snapshot when the table changed since the last upload; keep its lane count
 * and largest per-port fan-out (the lane capacity a batch can need) with it. g_udpdk.lock held. */
int h_snapshot_refresh(void)
{
    if (g_udpdk.snap_version == g_udpdk.version) return 0;
    udpdk_bind_snapshot_t snap;
    if (udpdk_btable_snapshot(&snap, 0)) return -1;
    int rc = udpdk_gpu_bind_snapshot_upload(g_udpdk.gpu, &snap);
    for (uint32_t k = 0; !rc && g_udpdk.n_shards > 1 && k < g_udpdk.n_shards; k++)
        rc = udpdk_gpu_bind_snapshot_upload(g_udpdk.shard[k].g, &snap);
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
/* Whether the batch's in-range frames are disjoint and in ascending buffer order (each frame ends
 * at or before the next one starts): the precondition of udpdk_gpu_rx_reassemble_inplace, which
 * moves fragment bytes inside the buffer that the direct frames are later gathered from. A caller
 * whose descriptors alias (overlapping or repeated offsets, a frame inside another) keeps the
 * copying reassembly. Out-of-range descriptors are BAD_DESC and never read. */
static int h_desc_disjoint(const uint32_t *offset, const uint16_t *length, uint32_t n, uint64_t frames_bytes)
{
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t o = offset[i], l = length[i];
        if (l > frames_bytes || o > frames_bytes - l) continue;
        if (o < end) return 0;
        end = o + l;
    }
    return 1;
}

static int h_frag_pass(const udpdk_rx_batch_t *staged, const uint32_t *meta_dev, uint64_t nfrag,
                       uint32_t lanes, uint32_t maxfan, int inplace, udpdk_rx_batch_t *rb, uint32_t *nd)
{
    *nd = 0;
    if (!nfrag) return 0;                   /* the batch's FRAG verdict count (RX counters) */
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    int rc;
    if (!g_udpdk.frag_ready) {
        /* max_entries: [gpu] frag_max_entries, else the poller's NUM_FLOWS_MAX = UINT16_MAX
         * (udpdk_poller.c:130-131, udpdk_constants.h:34) where the table has more entries than
         * that (the reference's 4096 x 16 = 65536), else every entry */
        uint64_t ent = 1;
        while (ent < (uint64_t)g_udpdk.frag_buckets * g_udpdk.frag_entries) ent <<= 1;
        const uint32_t mx = g_udpdk.frag_max_entries ? g_udpdk.frag_max_entries
                          : ent > 0xFFFFu ? 0xFFFFu : 0u;
        udpdk_frag_table_cfg_t fc = {g_udpdk.frag_buckets, g_udpdk.frag_entries, g_udpdk.frag_ttl_ms,
                                     g_udpdk.frag_max_dgram, mx, g_udpdk.frag_flags, 0};
        if ((rc = udpdk_gpu_frag_table_create(g, &fc))) { errno = -rc; return -1; }
        g_udpdk.frag_ready = 1;
    }
    /* the staged frames are the library's device copy of the burst and the FRAG frames' bytes
     * are not read again after this pass: when the burst's frames are disjoint (inplace),
     * datagrams whose fragments arrived back to back are closed up in that buffer instead of
     * copied (udpdk_gpu_rx_reassemble_inplace); otherwise a moved fragment could overwrite bytes
     * another descriptor still delivers, and the pass copies */
    udpdk_reasm_out_t ro;
    udpdk_rx_batch_t sb = *staged;
    rc = inplace ? udpdk_gpu_rx_reassemble_inplace(g, &sb, meta_dev, h_now_ms(), &ro)
                 : udpdk_gpu_rx_reassemble(g, &sb, meta_dev, h_now_ms(), &ro);
    if (rc) { errno = -rc; return -1; }
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
static int h_gather(udpdk_gpu_ctx *g, struct h_gbuf *gb, const udpdk_rx_batch_t *b, const uint32_t *acc,
                    const uint32_t *offs, uint32_t count, struct h_arena **out)
{
    *out = NULL;
    if (!count) return 0;
    const uint64_t bytes = offs[count] ? offs[count] : 16u;
    struct h_arena *a = h_arena_get(count, bytes);
    if (!a) return -1;                             /* ENOBUFS (budget) or ENOMEM */
    int rc;
    if (h_grow_dev_on(g, &gb->acc, &gb->acc_cap, 8ull * count + 4) ||
        h_grow_dev_on(g, &gb->pay, &gb->pay_cap, bytes) ||
        h_grow_dev_on(g, &gb->len, &gb->len_cap, 4ull * count) ||
        h_grow_dev_on(g, &gb->sip, &gb->sip_cap, 4ull * count) ||
        h_grow_dev_on(g, &gb->spt, &gb->spt_cap, 2ull * count)) {
        h_arena_put(a);
        return -1;
    }
    udpdk_rx_gather_t go = {gb->pay, 16u, gb->len, gb->sip, gb->spt};
    uint32_t *dacc = gb->acc, *doff = dacc + count;
    if ((rc = udpdk_gpu_h2d(g, dacc, acc, 4ull * count)) ||
        (rc = udpdk_gpu_h2d(g, doff, offs, 4ull * count + 4)) ||
        (rc = udpdk_gpu_rx_gather_packed(g, b, dacc, 0, count, doff, &go)) ||
        (rc = udpdk_gpu_d2h(g, a->payload, gb->pay, bytes)) ||
        (rc = udpdk_gpu_d2h(g, a->len, gb->len, 4ull * count)) ||
        (rc = udpdk_gpu_d2h(g, a->src_ip, gb->sip, 4ull * count)) ||
        (rc = udpdk_gpu_d2h(g, a->src_port, gb->spt, 2ull * count))) {
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
    uint32_t n;                       /* frames in the batch: every lane entry is below it */
    atomic_int bad;                   /* a lane entry was not (the device returned garbage) */
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
    if (!A->fill) {
        for (uint32_t x = a0; x < a1; x++) {
            if (lpkt[x] >= A->n) {
                atomic_store_explicit((atomic_int *)&A->bad, 1, memory_order_relaxed);
                return;
            }
        }
    }
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
    int sharded;                 /* direct entries in per-shard slabs (acc_dk / acc_di) */
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
                    struct h_arena *ad = P->sharded ? g_udpdk.shard[g_udpdk.acc_dk[kd]].arena : P->ad;
                    const uint32_t j = P->sharded ? g_udpdk.acc_di[kd] : kd;
                    d->arena = ad;
                    d->data = ad->payload + g_udpdk.acc_do[kd];
                    d->len = ad->len[j];
                    d->src_ip = ad->src_ip[j];
                    d->src_port = ad->src_port[j];
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

/* ---- payload copy on the host ---------------------------------------------------------------
 * The poll's frames are in host memory already (the caller's batch, a NIC's DMA target), so for
 * long datagrams the payloads are copied from there into the slab on the pool's threads instead of
 * being gathered on the GPU and copied back across PCIe (the 1500 B poll paid the link twice for
 * its payloads). Same result as rx_gather (rx_gather.hip): n = min(data_len - 42, dgram_len - 8
 * as uint16_t, slot room), source address and port as raw wire words (udpdk_syscall.c:436-466). */
struct h_hcopy {
    const uint8_t *frames;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *acc, *offs;
    uint32_t count;
    struct h_arena *a;
};

static void h_hcopy_job(void *ctx, uint32_t part, uint32_t parts)
{
    const struct h_hcopy *H = ctx;
    const uint32_t k0 = (uint32_t)((uint64_t)H->count * part / parts);
    const uint32_t k1 = (uint32_t)((uint64_t)H->count * (part + 1) / parts);
    for (uint32_t k = k0; k < k1; k++) {
        const uint32_t fi = H->acc[k];
        const uint8_t *f = H->frames + H->offset[fi];
        const uint32_t len = H->length[fi];
        const uint32_t seg = len >= 42u ? len - 42u : 0u;
        const uint32_t dl = ((uint32_t)f[38] << 8) | f[39];
        const uint32_t pl = (dl - 8u) & 0xFFFFu;
        const uint32_t cap = H->offs[k + 1] - H->offs[k];
        uint32_t n = seg < pl ? seg : pl;
        if (n > cap) n = cap;
        memcpy(H->a->payload + H->offs[k], f + 42, n);
        H->a->len[k] = n;
        memcpy(&H->a->src_ip[k], f + 26, 4);
        memcpy(&H->a->src_port[k], f + 34, 2);
    }
}

static int h_host_gather(const uint8_t *frames, const uint32_t *offset, const uint16_t *length,
                         const uint32_t *acc, const uint32_t *offs, uint32_t count, struct h_arena **out)
{
    *out = NULL;
    if (!count) return 0;
    struct h_arena *a = h_arena_get(count, offs[count] ? offs[count] : 16u);
    if (!a) return -1;
    struct h_hcopy H = {frames, offset, length, acc, offs, count, a};
    h_pool_run(h_hcopy_job, &H);
    *out = a;
    return 0;
}

/* ---- multi-device shards ------------------------------------------------------------------ */
struct h_sjob {
    const uint8_t *frames;
    uint64_t frames_bytes;
    const uint32_t *offset;
    const uint16_t *length;
    const uint32_t *ptype;
    uint32_t maxfan;
};

/* ---- RSS dispatch ([gpu] dispatch = rss) ---------------------------------------------------
 * The NIC's receive-side scaling in software (the reference asks for
 * ETH_MQ_RX_RSS with one ring and a "TODO add RSS support", udpdk_init.c:112-137): one RX queue
 * per device, a frame's queue = reta[Toeplitz hash], with udpdk_gpu_rss's hash definition
 * (rx_rss.hip: IPv4 gate as rx_classify, source + destination address, + ports for unfragmented
 * UDP) and its default key and redirection table, by the same 12 x 256 key-window table. Each
 * device then classifies its queue's frames; lanes are merged back in arrival order, so the rings
 * are the single-queue poller's. */
static uint32_t h_key_window(const uint8_t *key, uint32_t b)   /* key bits [b, b + 32), MSB first */
{
    uint64_t w = 0;
    for (uint32_t i = 0; i < 5; i++) w = (w << 8) | key[(b >> 3) + i];
    return (uint32_t)(w >> (8u - (b & 7u)));
}

int h_rss_setup(void)
{
    udpdk_rss_conf_t conf;
    if (udpdk_gpu_rss_default_conf(&conf, g_udpdk.n_shards)) return -1;
    for (uint32_t p = 0; p < 12; p++)
        for (uint32_t v = 0; v < 256; v++) {
            uint32_t t = 0;
            for (uint32_t j = 0; j < 8; j++)
                if (v & (0x80u >> j)) t ^= h_key_window(conf.key, 8u * p + j);
            g_udpdk.rss_tab[p][v] = t;
        }
    memcpy(g_udpdk.rss_reta, conf.reta, sizeof(uint16_t) * conf.reta_size);
    g_udpdk.rss_reta_size = conf.reta_size;
    g_udpdk.rss_types = conf.hash_types;
    g_udpdk.rss_ready = 1;
    return 0;
}

/* frame i's RX queue (= shard) */
static uint32_t h_rss_queue(const struct h_sjob *J, uint32_t i)
{
    const uint64_t o = J->offset[i];
    const uint32_t len = J->length[i];
    uint32_t hash = 0;
    if (len >= 34u && o + len <= J->frames_bytes) {
        const uint8_t *f = J->frames + o;
        const uint32_t pt = J->ptype ? J->ptype[i] : (f[12] == 0x08 && f[13] == 0x00 ? 0x211u : 0x1u);
        if (pt & 0x10u) {
            const uint32_t ff = ((uint32_t)f[20] << 8) | f[21];
            const int udp4 = !(ff & 0x3FFFu) && f[23] == 17 && len >= 38u && (g_udpdk.rss_types & 2u);
            if (udp4 || (g_udpdk.rss_types & 1u)) {
                const uint32_t (*T)[256] = g_udpdk.rss_tab;
                for (uint32_t b = 0; b < (udp4 ? 12u : 8u); b++) hash ^= T[b][f[26 + b]];
            }
        }
    }
    return g_udpdk.rss_reta[hash & (g_udpdk.rss_reta_size - 1u)];
}

/* Two passes over contiguous parts of the poll: queue of every frame and per-part counts per
 * shard, then (at per-part, per-shard bases) every shard's frames in arrival order. */
struct h_rss {
    const struct h_sjob *J;
    uint32_t n, N;
    int fill;
    uint32_t cnt[H_MAX_WORKERS + 2][H_MAX_DEVS];
};

static void h_rss_job(void *ctx, uint32_t part, uint32_t parts)
{
    struct h_rss *R = ctx;
    const uint32_t i0 = (uint32_t)((uint64_t)R->n * part / parts), i1 = (uint32_t)((uint64_t)R->n * (part + 1) / parts);
    uint8_t *sh = g_udpdk.rss_sh;
    if (!R->fill) {
        uint32_t c[H_MAX_DEVS] = {0};
        for (uint32_t i = i0; i < i1; i++) {
            const uint32_t k = h_rss_queue(R->J, i) % R->N;
            sh[i] = (uint8_t)k;
            c[k]++;
        }
        memcpy(R->cnt[part], c, sizeof(c));
    } else {
        uint32_t w[H_MAX_DEVS];
        memcpy(w, R->cnt[part], sizeof(w));
        for (uint32_t i = i0; i < i1; i++) {
            const uint32_t k = sh[i], r = w[k]++;
            g_udpdk.shard[k].idx[r] = i;
            g_udpdk.rss_loc[i] = r;
        }
    }
}

static int h_rss_assign(const struct h_sjob *J, uint32_t n)
{
    const uint32_t N = g_udpdk.n_shards;
    if (h_grow_host((void **)&g_udpdk.rss_sh, &g_udpdk.rss_sh_cap, (uint64_t)n + 1) ||
        h_grow_host((void **)&g_udpdk.rss_loc, &g_udpdk.rss_loc_cap, 4ull * n + 4))
        return -1;
    struct h_rss R;
    memset(&R, 0, sizeof(R));
    R.J = J;
    R.n = n;
    R.N = N;
    const uint32_t parts = h_pool_parts();
    h_pool_run(h_rss_job, &R);
    uint32_t tot[H_MAX_DEVS] = {0};
    for (uint32_t p = 0; p < parts; p++)          /* per-part counts -> per-part bases */
        for (uint32_t k = 0; k < N; k++) {
            const uint32_t c = R.cnt[p][k];
            R.cnt[p][k] = tot[k];
            tot[k] += c;
        }
    for (uint32_t k = 0; k < N; k++) {
        struct h_shard *S = &g_udpdk.shard[k];
        S->n = tot[k];
        S->i0 = 0;
        if (h_grow_host((void **)&S->idx, &S->idx_cap, 4ull * tot[k] + 4)) return -1;
    }
    R.fill = 1;
    h_pool_run(h_rss_job, &R);
    return 0;
}

/* The lanes a shard's device returned, checked before any of them is used as a host index (the
 * merge indexes S->lpkt / S->idx with them and writes the poll's lane array): offsets from 0,
 * non-decreasing, the total within the shard's entry buffer, every entry a frame of the shard. */
static int h_shard_lanes_ok(const struct h_shard *S, uint32_t lanes, uint64_t cap)
{
    if (S->loff[0] != 0u) return 0;
    for (uint32_t l = 0; l < lanes; l++)
        if (S->loff[l] > S->loff[l + 1]) return 0;
    const uint32_t D = S->loff[lanes];
    if (D > cap) return 0;
    for (uint32_t e = 0; e < D; e++)
        if (S->lpkt[e] >= S->n) return 0;
    return 1;
}

/* Shard k's RX on its own context: descriptors rebased to the 16-byte-aligned start of the frame
 * bytes the shard spans (a descriptor outside the caller's frames keeps pointing outside the
 * shard's, so it stays BAD_DESC), then udpdk_gpu_rx_host (H2D, kernels, D2H of its lanes). */
static void h_shard_rx(const struct h_sjob *J, struct h_shard *S)
{
    S->err = 0;
    memset(&S->st, 0, sizeof(S->st));
    const uint32_t lanes = g_udpdk.snap_lanes;
    if (h_grow_host((void **)&S->loff, &S->loff_cap, 4ull * (lanes + 1))) { S->err = errno; return; }
    if (!S->n) {
        memset(S->loff, 0, 4ull * (lanes + 1));
        return;
    }
    if (g_udpdk.dispatch_rss) {
        /* the queue's frames packed back to back (+ 16 readable bytes), descriptors and ptypes
         * in queue order; a descriptor outside the caller's frames stays out of range */
        uint64_t bytes = 0;
        for (uint32_t i = 0; i < S->n; i++) bytes += J->length[S->idx[i]];
        const uint64_t cap = (uint64_t)S->n * J->maxfan;
        if (h_grow_host((void **)&S->pack, &S->pack_cap, bytes + 64) ||
            h_grow_host((void **)&S->off, &S->off_cap, 4ull * S->n) ||
            h_grow_host((void **)&S->plen, &S->plen_cap, 2ull * S->n) ||
            h_grow_host((void **)&S->ppt, &S->ppt_cap, 4ull * S->n) ||
            h_grow_host((void **)&S->meta, &S->meta_cap, 4ull * S->n + 4) ||
            h_grow_host((void **)&S->lpkt, &S->lpkt_cap, 4ull * cap + 4)) { S->err = errno; return; }
        uint64_t pos = 0;
        for (uint32_t i = 0; i < S->n; i++) {
            const uint32_t gi = S->idx[i];
            const uint64_t o = J->offset[gi];
            const uint32_t l = J->length[gi];
            S->plen[i] = (uint16_t)l;
            S->ppt[i] = J->ptype ? J->ptype[gi] : 0u;
            if (l <= J->frames_bytes && o <= J->frames_bytes - l) {
                memcpy(S->pack + pos, J->frames + o, l);
                S->off[i] = (uint32_t)pos;
                pos += l;
            } else {
                S->off[i] = 0xFFFFFFFFu;
            }
        }
        memset(S->pack + pos, 0, 16);
        S->lo = 0;
        S->bytes = pos;
        const int rc = udpdk_gpu_rx_host(S->g, S->pack, pos, S->off, S->plen, J->ptype ? S->ppt : NULL, S->n,
                                         S->meta, S->loff, S->lpkt, cap > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap,
                                         &S->st);
        if (rc) S->err = -rc;
        else if (!h_shard_lanes_ok(S, lanes, cap)) S->err = EIO;
        return;
    }
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t i = 0; i < S->n; i++) {
        const uint64_t o = J->offset[S->i0 + i], e = o + J->length[S->i0 + i];
        if (J->length[S->i0 + i] <= J->frames_bytes && o <= J->frames_bytes - J->length[S->i0 + i]) {
            if (o < lo) lo = o;
            if (e > hi) hi = e;
        }
    }
    if (lo == UINT64_MAX) lo = hi = 0;
    lo &= ~(uint64_t)15u;
    S->lo = lo;
    S->bytes = hi - lo;
    const uint64_t cap = (uint64_t)S->n * J->maxfan;
    if (h_grow_host((void **)&S->off, &S->off_cap, 4ull * S->n) ||
        h_grow_host((void **)&S->meta, &S->meta_cap, 4ull * S->n + 4) ||
        h_grow_host((void **)&S->lpkt, &S->lpkt_cap, 4ull * cap + 4)) { S->err = errno; return; }
    for (uint32_t i = 0; i < S->n; i++) {
        const uint64_t o = J->offset[S->i0 + i];
        const uint32_t l = J->length[S->i0 + i];
        const int ok = l <= J->frames_bytes && o <= J->frames_bytes - l;
        S->off[i] = ok ? (uint32_t)(o - lo) : 0xFFFFFFFFu;    /* out of the shard: BAD_DESC */
    }
    const int rc = udpdk_gpu_rx_host(S->g, J->frames + lo, S->bytes, S->off, J->length + S->i0,
                                     J->ptype ? J->ptype + S->i0 : NULL, S->n, S->meta, S->loff, S->lpkt,
                                     cap > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap, &S->st);
    if (rc) S->err = -rc;
    else if (!h_shard_lanes_ok(S, lanes, cap)) S->err = EIO;
}

static void h_shard_rx_job(void *ctx, uint32_t part, uint32_t parts)
{
    for (uint32_t k = part; k < g_udpdk.n_shards; k += parts) h_shard_rx(ctx, &g_udpdk.shard[k]);
}

/* the shards' lanes concatenated per socket in shard order, sockets split over the pool */
struct h_merge {
    uint32_t lanes;
    uint32_t *loff, *lpkt;
    uint32_t sb[H_MAX_WORKERS + 3];
};

static void h_merge_job(void *ctx, uint32_t part, uint32_t parts)
{
    const struct h_merge *M = ctx;
    (void)parts;
    if (g_udpdk.dispatch_rss) {
        /* every shard's list for the socket holds its frames in arrival order: merge them by
         * poll index (the single-queue arrival order) */
        const uint32_t N = g_udpdk.n_shards;
        for (uint32_t l = M->sb[part]; l < M->sb[part + 1]; l++) {
            uint32_t w = M->loff[l], e[H_MAX_DEVS], b[H_MAX_DEVS];
            for (uint32_t k = 0; k < N; k++) {
                const struct h_shard *S = &g_udpdk.shard[k];
                e[k] = S->n ? S->loff[l] : 0u;
                b[k] = S->n ? S->loff[l + 1] : 0u;
            }
            for (;;) {
                uint32_t best = UINT32_MAX, bk = 0;
                for (uint32_t k = 0; k < N; k++) {
                    if (e[k] >= b[k]) continue;
                    const uint32_t gi = g_udpdk.shard[k].idx[g_udpdk.shard[k].lpkt[e[k]]];
                    if (gi < best) { best = gi; bk = k; }
                }
                if (best == UINT32_MAX) break;
                M->lpkt[w++] = best;
                e[bk]++;
            }
        }
        return;
    }
    for (uint32_t l = M->sb[part]; l < M->sb[part + 1]; l++) {
        uint32_t w = M->loff[l];
        for (uint32_t k = 0; k < g_udpdk.n_shards; k++) {
            const struct h_shard *S = &g_udpdk.shard[k];
            if (!S->n) continue;
            const uint32_t a = S->loff[l], b = S->loff[l + 1], base = S->i0;
            for (uint32_t e = a; e < b; e++) M->lpkt[w++] = S->lpkt[e] + base;
        }
    }
}

/* Step 1 over the shards: per-shard RX in parallel, then stats summed, lanes merged, verdict
 * words concatenated (the FRAG frames are found in them). */
static int h_shards_rx(const struct h_sjob *J, uint32_t n, uint32_t lanes, uint32_t *meta, uint32_t *loff,
                       uint32_t *lpkt, udpdk_rx_stats_t *st)
{
    const uint32_t N = g_udpdk.n_shards;
    if (g_udpdk.dispatch_rss) {
        if (h_rss_assign(J, n)) return -1;
    } else {
        for (uint32_t k = 0; k < N; k++) {
            struct h_shard *S = &g_udpdk.shard[k];
            S->i0 = (uint32_t)((uint64_t)n * k / N);
            S->n = (uint32_t)((uint64_t)n * (k + 1) / N) - S->i0;
        }
    }
    h_pool_run(h_shard_rx_job, (void *)J);
    memset(st, 0, sizeof(*st));
    for (uint32_t k = 0; k < N; k++) {
        const struct h_shard *S = &g_udpdk.shard[k];
        if (S->err) { errno = S->err; return -1; }
        for (int c = 0; c < UDPDK_N_COUNTERS; c++) st->counters[c] += S->st.counters[c];
        st->deliveries += S->st.deliveries;
        st->overflow |= S->st.overflow;
        if (!S->n) continue;
        if (g_udpdk.dispatch_rss)
            for (uint32_t i = 0; i < S->n; i++) meta[S->idx[i]] = S->meta[i];
        else
            memcpy(meta + S->i0, S->meta, 4ull * S->n);
    }
    for (uint32_t l = 0; l <= lanes; l++) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < N; k++)
            if (g_udpdk.shard[k].n) v += g_udpdk.shard[k].loff[l];
        loff[l] = v;
    }
    struct h_merge M = {lanes, loff, lpkt, {0}};
    const uint32_t parts = h_pool_parts(), D = loff[lanes];
    uint32_t l = 0;
    for (uint32_t p = 1; p < parts; p++) {
        const uint64_t want = (uint64_t)D * p / parts;
        while (l < lanes && loff[l] < want) l++;
        M.sb[p] = l;
    }
    M.sb[0] = 0;
    M.sb[parts] = lanes;
    h_pool_run(h_merge_job, &M);
    return 0;
}

/* The FRAG frames of a sharded poll, in arrival order, copied into one host batch that the main
 * context classifies (staging it on its device for the reassembly pass). fb_idx[j] = the poll
 * index of sub-batch frame j. */
static int h_frag_subbatch(const struct h_sjob *J, const uint32_t *meta, uint32_t n, uint32_t nfrag,
                           uint32_t maxfan, udpdk_rx_batch_t *staged, const uint32_t **meta_dev)
{
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < n; i++)
        if (UDPDK_META_VERDICT(meta[i]) == UDPDK_V_FRAG) bytes += J->length[i];
    const uint32_t lanes = g_udpdk.snap_lanes;
    if (h_grow_host((void **)&g_udpdk.fb_frames, &g_udpdk.fb_frames_cap, bytes + 64) ||
        h_grow_host((void **)&g_udpdk.fb_off, &g_udpdk.fb_off_cap, 4ull * nfrag) ||
        h_grow_host((void **)&g_udpdk.fb_len, &g_udpdk.fb_len_cap, 2ull * nfrag) ||
        h_grow_host((void **)&g_udpdk.fb_idx, &g_udpdk.fb_idx_cap, 4ull * nfrag) ||
        h_grow_host((void **)&g_udpdk.fb_pt, &g_udpdk.fb_pt_cap, 4ull * nfrag) ||
        h_grow_host((void **)&g_udpdk.fb_meta, &g_udpdk.fb_meta_cap, 4ull * nfrag) ||
        h_grow_host((void **)&g_udpdk.fb_loff, &g_udpdk.fb_loff_cap, 4ull * (lanes + 1)) ||
        h_grow_host((void **)&g_udpdk.fb_lpkt, &g_udpdk.fb_lpkt_cap, 4ull * nfrag * maxfan + 4))
        return -1;
    uint32_t j = 0;
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n && j < nfrag; i++) {
        if (UDPDK_META_VERDICT(meta[i]) != UDPDK_V_FRAG) continue;
        memcpy(g_udpdk.fb_frames + pos, J->frames + J->offset[i], J->length[i]);
        g_udpdk.fb_off[j] = (uint32_t)pos;
        g_udpdk.fb_len[j] = J->length[i];
        g_udpdk.fb_pt[j] = J->ptype ? J->ptype[i] : 0u;
        g_udpdk.fb_idx[j++] = i;
        pos += J->length[i];
    }
    memset(g_udpdk.fb_frames + pos, 0, 16);
    udpdk_rx_stats_t st;
    int rc = udpdk_gpu_rx_host(g_udpdk.gpu, g_udpdk.fb_frames, pos, g_udpdk.fb_off, g_udpdk.fb_len,
                               J->ptype ? g_udpdk.fb_pt : NULL, j, g_udpdk.fb_meta, g_udpdk.fb_loff,
                               g_udpdk.fb_lpkt, j * maxfan, &st);
    if (rc && rc != -ENOSPC) { errno = -rc; return -1; }
    if ((rc = udpdk_gpu_rx_host_batch(g_udpdk.gpu, staged, meta_dev))) { errno = -rc; return -1; }
    return 0;
}

static void h_shard_gather_job(void *ctx, uint32_t part, uint32_t parts)
{
    (void)ctx;
    for (uint32_t k = part; k < g_udpdk.n_shards; k += parts) {
        struct h_shard *S = &g_udpdk.shard[k];
        S->err = 0;
        S->arena = NULL;
        if (!S->nacc) continue;
        udpdk_rx_batch_t b;
        int rc = udpdk_gpu_rx_host_batch(S->g, &b, NULL);
        if (rc) { S->err = -rc; continue; }
        if (h_gather(S->g, &S->gb, &b, S->acc, S->acco, S->nacc, &S->arena)) { S->err = errno; continue; }
        if ((rc = udpdk_gpu_sync(S->g))) S->err = -rc;
    }
}

/* Step 4 over the shards: each accepted direct entry goes to its frame's shard (acc_dk), at the
 * next index of that shard's slab (acc_di) and slot offset (acc_do, rewritten per shard); each
 * shard gathers its entries on its own device into a slab of its own. */
static int h_shards_gather(uint32_t nad)
{
    const uint32_t N = g_udpdk.n_shards;
    if (h_grow_host((void **)&g_udpdk.acc_dk, &g_udpdk.acc_dk_cap, (uint64_t)nad + 1) ||
        h_grow_host((void **)&g_udpdk.acc_di, &g_udpdk.acc_di_cap, 4ull * nad + 4))
        return -1;
    for (uint32_t k = 0; k < N; k++) {
        struct h_shard *S = &g_udpdk.shard[k];
        S->nacc = 0;
        S->acc_bytes = 0;
        const uint64_t d = S->n ? (uint64_t)S->loff[g_udpdk.snap_lanes] : 0u;
        if (h_grow_host((void **)&S->acc, &S->acc_cap, 4ull * d + 4) ||
            h_grow_host((void **)&S->acco, &S->acco_cap, 4ull * d + 8))
            return -1;
    }
    const uint32_t *slot = g_udpdk.acc_do;           /* packed slot offsets: sizes by difference */
    for (uint32_t kd = 0; kd < nad; kd++) {
        const uint32_t fi = g_udpdk.acc_d[kd];
        uint32_t k = N - 1, local;
        if (g_udpdk.dispatch_rss) {
            k = g_udpdk.rss_sh[fi];
            local = g_udpdk.rss_loc[fi];
        } else {
            while (k && g_udpdk.shard[k].i0 > fi) k--;
            local = fi - g_udpdk.shard[k].i0;
        }
        struct h_shard *S = &g_udpdk.shard[k];
        const uint32_t r = S->nacc++;
        const uint32_t sz = slot[kd + 1] - slot[kd];
        g_udpdk.acc_dk[kd] = (uint8_t)k;
        g_udpdk.acc_di[kd] = r;
        S->acc[r] = local;
        S->acco[r] = (uint32_t)S->acc_bytes;
        S->acc_bytes += sz;
    }
    for (uint32_t k = 0; k < N; k++) {
        struct h_shard *S = &g_udpdk.shard[k];
        if (S->acc_bytes > 0xFFFFFFF0ull) { errno = ENOBUFS; return -1; }
        S->acco[S->nacc] = (uint32_t)S->acc_bytes;
    }
    /* the slot offsets now index the shards' slabs */
    for (uint32_t kd = 0; kd < nad; kd++)
        g_udpdk.acc_do[kd] = g_udpdk.shard[g_udpdk.acc_dk[kd]].acco[g_udpdk.acc_di[kd]];
    h_pool_run(h_shard_gather_job, NULL);
    int err = 0;
    for (uint32_t k = 0; k < N; k++)
        if (g_udpdk.shard[k].err && !err) err = g_udpdk.shard[k].err;
    if (err) {
        for (uint32_t k = 0; k < N; k++) {
            if (g_udpdk.shard[k].arena) h_arena_put(g_udpdk.shard[k].arena);
            g_udpdk.shard[k].arena = NULL;
        }
        errno = err;
        return -1;
    }
    return 0;
}

/* ---- pipelined form of an unsharded poll over a large host batch ----
 * The poller takes its bursts one after another (udpdk_poller.c:516-545); here a batch of at
 * least two [gpu] poll_chunk_mb chunks is cut into K chunks at burst boundaries and each chunk
 * runs the one-piece steps (RX, FRAG pass, admission, gather, publication) in order, on pipe
 * 1 + k % 3 of the context: chunk k + 1's RX (frames H2D, classify, verdicts and lanes D2H) is
 * enqueued before chunk k's admission and runs while chunk k - 1's payload slab comes back,
 * so the two PCIe directions overlap instead of following each other (58.8 ms for 1 M x 1500 B
 * in one piece: 30 ms of frames in, 29 ms of payloads out). A chunk is admitted only after the
 * chunk before it is published, so every burst's decision reads the room its ring has after
 * the bursts before it, as in the one-piece poll and the reference's burst loop. Chunks need
 * the batch's descriptors in range, ascending and disjoint (the network order a NIC ring gives);
 * others take the one-piece path. */
#define H_CHUNKS_MAX 32u

struct h_chunk {
    uint32_t f0, n;              /* frames [f0, f0 + n) of the poll                              */
    uint64_t lo, bytes;          /* the frame bytes they span (lo 16-byte aligned)               */
    udpdk_rx_stats_t st;
};

/* descriptors in range, ascending and disjoint (each frame ends at or before the next starts) */
static int h_desc_sorted(const uint32_t *offset, const uint16_t *length, uint32_t n, uint64_t frames_bytes)
{
    uint64_t end = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t o = offset[i], l = length[i];
        if (l > frames_bytes || o > frames_bytes - l || o < end) return 0;
        end = o + l;
    }
    return 1;
}

static inline int h_pipe_of(uint32_t k) { return 1 + (int)(k % 3u); }

/* The direct and reassembled payload gathers of one chunk on its pipe's stream: gather lists
 * H2D from pinned memory, the packed gather, the slabs' D2H. Both gathers share the device
 * buffers, in stream order. *ad / *af: the slabs (NULL when that count is 0). */
static int h_gather_chunk(udpdk_gpu_ctx *g, int pipe, const udpdk_rx_batch_t *b, uint32_t nad,
                          const udpdk_rx_batch_t *rb, uint32_t naf, struct h_arena **ad, struct h_arena **af)
{
    *ad = *af = NULL;
    const uint64_t bd = g_udpdk.acc_do[nad] ? g_udpdk.acc_do[nad] : 16u;
    const uint64_t bf = g_udpdk.acc_fo[naf] ? g_udpdk.acc_fo[naf] : 16u;
    const uint32_t cmax = nad > naf ? nad : naf;
    const uint64_t bmax = bd > bf ? bd : bf;
    struct h_gbuf *gb = &g_udpdk.gb;
    if (h_grow_pinned((void **)&g_udpdk.pc_acc, &g_udpdk.pc_acc_cap, 8ull * (nad + naf) + 8) ||
        h_grow_dev_on(g, &gb->acc, &gb->acc_cap, 8ull * cmax + 4) ||
        h_grow_dev_on(g, &gb->pay, &gb->pay_cap, bmax) ||
        h_grow_dev_on(g, &gb->len, &gb->len_cap, 4ull * cmax) ||
        h_grow_dev_on(g, &gb->sip, &gb->sip_cap, 4ull * cmax) ||
        h_grow_dev_on(g, &gb->spt, &gb->spt_cap, 2ull * cmax))
        return -1;
    const udpdk_rx_gather_t go = {gb->pay, 16u, gb->len, gb->sip, gb->spt};
    uint32_t *dacc = gb->acc;
    uint32_t *hl = g_udpdk.pc_acc;
    /* both slabs before any GPU work is queued: a chunk dropped for want of a slab (ENOBUFS)
     * leaves nothing in flight on its pipe that could still write gb or pc_acc, or the slab it
     * got, while the next chunk uses them */
    if (nad && !(*ad = h_arena_get(nad, bd))) return -1;     /* ENOBUFS (budget) or ENOMEM */
    if (naf && !(*af = h_arena_get(naf, bf))) {
        const int e = errno;
        if (*ad) h_arena_put(*ad);
        *ad = NULL;
        errno = e;
        return -1;
    }
    for (int part = 0; part < 2; part++) {
        const uint32_t cnt = part ? naf : nad;
        if (!cnt) continue;
        const uint32_t *acc = part ? g_udpdk.acc_f : g_udpdk.acc_d, *offs = part ? g_udpdk.acc_fo : g_udpdk.acc_do;
        const uint64_t bytes = part ? bf : bd;
        struct h_arena *a = part ? *af : *ad;
        memcpy(hl, acc, 4ull * cnt);
        memcpy(hl + cnt, offs, 4ull * cnt + 4);
        int rc;
        if ((rc = udpdk_gpu_pipe_h2d(g, pipe, dacc, hl, 8ull * cnt + 4)) ||
            (rc = udpdk_gpu_pipe_gather_packed(g, pipe, part ? rb : b, dacc, 0, cnt, dacc + cnt, &go)) ||
            (rc = udpdk_gpu_pipe_d2h(g, pipe, a->payload, gb->pay, bytes)) ||
            (rc = udpdk_gpu_pipe_d2h(g, pipe, a->len, gb->len, 4ull * cnt)) ||
            (rc = udpdk_gpu_pipe_d2h(g, pipe, a->src_ip, gb->sip, 4ull * cnt)) ||
            (rc = udpdk_gpu_pipe_d2h(g, pipe, a->src_port, gb->spt, 2ull * cnt))) {
            errno = -rc;
            return -1;
        }
        hl += 2 * cnt + 1;
    }
    return 0;
}

/* 1: not taken (the caller polls in one piece); 0: done; -1: error (errno). */
static int h_poll_chunked(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                          const uint16_t *length, const uint32_t *ptype, uint32_t n, uint32_t lanes,
                          uint32_t maxfan, udpdk_rx_stats_t *stats_out)
{
    /* only batches of long frames ([gpu] poll_chunk_min_avg, default 1 KiB on average): there
     * the poll is the two PCIe legs and overlapping them pays (1 M x 1500 B: 60 -> 40 ms); with
     * short frames each socket's
     * datagrams end up in one slab region per chunk, and recvfrom's loop over them lost more than
     * the poll gained (1 M IMIX: poll 15.9 -> 12.7 ms, recvfrom 16.1 -> 24.0 ms) */
    const uint64_t chunk = (uint64_t)g_udpdk.poll_chunk_mb << 20;
    if (!chunk || g_udpdk.host_copy_min || frames_bytes < 2 * chunk || frames_bytes >= (1ull << 32) ||
        frames_bytes < (uint64_t)n * g_udpdk.poll_chunk_min_avg ||
        n < 2u * H_BURST_SIZE || (uint64_t)n * maxfan > (1ull << 28) ||
        !h_desc_sorted(offset, length, n, frames_bytes))
        return 1;
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    uint64_t kk = frames_bytes / chunk;
    const uint32_t want = kk > H_CHUNKS_MAX ? H_CHUNKS_MAX : (uint32_t)kk;
    struct h_chunk ck[H_CHUNKS_MAX];
    uint32_t K = 0, f = 0;
    for (uint32_t k = 1; k <= want; k++) {             /* byte-balanced cuts at burst boundaries */
        uint32_t e = n;
        if (k < want) {
            const uint64_t target = frames_bytes * k / want;
            uint32_t a = f, b = n;
            while (a < b) {
                const uint32_t m = a + (b - a) / 2;
                if (offset[m] < target) a = m + 1; else b = m;
            }
            e = a - a % H_BURST_SIZE;
            if (e <= f) continue;
        }
        const uint64_t lo = offset[f] & ~(uint64_t)15u, hi = (uint64_t)offset[e - 1] + length[e - 1];
        ck[K].f0 = f;
        ck[K].n = e - f;
        ck[K].lo = lo;
        ck[K].bytes = hi > lo ? hi - lo : 0;
        K++;
        f = e;
    }
    if (K < 2) return 1;
    const uint32_t L1 = lanes + 1, SL = lanes < UDPDK_MAX_SOCKETS ? lanes : UDPDK_MAX_SOCKETS;
    /* (pinned staging that cannot be had: the one-piece poll, which stages in pageable memory) */
    if (h_grow_pinned((void **)&g_udpdk.pc_meta, &g_udpdk.pc_meta_cap, 4ull * n + 4) ||
        h_grow_pinned((void **)&g_udpdk.pc_loff, &g_udpdk.pc_loff_cap, 4ull * L1 * K) ||
        h_grow_pinned((void **)&g_udpdk.pc_lpkt, &g_udpdk.pc_lpkt_cap, 4ull * n * maxfan + 4))
        return 1;
    int rc, err = 0;
    struct h_arena *ad = NULL, *af = NULL;       /* slabs of the chunk whose gather is in flight */
    uint32_t pnad = 0, pnaf = 0;
    int pend = -1;
    struct h_adm A;
    udpdk_rx_stats_t tot;
    memset(&tot, 0, sizeof(tot));
#define CK_ISSUE(k) udpdk_gpu_pipe_rx_host(g, h_pipe_of(k), frames + ck[k].lo, ck[k].bytes, offset + ck[k].f0,     \
                                           (uint32_t)ck[k].lo, length + ck[k].f0, ptype ? ptype + ck[k].f0 : NULL, \
                                           ck[k].n, g_udpdk.pc_meta + ck[k].f0, g_udpdk.pc_loff + (uint64_t)L1 * (k), \
                                           g_udpdk.pc_lpkt + (uint64_t)ck[k].f0 * maxfan, ck[k].n * maxfan, &ck[k].st)
    double t0 = 0, t1 = 0;
    (void)t0; (void)t1;
    if ((rc = CK_ISSUE(0))) { errno = -rc; return -1; }
    for (uint32_t k = 0; k < K && !err; k++) {
        CPROF_T(t0);
        if (k + 1 < K && (rc = CK_ISSUE(k + 1))) { err = -rc; break; }
        CPROF_T(t1); CPROF_ADD(0, t0, t1);
        rc = udpdk_gpu_pipe_wait(g, h_pipe_of(k));
        if (rc && rc != -ENOSPC) { err = -rc; break; }
        CPROF_T(t0); CPROF_ADD(1, t1, t0);
        /* chunk k - 1: its payloads are home, publish them */
        if (pend >= 0) {
            if ((rc = udpdk_gpu_pipe_wait(g, h_pipe_of((uint32_t)pend)))) { err = -rc; break; }
            CPROF_T(t1); CPROF_ADD(2, t0, t1); t0 = t1;
            if (ad) atomic_store_explicit(&ad->refs, pnad, memory_order_relaxed);
            if (af) atomic_store_explicit(&af->refs, pnaf, memory_order_relaxed);
            struct h_pub P = {&A, ad, af, 0};
            h_pool_run(h_pub_job, &P);
            ad = af = NULL;
            pend = -1;
            CPROF_T(t1); CPROF_ADD(3, t0, t1); t0 = t1;
        }
        const struct h_chunk *C = &ck[k];
        const uint32_t *loff = g_udpdk.pc_loff + (uint64_t)L1 * k, *lpkt = g_udpdk.pc_lpkt + (uint64_t)C->f0 * maxfan;
        for (uint32_t v = 0; v < UDPDK_N_COUNTERS; v++) tot.counters[v] += C->st.counters[v];
        tot.deliveries += C->st.deliveries;
        tot.overflow |= C->st.overflow;
        udpdk_rx_batch_t staged, rb;
        const uint32_t *meta_dev = NULL;
        if ((rc = udpdk_gpu_pipe_batch(g, h_pipe_of(k), &staged, &meta_dev))) { err = -rc; break; }
        uint32_t nd = 0;
        const uint64_t nfrag = C->st.counters[UDPDK_V_FRAG];
        if (h_frag_pass(&staged, meta_dev, nfrag, lanes, maxfan, 1, &rb, &nd)) { err = errno; break; }
        CPROF_T(t1); CPROF_ADD(4, t0, t1); t0 = t1;
        const uint32_t *floff = nd ? g_udpdk.fr_loff : NULL;
        const uint32_t cap = C->n * maxfan, D = loff[lanes], DF = nd ? floff[lanes] : 0u;
        int lanes_ok = loff[0] == 0u && D <= cap;
        for (uint32_t s = 0; lanes_ok && s < lanes; s++) lanes_ok = loff[s] <= loff[s + 1];
        if (!lanes_ok) { err = EIO; break; }
        if (h_grow_host((void **)&g_udpdk.acc_d, &g_udpdk.acc_d_cap, 4ull * D + 4) ||
            h_grow_host((void **)&g_udpdk.acc_f, &g_udpdk.acc_f_cap, 4ull * DF + 4) ||
            h_grow_host((void **)&g_udpdk.acc_do, &g_udpdk.acc_do_cap, 4ull * D + 8) ||
            h_grow_host((void **)&g_udpdk.acc_fo, &g_udpdk.acc_fo_cap, 4ull * DF + 8) ||
            h_grow_host((void **)&g_udpdk.acc_sock, &g_udpdk.acc_sock_cap, 4ull * (D + DF) + 4)) {
            err = errno;
            break;
        }
        /* admission of the chunk's bursts (frame indices chunk-local; cuts at burst boundaries
         * keep the bursts the one-piece poll would form) */
        A.loff = loff; A.lpkt = lpkt; A.floff = floff; A.flpkt = g_udpdk.fr_lpkt; A.forg = g_udpdk.fr_org;
        A.length = length + C->f0; A.lanes = SL; A.fill = 0; A.n = C->n;
        atomic_init(&A.bad, 0);
        h_adm_split(&A, h_pool_parts());
        h_pool_run(h_adm_job, &A);
        if (atomic_load(&A.bad)) { err = EIO; break; }
        uint32_t nad = 0, naf = 0;
        uint64_t offd = 0, offf = 0;
        for (uint32_t s = 0; s < A.lanes; s++) {
            s_kd[s] = nad; s_kf[s] = naf; s_od[s] = offd; s_of[s] = offf;
            nad += s_nd[s]; naf += s_nf[s]; offd += s_bd[s]; offf += s_bf[s];
        }
        if (offd > 0xFFFFFFF0ull || offf > 0xFFFFFFF0ull) { err = ENOBUFS; break; }
        A.fill = 1;
        h_pool_run(h_adm_job, &A);
        g_udpdk.acc_do[nad] = (uint32_t)offd;
        g_udpdk.acc_fo[naf] = (uint32_t)offf;
        CPROF_T(t1); CPROF_ADD(5, t0, t1); t0 = t1;
        if (nad + naf && h_gather_chunk(g, h_pipe_of(k), &staged, nad, &rb, naf, &ad, &af)) {
            if (errno != ENOBUFS) { err = errno; break; }
            /* slab budget exhausted by datagrams still queued: this chunk's bursts are dropped
             * (h_gather_chunk queued nothing; the wait only orders the chunk's own reassembly
             * work before the next chunk reuses the pipe's buffers) */
            if ((rc = udpdk_gpu_pipe_wait(g, h_pipe_of(k)))) { err = -rc; break; }
            if (ad) h_arena_put(ad);
            if (af) h_arena_put(af);
            ad = af = NULL;
            __atomic_fetch_add(&g_udpdk.rx_nobufs, (uint64_t)nad + naf, __ATOMIC_RELAXED);
            continue;
        }
        if (nad + naf) { pend = (int)k; pnad = nad; pnaf = naf; }
        CPROF_T(t1); CPROF_ADD(6, t0, t1);
    }
#undef CK_ISSUE
    if (!err && pend >= 0) {
        if ((rc = udpdk_gpu_pipe_wait(g, h_pipe_of((uint32_t)pend)))) {
            err = -rc;
        } else {
            if (ad) atomic_store_explicit(&ad->refs, pnad, memory_order_relaxed);
            if (af) atomic_store_explicit(&af->refs, pnaf, memory_order_relaxed);
            struct h_pub P = {&A, ad, af, 0};
            h_pool_run(h_pub_job, &P);
            ad = af = NULL;
        }
    }
    if (err) {                                   /* nothing of ours left in flight */
        for (uint32_t k = 0; k < 3; k++) (void)udpdk_gpu_pipe_wait(g, h_pipe_of(k));
        if (ad) h_arena_put(ad);
        if (af) h_arena_put(af);
        errno = err;
        return -1;
    }
    if (stats_out) *stats_out = tot;
#ifdef UDPDK_POLL_PROFILE
    {   /* the first call (allocations) is left out */
        static int first = 1;
        if (first) memset(g_cprof, 0, sizeof(g_cprof));
        else g_cprof[7] += 1;
        first = 0;
    }
#endif
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
    PROF_T(p0);
    if (h_snapshot_refresh()) goto out;
    PROF_T(p1);
    const uint32_t lanes = g_udpdk.snap_lanes, maxfan = g_udpdk.snap_maxfan;
    if (g_udpdk.n_shards <= 1) {
        const int r = h_poll_chunked(frames, frames_bytes, offset, length, ptype, n, lanes, maxfan, stats_out);
        if (r <= 0) { ret = r; goto out; }
    }
    const uint64_t cap64 = (uint64_t)n * maxfan;
    const uint32_t cap = cap64 > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap64;
    if (h_grow_host((void **)&g_udpdk.rx_meta, &g_udpdk.rx_meta_cap, 4ull * n + 4) ||
        h_grow_host((void **)&g_udpdk.rx_loff, &g_udpdk.rx_loff_cap, 4ull * (lanes + 1)) ||
        h_grow_host((void **)&g_udpdk.rx_lpkt, &g_udpdk.rx_lpkt_cap, 4ull * cap + 4))
        goto out;
    uint32_t *meta = g_udpdk.rx_meta, *loff = g_udpdk.rx_loff, *lpkt = g_udpdk.rx_lpkt;
    udpdk_rx_stats_t st;
    const int sharded = g_udpdk.n_shards > 1;
    const struct h_sjob J = {frames, frames_bytes, offset, length, ptype, maxfan};
    udpdk_rx_batch_t staged;
    const uint32_t *meta_dev = NULL;
    if (sharded) {
        if (h_shards_rx(&J, n, lanes, meta, loff, lpkt, &st)) goto out;
    } else {
        if ((rc = udpdk_gpu_rx_host(g, frames, frames_bytes, offset, length, ptype, n, meta, loff, lpkt,
                                    cap, &st))) { errno = -rc; goto out; }
        if ((rc = udpdk_gpu_rx_host_batch(g, &staged, &meta_dev))) { errno = -rc; goto out; }
    }
    PROF_T(p2);
    udpdk_rx_batch_t rb;
    uint32_t nd = 0;
    const uint32_t nfrag = (uint32_t)st.counters[UDPDK_V_FRAG];
    if (sharded && nfrag) {
        /* every shard's FRAG frames, in arrival order, through the main context's table */
        udpdk_rx_batch_t fsub;
        const uint32_t *fmeta = NULL;
        /* (the sub-batch packs the FRAG frames back to back: disjoint, and the direct frames
         * are gathered from the shards' own staging) */
        if (h_frag_subbatch(&J, meta, n, nfrag, maxfan, &fsub, &fmeta) ||
            h_frag_pass(&fsub, fmeta, nfrag, lanes, maxfan, 1, &rb, &nd))
            goto out;
        for (uint32_t d = 0; d < nd; d++) g_udpdk.fr_org[d] = g_udpdk.fb_idx[g_udpdk.fr_org[d]];
    } else if (!sharded) {
        const int inplace = nfrag && h_desc_disjoint(offset, length, n, frames_bytes);
        if (h_frag_pass(&staged, meta_dev, nfrag, lanes, maxfan, inplace, &rb, &nd)) goto out;
    }
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
    struct h_adm A = {loff, lpkt, floff, flpkt, forg, length, lanes < UDPDK_MAX_SOCKETS ? lanes : UDPDK_MAX_SOCKETS, 0, {0}, n, 0};
    /* the lanes as the device returned them: offsets from 0, non-decreasing, within the entry
     * buffer, entries below n (pass 1) — never trusted blindly as host indices */
    int lanes_ok = loff[0] == 0u && D <= cap;
    for (uint32_t s = 0; lanes_ok && s < lanes; s++) lanes_ok = loff[s] <= loff[s + 1];
    if (!lanes_ok) { errno = EIO; goto out; }
    h_adm_split(&A, h_pool_parts());
    h_pool_run(h_adm_job, &A);                       /* pass 1: what each socket admits */
    if (atomic_load(&A.bad)) { errno = EIO; goto out; }
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
    /* direct payloads: the GPU gather, or, with [gpu] host_copy_min set, a host copy from the
     * caller's frames when the poll's datagrams carry at least that many payload bytes on average
     * (off by default: on three boxes the GPU gather + slab D2H took 58-62 ms per 1 M x 1500 B
     * poll against 54-85 ms for the host copy, which depends on the host's memory bandwidth) */
    const int hcopy = nad && g_udpdk.host_copy_min && offd >= (uint64_t)nad * g_udpdk.host_copy_min;
    if ((hcopy ? h_host_gather(frames, offset, length, g_udpdk.acc_d, g_udpdk.acc_do, nad, &ad)
               : sharded ? h_shards_gather(nad)
                         : h_gather(g, &g_udpdk.gb, &staged, g_udpdk.acc_d, g_udpdk.acc_do, nad, &ad)) ||
        (naf && h_gather(g, &g_udpdk.gb, &rb, g_udpdk.acc_f, g_udpdk.acc_fo, naf, &af))) {
        if (errno != ENOBUFS) goto out;
        /* slab budget exhausted by datagrams still queued: this poll's bursts are dropped */
        __atomic_fetch_add(&g_udpdk.rx_nobufs, (uint64_t)nad + naf, __ATOMIC_RELAXED);
        if (stats_out) *stats_out = st;
        ret = 0;
        goto out;
    }
    PROF_T(p5);
    if ((rc = udpdk_gpu_sync(g))) { errno = -rc; goto out; }
    PROF_T(p6);
    if (ad) atomic_store_explicit(&ad->refs, nad, memory_order_relaxed);
    if (af) atomic_store_explicit(&af->refs, naf, memory_order_relaxed);
    for (uint32_t k = 0; sharded && !hcopy && k < g_udpdk.n_shards; k++)
        if (g_udpdk.shard[k].arena)
            atomic_store_explicit(&g_udpdk.shard[k].arena->refs, g_udpdk.shard[k].nacc, memory_order_relaxed);
    /* publish: each socket's entries go to its ring in bulk enqueues, sockets over the pool */
    {
        struct h_pub P = {&A, ad, af, sharded && !hcopy};
        h_pool_run(h_pub_job, &P);
    }
    ad = af = NULL;
    for (uint32_t k = 0; sharded && k < g_udpdk.n_shards; k++) g_udpdk.shard[k].arena = NULL;
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
    for (uint32_t k = 0; k < g_udpdk.n_shards; k++) {
        if (g_udpdk.shard[k].arena) h_arena_put(g_udpdk.shard[k].arena);
        g_udpdk.shard[k].arena = NULL;
    }
    pthread_mutex_unlock(&g_udpdk.lock);
    return ret;
}
