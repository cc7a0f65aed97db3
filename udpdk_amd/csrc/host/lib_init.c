/*
 * lib_init.c — udpdk_init / udpdk_interrupt / udpdk_cleanup, configuration, and the GPU poller
 * entry point udpdk_poll_rx.
 *
 * udpdk_init follows udpdk_init.c:282-371 minus the DPDK bring-up: parse the .ini the same way
 * (udpdk_args.c:21-49, 122-163), then create the GPU context instead of forking a poller.
 * udpdk_poll_rx stands in for one turn of poller_body's RX half (udpdk_poller.c:516-545): the
 * frames are classified and demultiplexed on the GPU, then each socket's deliveries are appended
 * to its RX ring in arrival order, all-or-nothing per socket (flush_rx_queue, :274-292).
 */
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "host_state.h"

__attribute__((constructor)) static void h_lib_load(void)
{
    h_btable_reset();
    h_sockets_reset();
    g_udpdk.snap_version = UINT64_MAX;
    g_udpdk.gpu_max_frames = 1u << 20;
    g_udpdk.gpu_max_lanes = UDPDK_MAX_SOCKETS;
    g_udpdk.frag_buckets = 0x1000;     /* NUM_FLOWS_DEF, udpdk_constants.h:32 */
    g_udpdk.frag_entries = 16;         /* IP_FRAG_TBL_BUCKET_ENTRIES */
    g_udpdk.frag_max_dgram = 65515;
    g_udpdk.frag_ttl_ms = 1000;        /* MAX_FLOW_TTL = MS_PER_S */
}

void udpdk_host_reset(void)
{
    h_btable_reset();
    h_sockets_reset();
    g_udpdk.interrupted = 0;
    g_udpdk.txq_bytes = 0;
    g_udpdk.txq_n = 0;
    g_udpdk.snap_version = UINT64_MAX;
}

static int h_parse_mac(const char *v, uint8_t mac[6])
{
    unsigned b[6];
    if (sscanf(v, "%x:%x:%x:%x:%x:%x", &b[0], &b[1], &b[2], &b[3], &b[4], &b[5]) != 6) return -1;
    for (int i = 0; i < 6; i++) {
        if (b[i] > 0xFF) return -1;
        mac[i] = (uint8_t)b[i];
    }
    return 0;
}

static char *h_trim(char *s)
{
    while (isspace((unsigned char)*s)) s++;
    char *e = s + strlen(s);
    while (e > s && isspace((unsigned char)e[-1])) *--e = 0;
    return s;
}

/* Minimal INI reader for the keys the reference understands plus a [gpu] section. */
static int h_load_ini(const char *path)
{
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char line[512], section[64] = "";
    int rc = 0;
    while (fgets(line, sizeof(line), f)) {
        char *s = h_trim(line);
        if (!*s || *s == '#' || *s == ';') continue;
        if (*s == '[') {
            char *e = strchr(s, ']');
            if (!e) { rc = -1; break; }
            *e = 0;
            snprintf(section, sizeof(section), "%s", s + 1);
            continue;
        }
        char *eq = strchr(s, '=');
        if (!eq) { rc = -1; break; }
        *eq = 0;
        const char *k = h_trim(s), *v = h_trim(eq + 1);
        if (!strcmp(section, "port0") && !strcmp(k, "mac_addr")) {
            if (h_parse_mac(v, g_udpdk.src_mac)) { rc = -1; break; }
        } else if (!strcmp(section, "port0") && !strcmp(k, "ip_addr")) {
            g_udpdk.src_ip = inet_addr(v);
        } else if (!strcmp(section, "port0_dst") && !strcmp(k, "mac_addr")) {
            if (h_parse_mac(v, g_udpdk.dst_mac)) { rc = -1; break; }
        } else if (!strcmp(section, "gpu") && !strcmp(k, "device")) {
            g_udpdk.gpu_device = atoi(v);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "max_frames")) {
            g_udpdk.gpu_max_frames = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "max_lanes")) {
            g_udpdk.gpu_max_lanes = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_buckets")) {
            g_udpdk.frag_buckets = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_bucket_entries")) {
            g_udpdk.frag_entries = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_max_dgram")) {
            g_udpdk.frag_max_dgram = (uint32_t)strtoul(v, NULL, 0);
        }
        /* [dpdk] lcores / n_mem_channels configure EAL, which does not exist here */
    }
    fclose(f);
    return rc;
}

int udpdk_init(int argc, char *argv[])
{
    const char *cfg = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--")) break;
        if (!strcmp(argv[i], "-c") && i + 1 < argc) cfg = argv[++i];
        else if (!strncmp(argv[i], "-c", 2) && argv[i][2]) cfg = argv[i] + 2;
    }
    if (!cfg) { errno = EINVAL; return -1; }       /* config file is mandatory (args.c:150-155) */
    if (h_load_ini(cfg)) { errno = EINVAL; return -1; }
    if (g_udpdk.gpu) return 0;
    const int rc = udpdk_gpu_ctx_create(g_udpdk.gpu_device, g_udpdk.gpu_max_frames,
                                        g_udpdk.gpu_max_lanes, &g_udpdk.gpu);
    if (rc) { errno = rc == -ENODEV ? ENODEV : -rc; g_udpdk.gpu = NULL; return -1; }
    g_udpdk.snap_version = UINT64_MAX;
    return 0;
}

void udpdk_interrupt(int signum)
{
    (void)signum;
    g_udpdk.interrupted = 1;
}

void udpdk_cleanup(void)
{
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++)
        if (g_udpdk.slots[s].used) udpdk_close(s);
    void **dev[] = {&g_udpdk.fd_frames, &g_udpdk.fd_offset, &g_udpdk.fd_length, &g_udpdk.fd_meta,
                    &g_udpdk.fd_meta2, &g_udpdk.fd_loff2, &g_udpdk.fd_lpkt2};
    for (unsigned k = 0; k < sizeof(dev) / sizeof(dev[0]); k++) {
        if (*dev[k] && g_udpdk.gpu) udpdk_gpu_free(g_udpdk.gpu, *dev[k]);
        *dev[k] = NULL;
    }
    g_udpdk.fd_frames_cap = 0;
    g_udpdk.fd_n_cap = 0;
    g_udpdk.frag_ready = 0;
    udpdk_gpu_ctx_destroy(g_udpdk.gpu);
    g_udpdk.gpu = NULL;
    free(g_udpdk.txq);
    free(g_udpdk.txq_len);
    g_udpdk.txq = NULL;
    g_udpdk.txq_len = NULL;
    g_udpdk.txq_bytes = g_udpdk.txq_cap = 0;
    g_udpdk.txq_n = g_udpdk.txq_ncap = 0;
    g_udpdk.snap_version = UINT64_MAX;
}

udpdk_gpu_ctx *udpdk_gpu_context(void) { return g_udpdk.gpu; }

int udpdk_config_set(const uint8_t src_mac[6], const uint8_t dst_mac[6], uint32_t src_ip)
{
    if (!src_mac || !dst_mac) { errno = EINVAL; return -1; }
    memcpy(g_udpdk.src_mac, src_mac, 6);
    memcpy(g_udpdk.dst_mac, dst_mac, 6);
    g_udpdk.src_ip = src_ip;
    return 0;
}

int udpdk_config_get(uint8_t src_mac[6], uint8_t dst_mac[6], uint32_t *src_ip)
{
    if (src_mac) memcpy(src_mac, g_udpdk.src_mac, 6);
    if (dst_mac) memcpy(dst_mac, g_udpdk.dst_mac, 6);
    if (src_ip) *src_ip = g_udpdk.src_ip;
    return 0;
}

void udpdk_dump_payload(const char *payload, int len)
{
    const unsigned char *p = (const unsigned char *)payload;
    printf("Dumping payload [len = %d]:\n", len);
    for (int i = 0; i < len; i += 16) {
        char hex[16 * 3 + 1] = {0}, asc[17] = {0};
        int n = len - i < 16 ? len - i : 16;
        for (int j = 0; j < n; j++) {
            snprintf(hex + 3 * j, 4, "%02x ", p[i + j]);
            asc[j] = isprint(p[i + j]) ? (char)p[i + j] : '.';
        }
        printf("%5d: %-48s%s\n", i, hex, asc);
    }
}

/* recvfrom's payload rule (udpdk_syscall.c:438, :459-466): min(data_len - 42, dgram_len - 8)
 * bytes from frame byte 42 (Ethernet padding trimmed), source address from the headers. */
static int h_make_dgram(const uint8_t *f, uint32_t flen, struct h_dgram *d)
{
    const uint16_t dl = (uint16_t)(((uint32_t)f[38] << 8) | f[39]);
    const uint16_t pl = (uint16_t)(dl - 8u);
    uint32_t plen = flen - 42u;
    if (plen > pl) plen = pl;
    d->len = plen;
    d->data = malloc(plen ? plen : 1);
    if (!d->data) return -1;
    memcpy(d->data, f + 42, plen);
    memcpy(&d->src_ip, f + 26, 4);
    d->src_port = (uint32_t)f[34] | ((uint32_t)f[35] << 8);
    return 0;
}

static uint64_t h_now_ms(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000u + (uint64_t)ts.tv_nsec / 1000000u;
}

static int h_grow_dev(void **p, uint64_t *cap, uint64_t need)
{
    if (*p && *cap >= need) return 0;
    if (*p) udpdk_gpu_free(g_udpdk.gpu, *p);
    *p = NULL;
    *cap = 0;
    const int rc = udpdk_gpu_alloc(g_udpdk.gpu, need ? need : 16, p);
    if (rc) { errno = -rc; return -1; }
    *cap = need;
    return 0;
}

/* The batch's FRAG frames (udpdk_poller.c:338-361) through the device reassembly table, then the
 * completed datagrams through the demux. Out: per-lane delivery ranges f_off[lanes + 1], each
 * delivery's arrival index (that of the fragment that completed its datagram: where the
 * reference delivers it) and its payload. Nothing is allocated when there is no datagram. */
static int h_frag_pass(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                       const uint16_t *length, const uint32_t *meta, uint32_t n, uint32_t lanes,
                       uint32_t maxfan, uint32_t **f_off, uint32_t **f_idx, struct h_dgram **f_d)
{
    *f_off = NULL; *f_idx = NULL; *f_d = NULL;
    uint32_t nfrag = 0;
    for (uint32_t i = 0; i < n; i++) nfrag += (meta[i] & 0xFu) == UDPDK_V_FRAG;
    if (!nfrag) return 0;
    udpdk_gpu_ctx *g = g_udpdk.gpu;
    int rc;
    if (!g_udpdk.frag_ready) {
        udpdk_frag_table_cfg_t fc = {g_udpdk.frag_buckets, g_udpdk.frag_entries, g_udpdk.frag_ttl_ms,
                                     g_udpdk.frag_max_dgram};
        rc = udpdk_gpu_frag_table_create(g, &fc);
        if (rc) { errno = -rc; return -1; }
        g_udpdk.frag_ready = 1;
    }
    if (h_grow_dev(&g_udpdk.fd_frames, &g_udpdk.fd_frames_cap, frames_bytes + UDPDK_GPU_FRAMES_TAILROOM)) return -1;
    if (n > g_udpdk.fd_n_cap) {
        uint64_t c0 = 0, c1 = 0, c2 = 0;
        if (h_grow_dev(&g_udpdk.fd_offset, &c0, 4ull * n) || h_grow_dev(&g_udpdk.fd_length, &c1, 2ull * n) ||
            h_grow_dev(&g_udpdk.fd_meta, &c2, 4ull * n))
            return -1;
        g_udpdk.fd_n_cap = n;
    }
    if ((rc = udpdk_gpu_h2d(g, g_udpdk.fd_frames, frames, frames_bytes)) ||
        (rc = udpdk_gpu_h2d(g, g_udpdk.fd_offset, offset, 4ull * n)) ||
        (rc = udpdk_gpu_h2d(g, g_udpdk.fd_length, length, 2ull * n)) ||
        (rc = udpdk_gpu_h2d(g, g_udpdk.fd_meta, meta, 4ull * n))) {
        errno = -rc;
        return -1;
    }
    udpdk_rx_batch_t b = {g_udpdk.fd_frames, frames_bytes, g_udpdk.fd_offset, g_udpdk.fd_length, NULL, n};
    udpdk_reasm_out_t ro;
    if ((rc = udpdk_gpu_rx_reassemble(g, &b, g_udpdk.fd_meta, h_now_ms(), &ro))) { errno = -rc; return -1; }
    const uint32_t C = ro.batch.n;
    if (!C) return 0;
    const uint64_t cap64 = (uint64_t)C * maxfan;
    const uint32_t cap = cap64 > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap64;
    uint64_t m0 = 0, m1 = 0, m2 = 0;
    if (h_grow_dev(&g_udpdk.fd_meta2, &m0, 4ull * C) || h_grow_dev(&g_udpdk.fd_loff2, &m1, 4ull * (lanes + 1)) ||
        h_grow_dev(&g_udpdk.fd_lpkt2, &m2, 4ull * cap))
        return -1;
    udpdk_rx_out_t o2 = {g_udpdk.fd_meta2, g_udpdk.fd_loff2, g_udpdk.fd_lpkt2, cap};
    udpdk_rx_stats_t st2;
    if ((rc = udpdk_gpu_rx(g, &ro.batch, &o2))) { errno = -rc; return -1; }
    if ((rc = udpdk_gpu_rx_stats(g, &st2))) { errno = -rc; return -1; }
    const uint32_t D = st2.deliveries;
    uint32_t *loff = malloc(4ull * (lanes + 1)), *lpkt = malloc(4ull * (D + 1));
    uint32_t *org = malloc(4ull * C), *roff = malloc(4ull * C);
    uint16_t *rlen = malloc(2ull * C);
    uint8_t *rfr = malloc(ro.batch.frames_bytes + 1);
    uint32_t *idx = malloc(4ull * (D + 1));
    struct h_dgram *dg = calloc(D + 1, sizeof(*dg));
    int ret = -1;
    if (!loff || !lpkt || !org || !roff || !rlen || !rfr || !idx || !dg) { errno = ENOMEM; goto out; }
    if ((rc = udpdk_gpu_d2h(g, loff, g_udpdk.fd_loff2, 4ull * (lanes + 1))) ||
        (rc = udpdk_gpu_d2h(g, lpkt, g_udpdk.fd_lpkt2, 4ull * D)) ||
        (rc = udpdk_gpu_d2h(g, org, ro.origin_dev, 4ull * C)) ||
        (rc = udpdk_gpu_d2h(g, roff, ro.batch.offset_dev, 4ull * C)) ||
        (rc = udpdk_gpu_d2h(g, rlen, ro.batch.length_dev, 2ull * C)) ||
        (rc = udpdk_gpu_d2h(g, rfr, ro.batch.frames_dev, ro.batch.frames_bytes)) ||
        (rc = udpdk_gpu_sync(g))) {
        errno = -rc;
        goto out;
    }
    for (uint32_t e = 0; e < D; e++) {
        const uint32_t r = lpkt[e];
        idx[e] = org[r];
        if (h_make_dgram(rfr + roff[r], rlen[r], &dg[e])) {
            for (uint32_t z = 0; z < e; z++) free(dg[z].data);
            errno = ENOMEM;
            goto out;
        }
    }
    *f_off = loff; loff = NULL;
    *f_idx = idx; idx = NULL;
    *f_d = dg; dg = NULL;
    ret = 0;
out:
    free(loff); free(lpkt); free(org); free(roff); free(rlen); free(rfr); free(idx); free(dg);
    return ret;
}

int udpdk_poll_rx(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                  const uint16_t *length, const uint32_t *ptype, uint32_t n,
                  udpdk_rx_stats_t *stats_out)
{
    if (!g_udpdk.gpu) { errno = ENODEV; return -1; }
    if (n && (!frames || !offset || !length)) { errno = EINVAL; return -1; }
    if (g_udpdk.snap_version != g_udpdk.version) {
        udpdk_bind_snapshot_t snap;
        if (udpdk_btable_snapshot(&snap, 0)) return -1;
        const int rc = udpdk_gpu_bind_snapshot_upload(g_udpdk.gpu, &snap);
        if (rc) { errno = -rc; return -1; }
        g_udpdk.snap_version = g_udpdk.version;
    }
    udpdk_bind_snapshot_t cur;
    if (udpdk_btable_snapshot(&cur, 0)) return -1;
    const uint32_t lanes = cur.n_lanes;
    uint32_t maxfan = 1;
    for (uint32_t p = 0; p < 65536; p++)
        if (cur.port_count[p] > maxfan) maxfan = cur.port_count[p];
    const uint64_t cap64 = (uint64_t)n * maxfan;
    const uint32_t cap = cap64 > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)cap64;
    uint32_t *meta = malloc(((size_t)n + 1) * 4);
    uint32_t *loff = malloc(((size_t)lanes + 1) * 4);
    uint32_t *lpkt = malloc(((size_t)cap + 1) * 4);
    uint32_t *f_off = NULL, *f_idx = NULL;
    struct h_dgram *f_d = NULL;
    int ret = -1;
    udpdk_rx_stats_t st;
    if (!meta || !loff || !lpkt) { errno = ENOMEM; goto out; }
    int rc = udpdk_gpu_rx_host(g_udpdk.gpu, frames, frames_bytes, offset, length, ptype, n, meta,
                               loff, lpkt, cap, &st);
    if (rc) { errno = -rc; goto out; }
    if (h_frag_pass(frames, frames_bytes, offset, length, meta, n, lanes, maxfan, &f_off, &f_idx, &f_d))
        goto out;
    for (uint32_t s = 0; s < lanes && s < UDPDK_MAX_SOCKETS; s++) {
        const uint32_t a = loff[s], b = loff[s + 1];
        const uint32_t fa = f_off ? f_off[s] : 0u, fb = f_off ? f_off[s + 1] : 0u;
        if (a == b && fa == fb) continue;
        if (!g_udpdk.slots[s].used) {
            for (uint32_t e = fa; e < fb; e++) { free(f_d[e].data); f_d[e].data = NULL; }
            continue;
        }
        const uint32_t total = (b - a) + (fb - fa);
        struct h_dgram *d = calloc(total, sizeof(*d));
        if (!d) { errno = ENOMEM; goto out; }
        /* direct deliveries (frame index) and reassembled ones (index of the completing
         * fragment) merged in arrival order: the order the reference's rings receive them */
        uint32_t k = 0, e = a, q = fa;
        while (e < b || q < fb) {
            if (q >= fb || (e < b && lpkt[e] < f_idx[q])) {
                if (h_make_dgram(frames + offset[lpkt[e]], length[lpkt[e]], &d[k])) {
                    for (uint32_t z = 0; z < k; z++) free(d[z].data);
                    free(d);
                    errno = ENOMEM;
                    goto out;
                }
                e++;
            } else {
                d[k] = f_d[q];
                f_d[q].data = NULL;
                q++;
            }
            k++;
        }
        if (h_ring_push_bulk(&g_udpdk.slots[s].rx, d, k)) {
            for (uint32_t z = 0; z < k; z++) free(d[z].data);   /* ring full: drop the batch */
        }
        free(d);
    }
    if (stats_out) *stats_out = st;
    ret = 0;
out:
    if (f_d && f_off)
        for (uint32_t e = 0; e < f_off[lanes]; e++) free(f_d[e].data);
    free(f_off);
    free(f_idx);
    free(f_d);
    free(meta);
    free(loff);
    free(lpkt);
    return ret;
}
