/*
 * lib_init.c — udpdk_init / udpdk_interrupt / udpdk_cleanup, configuration, and the poller
 * thread with its ports (udpdk_port_attach, the built-in loopback port).
 *
 * udpdk_init follows udpdk_init.c:282-371 minus the DPDK bring-up: parse the .ini the same way
 * (udpdk_args.c:21-49, 122-163), then create the GPU context instead of forking a poller. The
 * poller itself is a thread started by udpdk_port_attach (poller_body, udpdk_poller.c:448-546,
 * against a port given as callbacks); its RX half is udpdk_poll_rx (rx_poll.c), its TX half
 * udpdk_tx_drain (tx_drain.c).
 */
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "host_state.h"

/* The [gpu] tunables' defaults: set at load and again by every udpdk_init that creates the
 * context, so one session's .ini never leaks into the next. */
static void h_config_defaults(void)
{
    g_udpdk.gpu_device = 0;
    g_udpdk.n_shards = 0;
    g_udpdk.dispatch_rss = 0;
    g_udpdk.rss_ready = 0;
    g_udpdk.poll_threads = 0;
    g_udpdk.host_copy_min = 0;         /* off: the GPU gather (tools/sock_tune.py) */
    g_udpdk.poll_chunk_mb = 128;       /* pipelined polls from 256 MB of frames (rx_poll.c) */
    g_udpdk.poll_chunk_min_avg = 1024; /* ... of 1 KiB frames on average */
    g_udpdk.gpu_max_frames = 1u << 20;
    g_udpdk.gpu_max_lanes = UDPDK_MAX_SOCKETS;
    g_udpdk.frag_buckets = 0x1000;     /* NUM_FLOWS_DEF, udpdk_constants.h:32 */
    g_udpdk.frag_entries = 16;         /* IP_FRAG_TBL_BUCKET_ENTRIES */
    g_udpdk.frag_max_dgram = 65515;
    g_udpdk.frag_ttl_ms = 1000;        /* MAX_FLOW_TTL = MS_PER_S */
    g_udpdk.frag_max_entries = 0;      /* NUM_FLOWS_MAX (rx_poll.c: h_frag_max_entries) */
    g_udpdk.frag_flags = 0;            /* RFC 1071 header checksum on reassembled datagrams */
    g_udpdk.arena_bytes_max = 4ull << 30;
    g_udpdk.arena_count_max = 1024;
    g_udpdk.port_spec[0] = g_udpdk.port_peer[0] = 0;
}

__attribute__((constructor)) static void h_lib_load(void)
{
    pthread_mutex_init(&g_udpdk.lock, NULL);
    pthread_mutex_init(&g_udpdk.tx_lock, NULL);
    pthread_mutex_init(&g_udpdk.arena_lock, NULL);
    g_udpdk.mtu = 1500;                /* IPV4_MTU_DEFAULT = RTE_ETHER_MTU */
    h_btable_reset();
    h_sockets_reset();
    g_udpdk.snap_version = UINT64_MAX;
    h_config_defaults();
}

static void h_lo_reset(void);

void udpdk_host_reset(void)
{
    udpdk_port_detach();
    h_lo_reset();
    pthread_mutex_lock(&g_udpdk.lock);
    pthread_mutex_lock(&g_udpdk.tx_lock);
    h_btable_reset();
    h_sockets_reset();
    pthread_mutex_unlock(&g_udpdk.tx_lock);
    atomic_store(&g_udpdk.interrupted, 0);
    g_udpdk.snap_version = UINT64_MAX;
    g_udpdk.mtu = 1500;
    pthread_mutex_unlock(&g_udpdk.lock);
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

/* "[gpu] devices = 0-3,5,5": the RX shard contexts, one per entry, in shard order (a device
 * may repeat: several contexts on one GPU). The first entry is also the main context's device.
 * Parsed into dev[H_MAX_DEVS]; returns the count, or -1. */
static int h_parse_device_list(const char *v, int *dev)
{
    uint32_t n = 0;
    const char *p = v;
    while (*p) {
        char *e;
        const long a = strtol(p, &e, 10);
        if (e == p || a < 0) return -1;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            if (e == p + 1 || b < a) return -1;
            p = e;
        }
        for (long d = a; d <= b; d++) {
            if (n == H_MAX_DEVS) return -1;
            dev[n++] = (int)d;
        }
        while (*p == ' ' || *p == '\t') p++;
        if (*p == ',') p++;
        else if (*p) return -1;
        while (*p == ' ' || *p == '\t') p++;
    }
    return n ? (int)n : -1;
}

static int h_parse_devices(const char *v)
{
    const int n = h_parse_device_list(v, g_udpdk.shard_dev);
    if (n < 0) return -1;
    g_udpdk.n_shards = (uint32_t)n;
    g_udpdk.gpu_device = g_udpdk.shard_dev[0];
    return 0;
}

/* The device plan udpdk_init would build from the config file, without touching a GPU: the
 * contexts in shard order ("[gpu] devices", two or more entries) or the one context of
 * "[gpu] device" (default 0). Every context of the plan binds its device (hipSetDevice) on each
 * C-ABI call, so each shard's pool thread allocates, copies and launches on its own GPU. */
int udpdk_shard_plan(const char *cfg_path, int *devices, int max)
{
    if (!cfg_path || max < 0 || (max && !devices)) return -EINVAL;
    FILE *f = fopen(cfg_path, "r");
    if (!f) return -ENOENT;
    char line[512], section[64] = "";
    /* the two keys tracked apart, as h_load_ini does: "devices" sets the shard list and the main
     * context's device; a later "device" moves only the main context's device */
    int dev[H_MAX_DEVS], n = 0, single = 0, rc = 0;
    while (fgets(line, sizeof(line), f)) {
        char *s = h_trim(line);
        if (!*s || *s == '#' || *s == ';') continue;
        if (*s == '[') {
            char *e = strchr(s, ']');
            if (!e) { rc = -EINVAL; break; }
            *e = 0;
            snprintf(section, sizeof(section), "%s", s + 1);
            continue;
        }
        char *eq = strchr(s, '=');
        if (!eq || strcmp(section, "gpu")) continue;
        *eq = 0;
        const char *k = h_trim(s), *v = h_trim(eq + 1);
        if (!strcmp(k, "device")) {
            single = atoi(v);
        } else if (!strcmp(k, "devices")) {
            n = h_parse_device_list(v, dev);
            if (n < 0) { rc = -EINVAL; break; }
            single = dev[0];
        }
    }
    fclose(f);
    if (rc) return rc;
    if (n < 2) {                        /* no shard list: the one context of gpu_device */
        n = 1;
        dev[0] = single;
    }
    for (int k = 0; k < n && k < max; k++) devices[k] = dev[k];
    return n;
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
        } else if (!strcmp(section, "port0") && !strcmp(k, "mtu")) {
            if (udpdk_config_mtu((uint32_t)strtoul(v, NULL, 0))) { rc = -1; break; }
        } else if (!strcmp(section, "gpu") && !strcmp(k, "device")) {
            g_udpdk.gpu_device = atoi(v);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "devices")) {
            if (h_parse_devices(v)) { rc = -1; break; }
        } else if (!strcmp(section, "gpu") && !strcmp(k, "dispatch")) {
            if (!strcmp(v, "rss")) g_udpdk.dispatch_rss = 1;
            else if (!strcmp(v, "contiguous")) g_udpdk.dispatch_rss = 0;
            else { rc = -1; break; }
        } else if (!strcmp(section, "gpu") && !strcmp(k, "max_frames")) {
            g_udpdk.gpu_max_frames = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "max_lanes")) {
            g_udpdk.gpu_max_lanes = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "poll_threads")) {
            g_udpdk.poll_threads = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "poll_chunk_mb")) {
            g_udpdk.poll_chunk_mb = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "poll_chunk_min_avg")) {
            g_udpdk.poll_chunk_min_avg = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "host_copy_min")) {
            g_udpdk.host_copy_min = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_buckets")) {
            g_udpdk.frag_buckets = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_bucket_entries")) {
            g_udpdk.frag_entries = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_max_dgram")) {
            g_udpdk.frag_max_dgram = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "frag_max_entries")) {
            g_udpdk.frag_max_entries = (uint32_t)strtoul(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "reasm_cksum")) {
            /* dpdk: the reassembled header's checksum left 0 as DPDK writes it (the reference's
             * "TODO must fix the IP header checksum", udpdk_poller.c:355-360); rfc1071 (default) */
            if (!strcmp(v, "dpdk")) g_udpdk.frag_flags |= UDPDK_FRAG_CKSUM_DPDK;
            else if (!strcmp(v, "rfc1071")) g_udpdk.frag_flags &= ~UDPDK_FRAG_CKSUM_DPDK;
            else { rc = -1; break; }
        } else if (!strcmp(section, "gpu") && !strcmp(k, "port")) {
            snprintf(g_udpdk.port_spec, sizeof(g_udpdk.port_spec), "%s", v);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "port_peer")) {
            snprintf(g_udpdk.port_peer, sizeof(g_udpdk.port_peer), "%s", v);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "slab_bytes_max")) {
            g_udpdk.arena_bytes_max = strtoull(v, NULL, 0);
        } else if (!strcmp(section, "gpu") && !strcmp(k, "slab_count_max")) {
            g_udpdk.arena_count_max = (uint32_t)strtoul(v, NULL, 0);
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
    if (!g_udpdk.gpu) h_config_defaults();
    if (h_load_ini(cfg)) { errno = EINVAL; return -1; }
    if (g_udpdk.gpu) return 0;
    int rc = udpdk_gpu_ctx_create(g_udpdk.gpu_device, g_udpdk.gpu_max_frames,
                                  g_udpdk.gpu_max_lanes, &g_udpdk.gpu);
    if (rc) { errno = rc == -ENODEV ? ENODEV : -rc; g_udpdk.gpu = NULL; return -1; }
    /* [gpu] devices with two or more entries: one RX shard context per entry (SURVEY.md §7 step
     * 8); a poll splits its batch into that many contiguous shards */
    if (g_udpdk.n_shards > 1) {
        for (uint32_t k = 0; k < g_udpdk.n_shards && !rc; k++) {
            g_udpdk.shard[k].device = g_udpdk.shard_dev[k];
            rc = udpdk_gpu_ctx_create(g_udpdk.shard_dev[k], g_udpdk.gpu_max_frames, g_udpdk.gpu_max_lanes,
                                      &g_udpdk.shard[k].g);
        }
        if (rc) {
            h_shards_destroy();
            udpdk_gpu_ctx_destroy(g_udpdk.gpu);
            g_udpdk.gpu = NULL;
            errno = rc == -ENODEV ? ENODEV : -rc;
            return -1;
        }
        if (g_udpdk.dispatch_rss && h_rss_setup()) {
            h_shards_destroy();
            udpdk_gpu_ctx_destroy(g_udpdk.gpu);
            g_udpdk.gpu = NULL;
            errno = EINVAL;
            return -1;
        }
    } else {
        g_udpdk.n_shards = 0;
    }
    g_udpdk.snap_version = UINT64_MAX;
    /* [gpu] port: start the poller thread on it now, as the reference forks its poller here
     * (udpdk_init.c:293, :362-368), so an unmodified application's sendto / recvfrom move
     * packets without further calls */
    if (g_udpdk.port_spec[0]) {
        udpdk_port_ops_t ops;
        int prc;
        if (!strncmp(g_udpdk.port_spec, "udp:", 4))
            prc = h_wire_open(g_udpdk.port_spec + 4, g_udpdk.port_peer, &ops);
        else if (!strcmp(g_udpdk.port_spec, "loopback"))
            prc = udpdk_port_loopback(&ops);
        else
            prc = (errno = EINVAL, -1);
        if (prc || udpdk_port_attach(&ops)) {
            const int e = errno;
            h_wire_close();
            udpdk_cleanup();
            errno = e;
            return -1;
        }
    }
    return 0;
}

int udpdk_shard_frames(uint32_t *frames, int max)
{
    const int n = g_udpdk.n_shards > 1 ? (int)g_udpdk.n_shards : 0;
    for (int k = 0; k < n && k < max; k++) frames[k] = g_udpdk.shard[k].n;
    return n;
}

int udpdk_shard_devices(int *devices, int max)
{
    const int n = g_udpdk.n_shards > 1 ? (int)g_udpdk.n_shards : (g_udpdk.gpu ? 1 : 0);
    for (int k = 0; devices && k < n && k < max; k++)
        devices[k] = g_udpdk.n_shards > 1 ? g_udpdk.shard[k].device : g_udpdk.gpu_device;
    return n;
}

void udpdk_interrupt(int signum)
{
    (void)signum;
    atomic_store(&g_udpdk.interrupted, 1);
}

void udpdk_cleanup(void)
{
    udpdk_port_detach();
    h_wire_close();
    h_lo_reset();
    udpdk_poll_profile_dump();
    h_pool_stop();
    for (int s = 0; s < UDPDK_MAX_SOCKETS; s++)
        if (g_udpdk.slots[s].used) udpdk_close(s);
    h_tx_reset();
    h_rx_buffers_free();
    h_tx_buffers_free();
    h_arenas_free_all();
    g_udpdk.frag_ready = 0;
    h_shards_destroy();
    udpdk_gpu_ctx_destroy(g_udpdk.gpu);
    g_udpdk.gpu = NULL;
    g_udpdk.snap_version = UINT64_MAX;
}

udpdk_gpu_ctx *udpdk_gpu_context(void) { return g_udpdk.gpu; }

int udpdk_config_mtu(uint32_t mtu)
{
    if (mtu < 68u || mtu > 9000u || (mtu - 20u) % 8u) { errno = EINVAL; return -1; }
    g_udpdk.mtu = mtu;
    return 0;
}

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

/* ---- the poller thread (poller_body, udpdk_poller.c:448-546) ------------------------------- */
static void *h_poller_main(void *arg)
{
    (void)arg;
    const udpdk_port_ops_t *P = &g_udpdk.port;
    const uint32_t nb = P->batch_frames ? P->batch_frames : 4096;
    const uint64_t cap = (uint64_t)nb * 2048 + UDPDK_GPU_FRAMES_TAILROOM;
    /* the RX buffer is pinned (a NIC's DMA target): udpdk_poll_rx's H2D reads it directly */
    uint8_t *rx = NULL, *tx = malloc(cap);
    if (udpdk_gpu_host_alloc(g_udpdk.gpu, cap, (void **)&rx)) rx = NULL;
    uint32_t *roff = malloc(4ull * nb), *toff = malloc(4ull * nb);
    uint16_t *rlen = malloc(2ull * nb), *tlen = malloc(2ull * nb);
    while (rx && tx && roff && toff && rlen && tlen &&
           atomic_load_explicit(&g_udpdk.poller_run, memory_order_acquire)) {
        int idle = 1;
        /* TX half first, as the poller loop does */
        uint32_t nt = 0;
        if (P->tx_burst && udpdk_tx_pending() && udpdk_tx_drain(tx, cap, toff, tlen, nb, &nt) == 0 && nt) {
            P->tx_burst(P->user, tx, toff, tlen, nt);
            idle = 0;
        }
        if (P->rx_burst) {
            const uint32_t n = P->rx_burst(P->user, rx, cap - UDPDK_GPU_FRAMES_TAILROOM, roff, rlen, nb);
            if (n) {
                uint64_t fb = 0;
                for (uint32_t i = 0; i < n; i++)
                    if ((uint64_t)roff[i] + rlen[i] > fb) fb = (uint64_t)roff[i] + rlen[i];
                udpdk_poll_rx(rx, fb, roff, rlen, NULL, n, NULL);
                idle = 0;
            }
        }
        if (idle) sched_yield();
    }
    if (rx) udpdk_gpu_host_free(g_udpdk.gpu, rx);
    free(tx); free(roff); free(toff); free(rlen); free(tlen);
    return NULL;
}

int udpdk_port_attach(const udpdk_port_ops_t *ops)
{
    if (!ops || (!ops->rx_burst && !ops->tx_burst)) { errno = EINVAL; return -1; }
    if (!g_udpdk.gpu) { errno = ENODEV; return -1; }
    if (g_udpdk.poller_started) { errno = EBUSY; return -1; }
    g_udpdk.port = *ops;
    atomic_store(&g_udpdk.poller_run, 1);
    if (pthread_create(&g_udpdk.poller, NULL, h_poller_main, NULL)) {
        atomic_store(&g_udpdk.poller_run, 0);
        errno = EAGAIN;
        return -1;
    }
    g_udpdk.poller_started = 1;
    return 0;
}

int udpdk_port_detach(void)
{
    if (!g_udpdk.poller_started) return 0;
    atomic_store(&g_udpdk.poller_run, 0);
    pthread_join(g_udpdk.poller, NULL);
    g_udpdk.poller_started = 0;
    return 0;
}

/* Loopback port: a FIFO of frames; tx_burst appends copies, rx_burst hands them back. */
static struct {
    pthread_mutex_t mu;
    uint8_t *buf;
    uint64_t bytes, cap, head;
    uint32_t *len;                /* frame lengths in FIFO order */
    uint64_t n, ncap, nhead;
} h_lo = {PTHREAD_MUTEX_INITIALIZER, NULL, 0, 0, 0, NULL, 0, 0, 0};

/* Empty the FIFO: frames of an earlier session never reach a later one's RX. */
static void h_lo_reset(void)
{
    pthread_mutex_lock(&h_lo.mu);
    h_lo.bytes = h_lo.head = 0;
    h_lo.n = h_lo.nhead = 0;
    pthread_mutex_unlock(&h_lo.mu);
}

static void h_lo_tx(void *user, const uint8_t *frames, const uint32_t *off, const uint16_t *len, uint32_t n)
{
    (void)user;
    pthread_mutex_lock(&h_lo.mu);
    for (uint32_t i = 0; i < n; i++) {
        if (h_lo.bytes + len[i] > h_lo.cap) {
            const uint64_t live = h_lo.bytes - h_lo.head;        /* compact, then grow */
            memmove(h_lo.buf, h_lo.buf + h_lo.head, live);
            h_lo.bytes = live;
            h_lo.head = 0;
            if (h_lo.bytes + len[i] > h_lo.cap) {
                uint64_t nc = h_lo.cap ? 2 * h_lo.cap : (1u << 20);
                while (nc < h_lo.bytes + len[i]) nc *= 2;
                uint8_t *nbuf = realloc(h_lo.buf, nc);
                if (!nbuf) break;
                h_lo.buf = nbuf;
                h_lo.cap = nc;
            }
        }
        if (h_lo.n == h_lo.ncap) {
            const uint64_t live = h_lo.n - h_lo.nhead;
            memmove(h_lo.len, h_lo.len + h_lo.nhead, live * sizeof(uint32_t));
            h_lo.n = live;
            h_lo.nhead = 0;
            if (h_lo.n == h_lo.ncap) {
                const uint64_t nc = h_lo.ncap ? 2 * h_lo.ncap : 4096;
                uint32_t *nl = realloc(h_lo.len, nc * sizeof(uint32_t));
                if (!nl) break;
                h_lo.len = nl;
                h_lo.ncap = nc;
            }
        }
        memcpy(h_lo.buf + h_lo.bytes, frames + off[i], len[i]);
        h_lo.bytes += len[i];
        h_lo.len[h_lo.n++] = len[i];
    }
    pthread_mutex_unlock(&h_lo.mu);
}

static uint32_t h_lo_rx(void *user, uint8_t *frames, uint64_t cap, uint32_t *off, uint16_t *len, uint32_t max)
{
    (void)user;
    pthread_mutex_lock(&h_lo.mu);
    uint32_t k = 0;
    uint64_t pos = 0;
    while (k < max && h_lo.nhead < h_lo.n && pos + h_lo.len[h_lo.nhead] <= cap) {
        const uint32_t l = h_lo.len[h_lo.nhead++];
        memcpy(frames + pos, h_lo.buf + h_lo.head, l);
        h_lo.head += l;
        off[k] = (uint32_t)pos;
        len[k] = (uint16_t)l;
        pos += l;
        k++;
    }
    pthread_mutex_unlock(&h_lo.mu);
    return k;
}

int udpdk_port_loopback(udpdk_port_ops_t *ops)
{
    if (!ops) { errno = EINVAL; return -1; }
    memset(ops, 0, sizeof(*ops));
    h_lo_reset();
    ops->rx_burst = h_lo_rx;
    ops->tx_burst = h_lo_tx;
    return 0;
}
