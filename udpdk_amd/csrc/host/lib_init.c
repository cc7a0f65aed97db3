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

#include "host_state.h"

__attribute__((constructor)) static void h_lib_load(void)
{
    h_btable_reset();
    h_sockets_reset();
    g_udpdk.snap_version = UINT64_MAX;
    g_udpdk.gpu_max_frames = 1u << 20;
    g_udpdk.gpu_max_lanes = UDPDK_MAX_SOCKETS;
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
    int ret = -1;
    udpdk_rx_stats_t st;
    if (!meta || !loff || !lpkt) { errno = ENOMEM; goto out; }
    int rc = udpdk_gpu_rx_host(g_udpdk.gpu, frames, frames_bytes, offset, length, ptype, n, meta,
                               loff, lpkt, cap, &st);
    if (rc) { errno = -rc; goto out; }
    for (uint32_t s = 0; s < lanes && s < UDPDK_MAX_SOCKETS; s++) {
        const uint32_t a = loff[s], b = loff[s + 1];
        if (a == b || !g_udpdk.slots[s].used) continue;
        struct h_dgram *d = calloc(b - a, sizeof(*d));
        if (!d) { errno = ENOMEM; goto out; }
        uint32_t k = 0;
        for (uint32_t e = a; e < b; e++, k++) {
            const uint8_t *f = frames + offset[lpkt[e]];
            const uint32_t flen = length[lpkt[e]];
            /* payload bytes: min(data_len - 42, dgram_len - 8) as recvfrom computes them
             * (udpdk_syscall.c:438, :459-466, trimming Ethernet padding) */
            const uint16_t dl = (uint16_t)(((uint32_t)f[38] << 8) | f[39]);
            const uint16_t pl = (uint16_t)(dl - 8u);
            uint32_t plen = flen - 42u;
            if (plen > pl) plen = pl;
            d[k].len = plen;
            d[k].data = malloc(plen ? plen : 1);
            if (!d[k].data) { for (uint32_t z = 0; z < k; z++) free(d[z].data); free(d); errno = ENOMEM; goto out; }
            memcpy(d[k].data, f + 42, plen);
            memcpy(&d[k].src_ip, f + 26, 4);
            d[k].src_port = (uint32_t)f[34] | ((uint32_t)f[35] << 8);
        }
        if (h_ring_push_bulk(&g_udpdk.slots[s].rx, d, k)) {
            for (uint32_t z = 0; z < k; z++) free(d[z].data);   /* ring full: drop the batch */
        }
        free(d);
    }
    if (stats_out) *stats_out = st;
    ret = 0;
out:
    free(meta);
    free(loff);
    free(lpkt);
    return ret;
}
