/*
 * bench_sock.c — the reference-API path end to end: frames in host memory ->
 * udpdk_poll_rx (pinned staging, H2D, GPU classify/demux, GPU payload gather into pinned slabs,
 * D2H, ring admission) -> udpdk_recvfrom on every socket until each ring is empty, written
 * against include/udpdk_api.h exactly as an application of the reference would be.
 *
 *   bench_sock <ini> <n_frames> <frame_bytes | 0 = IMIX 64/594/1500 7:4:1> <n_sockets> <reps>
 *
 * Sockets 0..S-1 are bound ANY to ports 10000..10000+S-1; frame i goes to port 10000 + i % S
 * (uniform), so each ring receives n / S datagrams per poll (n / S must stay <= 2047, the ring).
 * Prints one JSON object: poll and recvfrom time per batch, datagrams/s of each and end to end
 * (the two one after the other on one thread), then the reference's own arrangement (a poller
 * running beside the application, udpdk_poller.c:443-446 vs the app's recvfrom loop): a poller
 * thread polls batch k + 1 while the application thread drains batch k, at most two batches in
 * the rings (the first 1023 x S frames: <= 1023 datagrams per socket per batch, two batches fit a
 * 2047-entry ring), and the rate is
 * the datagrams the application received over the wall time of all reps ("overlap_mdgram_s").
 * "host_copy_gbps": this box's single-thread copy rate out of pinned memory (64 KiB memcpys from
 * a buffer of >= 256 MiB into one 64 KiB buffer): the bound of the recvfrom loop, which is one
 * memcpy per datagram on one thread. Boxes differ here by up to 2x, so recv_mdgram_s is read
 * against it: "recv_over_copy" = the loop's payload bytes per second over that rate.
 */
#include <arpa/inet.h>
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "udpdk_api.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint16_t csum_fold(uint32_t s)
{
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)s;
}

/* One Eth/IPv4/UDP frame of len bytes to dst port (host order), valid IPv4 checksum, UDP
 * checksum 0 (as the reference sends). */
static void make_frame(uint8_t *f, uint32_t len, uint16_t dport, uint32_t seq)
{
    static const uint8_t mac[12] = {0x68, 0x05, 0xca, 0x95, 0xf8, 0xec, 0x68, 0x05, 0xca, 0x95, 0xfa, 0x64};
    memcpy(f, mac, 12);
    f[12] = 0x08; f[13] = 0x00;
    uint8_t *ip = f + 14;
    memset(ip, 0, 20);
    ip[0] = 0x45; ip[8] = 64; ip[9] = 17;
    const uint16_t tl = (uint16_t)(len - 14);
    ip[2] = (uint8_t)(tl >> 8); ip[3] = (uint8_t)tl;
    ip[4] = (uint8_t)(seq >> 8); ip[5] = (uint8_t)seq;
    const uint32_t src = inet_addr("172.31.100.2"), dst = inet_addr("172.31.100.1");
    memcpy(ip + 12, &src, 4);
    memcpy(ip + 16, &dst, 4);
    uint32_t s = 0;
    for (int i = 0; i < 20; i += 2) s += ((uint32_t)ip[i] << 8) | ip[i + 1];
    const uint16_t c = (uint16_t)~csum_fold(s);
    ip[10] = (uint8_t)(c >> 8); ip[11] = (uint8_t)c;
    uint8_t *u = f + 34;
    u[0] = 0x27; u[1] = 0x10;                                   /* 10000 */
    u[2] = (uint8_t)(dport >> 8); u[3] = (uint8_t)dport;
    const uint16_t ul = (uint16_t)(len - 34);
    u[4] = (uint8_t)(ul >> 8); u[5] = (uint8_t)ul;
    u[6] = u[7] = 0;
    for (uint32_t i = 42; i < len; i++) f[i] = (uint8_t)(seq * 31u + i);
}

struct poller {
    const uint8_t *fr;
    uint64_t bytes;
    const uint32_t *off;
    const uint16_t *len;
    uint32_t n;
    int reps;
    atomic_int posted;       /* batches admitted to the rings */
    atomic_int consumed;     /* batches the application drained */
    int err;
};

static void *poller_main(void *arg)
{
    struct poller *P = arg;
    for (int r = 0; r < P->reps; r++) {
        while (atomic_load(&P->consumed) < r - 1) ;          /* at most two batches in the rings */
        udpdk_rx_stats_t st;
        if (udpdk_poll_rx(P->fr, P->bytes, P->off, P->len, NULL, P->n, &st) < 0) {
            P->err = errno;
            atomic_store(&P->posted, P->reps + 1);
            return NULL;
        }
        atomic_store(&P->posted, r + 1);
    }
    return NULL;
}

/* a run that stops receiving (a burst dropped somewhere) ends with EINTR instead of spinning */
static void *watchdog_main(void *arg)
{
    sleep(*(unsigned *)arg);
    udpdk_interrupt(2);
    return NULL;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s <ini> <n_frames> <frame_bytes|0> <n_sockets> <reps>\n", argv[0]);
        return 2;
    }
    const uint32_t n = (uint32_t)atoi(argv[2]), fsz = (uint32_t)atoi(argv[3]);
    const int S = atoi(argv[4]), reps = atoi(argv[5]);
    char *iargv[] = {argv[0], "-c", argv[1], NULL};
    if (udpdk_init(3, iargv) < 0) { perror("udpdk_init"); return 1; }
    for (int s = 0; s < S; s++) {
        const int fd = udpdk_socket(AF_INET, SOCK_DGRAM, 0);
        struct sockaddr_in a;
        memset(&a, 0, sizeof(a));
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)(10000 + s));
        a.sin_addr.s_addr = INADDR_ANY;
        if (fd != s || udpdk_bind(fd, (struct sockaddr *)&a, sizeof(a)) < 0) { perror("bind"); return 1; }
    }
    uint32_t *off = malloc(4ull * n);
    uint16_t *len = malloc(2ull * n);
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t l = fsz;
        if (!fsz) {                                             /* simple IMIX, 7:4:1 */
            const uint32_t r = (i * 2654435761u >> 16) % 12u;
            l = r < 7 ? 64 : r < 11 ? 594 : 1500;
        }
        off[i] = (uint32_t)bytes;
        len[i] = (uint16_t)l;
        bytes += l;
    }
    /* the frames where a NIC would DMA them: memory registered with the runtime (DPDK's
     * hugepage mbufs), so the poller's H2D is a straight DMA */
    uint8_t *fr = NULL;
    if (udpdk_gpu_host_alloc(udpdk_gpu_context(), bytes + 64, (void **)&fr)) { perror("host_alloc"); return 1; }
    for (uint32_t i = 0; i < n; i++) make_frame(fr + off[i], len[i], (uint16_t)(10000 + i % (uint32_t)S), i);
    static char buf[65536];                    /* up to the largest UDP payload */
    /* the host's single-thread copy rate out of pinned memory (see the top of this file) */
    double copy_gbps = 0;
    {
        uint64_t pay = 0;
        for (uint32_t i = 0; i < n; i++) pay += len[i] > 42 ? len[i] - 42u : 0u;
        const uint64_t cb = (pay > (256ull << 20) ? pay : (256ull << 20)) & ~(uint64_t)65535;
        uint8_t *src = NULL;
        if (!udpdk_gpu_host_alloc(udpdk_gpu_context(), cb, (void **)&src)) {
            memset(src, 1, cb);
            double best = 1e30;
            volatile uint8_t sink = 0;
            for (int r = 0; r < 3; r++) {
                const double c0 = now();
                for (uint64_t o = 0; o < cb; o += 65536) {
                    memcpy(buf, src + o, 65536);
                    sink ^= buf[o & 65535];
                }
                const double dt = now() - c0;
                if (dt < best) best = dt;
            }
            (void)sink;
            copy_gbps = (double)cb / best / 1e9;
            udpdk_gpu_host_free(udpdk_gpu_context(), src);
        }
    }
    double t_poll = 0, t_recv = 0;
    uint64_t got = 0, pbytes = 0;
    for (int r = 0; r < reps + 1; r++) {                        /* rep 0 warms up */
        udpdk_rx_stats_t st;
        const double t0 = now();
        if (udpdk_poll_rx(fr, bytes, off, len, NULL, n, &st) < 0) { perror("udpdk_poll_rx"); return 1; }
        const double t1 = now();
        uint64_t g = 0, pb = 0;
        const uint32_t per = n / (uint32_t)S;
        for (int s = 0; s < S; s++) {
            const uint32_t want = per + ((uint32_t)s < n % (uint32_t)S ? 1u : 0u);
            for (uint32_t k = 0; k < want; k++) {
                const ssize_t m = udpdk_recvfrom(s, buf, sizeof(buf), 0, NULL, NULL);
                if (m < 0) { perror("udpdk_recvfrom"); return 1; }
                pb += (uint64_t)m;
                g++;
            }
        }
        const double t2 = now();
        if (r) {
            t_poll += t1 - t0;
            t_recv += t2 - t1;
            got += g;
            pbytes += pb;
        }
    }
    /* the reference's arrangement: poller beside the application */
    /* two batches share a socket's 2047-entry ring: at most 1023 datagrams per socket per batch
     * (a burst that does not fit is dropped whole, as flush_rx_queue does, and would never come) */
    /* BENCH_SOCK_OVERLAP=0: the sequential part only (a poll profile of it alone) */
    const char *ov = getenv("BENCH_SOCK_OVERLAP");
    const int oreps = ov && !atoi(ov) ? 0 : 2 * reps + 2;
    const uint32_t n_ov = n < 1023u * (uint32_t)S ? n : 1023u * (uint32_t)S;
    const uint64_t bytes_ov = n_ov < n ? off[n_ov] : bytes;
    struct poller P = {fr, bytes_ov, off, len, n_ov, oreps, 0, 0, 0};
    pthread_t th, wd;
    static unsigned wd_s = 100;
    if (pthread_create(&wd, NULL, watchdog_main, &wd_s)) { perror("pthread_create"); return 1; }
    pthread_detach(wd);
    uint64_t ogot = 0;
    const double o0 = now();
    if (pthread_create(&th, NULL, poller_main, &P)) { perror("pthread_create"); return 1; }
    for (int r = 0; r < oreps; r++) {
        while (atomic_load(&P.posted) <= r) ;
        if (P.err) { errno = P.err; perror("udpdk_poll_rx (poller thread)"); return 1; }
        const uint32_t per = n_ov / (uint32_t)S;
        for (int s = 0; s < S; s++) {
            const uint32_t want = per + ((uint32_t)s < n_ov % (uint32_t)S ? 1u : 0u);
            for (uint32_t k = 0; k < want; k++) {
                if (udpdk_recvfrom(s, buf, sizeof(buf), 0, NULL, NULL) < 0) { perror("udpdk_recvfrom"); return 1; }
                ogot++;
            }
        }
        atomic_store(&P.consumed, r + 1);
    }
    const double o1 = now();
    pthread_join(th, NULL);
    const double dg = (double)got / reps;
    printf("{\"overlap_mdgram_s\": %.2f, \"overlap_batches\": %d, \"frames\": %u, \"frame_bytes\": %s, \"sockets\": %d, \"reps\": %d, "
           "\"poll_ms\": %.3f, \"recv_ms\": %.3f, \"poll_mdgram_s\": %.2f, \"recv_mdgram_s\": %.2f, "
           "\"end_to_end_mdgram_s\": %.2f, \"end_to_end_frame_gbps\": %.2f, \"delivered_per_batch\": %.0f, "
           "\"payload_bytes_per_batch\": %.0f, \"host_copy_gbps\": %.2f, \"recv_gbps\": %.2f, \"recv_over_copy\": %.3f}\n",
           oreps ? (double)ogot / (o1 - o0) / 1e6 : 0.0, oreps, n, fsz ? argv[3] : "\"IMIX\"", S, reps, 1e3 * t_poll / reps, 1e3 * t_recv / reps,
           dg / (t_poll / reps) / 1e6, dg / (t_recv / reps) / 1e6, dg / ((t_poll + t_recv) / reps) / 1e6,
           (double)bytes / ((t_poll + t_recv) / reps) / 1e9, dg, (double)pbytes / reps, copy_gbps,
           (double)pbytes / t_recv / 1e9, copy_gbps > 0 ? (double)pbytes / t_recv / 1e9 / copy_gbps : 0.0);
    udpdk_gpu_host_free(udpdk_gpu_context(), fr);
    udpdk_cleanup();
    return 0;
}
