/*
 * udpdk_api.h — POSIX-like UDP socket surface, source compatible with the reference's
 * udpdk/udpdk_api.h:19-41 (same ten functions, same argument meaning, -1 + errno on error) plus
 * udpdk_dump_payload (udpdk_api.symlist:11). Applications written against the reference
 * (apps/pktgen, apps/pingpong) compile against this header and link against libudpdk_amd.so
 * unchanged (tests/test_ref_apps.py builds both from /root/reference in place).
 *
 * What changed underneath: there is no forked DPDK poller. The per-packet RX work of
 * udpdk_poller.c runs as HIP kernels on an MI355X through udpdk_gpu.h; udpdk_init() creates the
 * GPU context (and fails with ENODEV when no GPU is present), and frame batches enter through
 * udpdk_poll_rx() (the replacement of poller.c:516-545's rte_eth_rx_burst loop). Datagrams queued
 * by udpdk_sendto() leave as frames built on the GPU through udpdk_tx_drain() (the replacement of
 * the poller's TX half, poller.c:453-514). A poller thread can drive both against a port
 * (udpdk_port_attach), as the reference's forked poller drives NIC port 0.
 *
 * Extensions below the reference surface are prefixed udpdk_ too and documented in
 * INTEGRATION.md.
 */
#ifndef UDPDK_API_H
#define UDPDK_API_H

/* What the reference header supplied to applications transitively through udpdk_types.h:19-23
 * (apps/pktgen/main.c:54-58 uses bool without including <stdbool.h> itself). */
#include <netinet/in.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include "udpdk_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference surface (udpdk_api.h:19-41) ------------------------------------------------ */

/* Parse "-c <file.ini>" (keys [port0] mac_addr / ip_addr, [port0_dst] mac_addr as in
 * udpdk_args.c:21-49; optional [gpu] device / devices / max_frames / max_lanes / port ...,
 * INTEGRATION.md) and create the GPU context(s). Returns 0, or -1 with errno. */
int udpdk_init(int argc, char *argv[]);

/* Make blocking calls (udpdk_recvfrom) return -1/EINTR (udpdk_init.c:374-378). */
void udpdk_interrupt(int signum);

/* Close every socket, free all queues and the GPU context (udpdk_init.c:392-424). */
void udpdk_cleanup(void);

int udpdk_socket(int domain, int type, int protocol);

int udpdk_getsockopt(int sockfd, int level, int optname, void *optval, socklen_t *optlen);

int udpdk_setsockopt(int sockfd, int level, int optname, const void *optval, socklen_t optlen);

int udpdk_bind(int s, const struct sockaddr *addr, socklen_t addrlen);

ssize_t udpdk_sendto(int sockfd, const void *buf, size_t len, int flags,
                     const struct sockaddr *dest_addr, socklen_t addrlen);

/* One reading thread per socket at a time: the socket's receive ring is single-consumer, like
 * the reference's SP/SC rx_q (udpdk_init.c:270-272). */
ssize_t udpdk_recvfrom(int s, void *buf, size_t len, int flags,
                       struct sockaddr *src_addr, socklen_t *addrlen);

int udpdk_close(int s);

void udpdk_dump_payload(const char *payload, int len);

/* ---- extensions ----------------------------------------------------------------------------- */

/* Sockets: NUM_SOCKETS_MAX is 1024 in the reference (udpdk_constants.h:12); widened here
 * (SURVEY.md §8 Q11). Per-socket RX ring: EXCH_RING_SIZE entries (udpdk_constants.h:49). */
#define UDPDK_MAX_SOCKETS  4096
#define UDPDK_RX_RING_SIZE 2048

/* RX entry point of the GPU poller (one turn of poller_body's RX half, udpdk_poller.c:516-545):
 * classify a batch of received frames (host memory, as they come off the NIC) on the GPU,
 * reassemble IPv4 fragments on the device, gather every accepted datagram's payload on the GPU
 * into pinned host slabs and append it to its socket's RX ring in arrival order. A socket's
 * deliveries are admitted per burst of BURST_SIZE = 128 frames (frame index / 128), each burst
 * all-or-nothing like the rte_ring_enqueue_bulk of flush_rx_queue (poller.c:274-292): a burst
 * whose datagrams do not fit the ring is dropped, later bursts may still fit. Reassembled
 * datagrams count at the index of the fragment that completed them. Safe to call from a poller
 * thread while application threads call the socket functions. stats may be NULL. Returns 0 or
 * -1 with errno. A batch polled in one piece publishes nothing when it fails; a large batch of
 * long frames polled in chunks ([gpu] poll_chunk_mb) may fail after its first chunks' bursts were
 * published (each chunk's bursts go to the rings before the next chunk is admitted, as the
 * reference's burst loop publishes each burst): a caller that retries such a batch receives those
 * datagrams twice, so retry only what the rings did not get, or poll with poll_chunk_mb = 0. */
int udpdk_poll_rx(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                  const uint16_t *length, const uint32_t *ptype, uint32_t n,
                  udpdk_rx_stats_t *stats);

/* Deliveries udpdk_poll_rx dropped because the pinned payload slabs ([gpu] slab_bytes_max /
 * slab_count_max, default 4 GiB / 1024 slabs) were all held by datagrams not yet received: the
 * reference's mbuf pool exhausted. */
uint64_t udpdk_rx_nobufs(void);

/* TX exit point (the poller's TX half, udpdk_poller.c:453-514): take queued datagrams in the
 * poller's order (sockets in index order, each drained while the burst holds fewer than
 * BURST_SIZE frames), build their frames on the GPU (header build, rte_ipv4_cksum, payload copy,
 * and the IPv4 fragmentation of frames longer than the MTU, udpdk_gpu_tx_build_mtu) and copy
 * them into out, back to back (out_off/out_len per frame; a datagram's fragments are
 * consecutive frames and never split across calls). At most max frames and out_cap bytes.
 * *n_out = frames written. Needs the GPU context (udpdk_init). Returns 0 or -1 with errno. */
int udpdk_tx_drain(uint8_t *out, uint64_t out_cap, uint32_t *out_off, uint16_t *out_len,
                   uint32_t max, uint32_t *n_out);

/* Datagrams waiting in the TX rings. */
uint64_t udpdk_tx_pending(void);

/* Datagrams udpdk_tx_drain dropped because they needed more frames or bytes than a drain with
 * the caller's limits can ever carry (they would otherwise block their socket's ring). */
uint64_t udpdk_tx_dropped(void);

/* ---- the poller thread ----------------------------------------------------------------------
 * The reference forks a poller process that busy-polls NIC port 0 (udpdk_init.c:293-368,
 * poller.c:448-546). Here a port is a pair of callbacks; udpdk_port_attach starts a poller
 * thread that loops: udpdk_tx_drain -> tx_burst, rx_burst -> udpdk_poll_rx, until
 * udpdk_port_detach or udpdk_cleanup. Applications that do not attach a port drive
 * udpdk_poll_rx / udpdk_tx_drain themselves, from one thread (the poller role). */
typedef struct udpdk_port_ops {
    /* Write up to max received frames back to back into frames (cap bytes; keep
     * UDPDK_GPU_FRAMES_TAILROOM bytes of it free), offset[i] / length[i] per frame; return the
     * frame count (0: nothing now). */
    uint32_t (*rx_burst)(void *user, uint8_t *frames, uint64_t cap, uint32_t *offset,
                         uint16_t *length, uint32_t max);
    /* Transmit n frames; the callee copies what it keeps. */
    void (*tx_burst)(void *user, const uint8_t *frames, const uint32_t *offset,
                     const uint16_t *length, uint32_t n);
    void    *user;
    uint32_t batch_frames;   /* frames per RX batch (0: 4096)                                   */
} udpdk_port_ops_t;

int udpdk_port_attach(const udpdk_port_ops_t *ops);
int udpdk_port_detach(void);
/* A built-in loopback port: frames drained from TX come back on RX (tests and demos). */
int udpdk_port_loopback(udpdk_port_ops_t *ops);

/* Flatten the bind table into a snapshot in list order (valid until the next call or the next
 * bind/close). compat != 0 keys lanes by the reference's (uint8_t) slot (poller.c:294). */
int udpdk_btable_snapshot(udpdk_bind_snapshot_t *snap, int compat);

/* The GPU context created by udpdk_init (NULL before). */
udpdk_gpu_ctx *udpdk_gpu_context(void);

/* The devices polls run on: with "[gpu] devices = 0-7" (two or more entries) udpdk_init creates
 * one RX shard context per entry and udpdk_poll_rx splits every batch into that many contiguous
 * shards, each classified, demultiplexed and gathered on its own device by its own pool thread;
 * the shards' lanes are concatenated in shard order before ring admission, so the rings are those
 * of a single-context poll. Fragments go through the main context's reassembly table. Writes up
 * to max device ids and returns how many there are (1 without "devices", 0 before udpdk_init). */
int udpdk_shard_devices(int *devices, int max);

/* The same device list read from a config file without creating any context (no GPU needed):
 * what udpdk_init(-c cfg_path) would bind, in shard order. Returns the count (1 for a single
 * "[gpu] device"), -EINVAL for a malformed list, -ENOENT for a missing file. */
int udpdk_shard_plan(const char *cfg_path, int *devices, int max);

/* With "[gpu] dispatch = rss" (and two or more devices) a poll sends each frame to the shard of
 * its RSS queue instead: one RX queue per device, queue = reta[Toeplitz hash] with
 * udpdk_gpu_rss's hash definition, default key and redirection table (the NIC's ETH_MQ_RX_RSS
 * that udpdk_init.c:112-137 asks for and leaves as a TODO); the shards' lanes are merged back in
 * arrival order, so the rings are still a single-context poll's. Writes the number of frames
 * each shard took in the last poll (up to max) and returns the shard count (0 without shards). */
int udpdk_shard_frames(uint32_t *frames, int max);

/* TX header configuration (what udpdk_init reads from the .ini). Raw network-order IPv4. */
int udpdk_config_set(const uint8_t src_mac[6], const uint8_t dst_mac[6], uint32_t src_ip_raw);
int udpdk_config_get(uint8_t src_mac[6], uint8_t dst_mac[6], uint32_t *src_ip_raw);
/* IPv4 MTU of the TX fragmentation (default IPV4_MTU_DEFAULT = 1500; (mtu - 20) % 8 == 0). */
int udpdk_config_mtu(uint32_t mtu);

/* Socket slot state (exch_slot_info, udpdk_types.h:40-47) for the GPU TX slot table. */
int udpdk_slot_table(udpdk_slot_t *slots, uint32_t n_slots);

/* Drop every socket, binding, queue and the interrupt flag without touching the GPU context
 * (test isolation; the reference only resets through process restart). */
void udpdk_host_reset(void);

#ifdef __cplusplus
}
#endif

#endif /* UDPDK_API_H */
