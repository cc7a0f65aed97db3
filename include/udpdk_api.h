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
 * udpdk_poll_rx() (the replacement of poller.c:516-545's rte_eth_rx_burst loop). Frames built by
 * udpdk_sendto() leave through udpdk_tx_drain() (the replacement of rte_eth_tx_burst,
 * poller.c:415-425).
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
 * udpdk_args.c:21-49; optional [gpu] device / max_frames / max_lanes) and create the GPU
 * context. Returns 0, or -1 with errno. */
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

ssize_t udpdk_recvfrom(int s, void *buf, size_t len, int flags,
                       struct sockaddr *src_addr, socklen_t *addrlen);

int udpdk_close(int s);

void udpdk_dump_payload(const char *payload, int len);

/* ---- extensions ----------------------------------------------------------------------------- */

/* Sockets: NUM_SOCKETS_MAX is 1024 in the reference (udpdk_constants.h:12); widened here
 * (SURVEY.md §8 Q11). Per-socket RX ring: EXCH_RING_SIZE entries (udpdk_constants.h:49). */
#define UDPDK_MAX_SOCKETS  4096
#define UDPDK_RX_RING_SIZE 2048

/* RX entry point of the GPU poller: classify a batch of received frames (host memory, as they
 * come off the NIC) on the GPU and append every delivered datagram to its socket's RX ring,
 * all-or-nothing per socket per call like rte_ring_enqueue_bulk (poller.c:287-290).
 * stats may be NULL. Returns 0 or -1 with errno. */
int udpdk_poll_rx(const uint8_t *frames, uint64_t frames_bytes, const uint32_t *offset,
                  const uint16_t *length, const uint32_t *ptype, uint32_t n,
                  udpdk_rx_stats_t *stats);

/* TX exit point: move up to max queued frames (built by udpdk_sendto) into out (packed back to
 * back, out_off/out_len per frame). *n_out = frames moved. Returns 0 or -1 with errno. */
int udpdk_tx_drain(uint8_t *out, uint64_t out_cap, uint32_t *out_off, uint16_t *out_len,
                   uint32_t max, uint32_t *n_out);

/* Flatten the bind table into a snapshot in list order (valid until the next call or the next
 * bind/close). compat != 0 keys lanes by the reference's (uint8_t) slot (poller.c:294). */
int udpdk_btable_snapshot(udpdk_bind_snapshot_t *snap, int compat);

/* The GPU context created by udpdk_init (NULL before). */
udpdk_gpu_ctx *udpdk_gpu_context(void);

/* TX header configuration (what udpdk_init reads from the .ini). Raw network-order IPv4. */
int udpdk_config_set(const uint8_t src_mac[6], const uint8_t dst_mac[6], uint32_t src_ip_raw);
int udpdk_config_get(uint8_t src_mac[6], uint8_t dst_mac[6], uint32_t *src_ip_raw);

/* Build the frame udpdk_sendto would build for sockfd (auto-binding it if unbound) into out
 * (len + 42 bytes) without queueing it. Returns frame length or -1 with errno. */
ssize_t udpdk_build_frame(int sockfd, const void *buf, size_t len,
                          const struct sockaddr *dest_addr, socklen_t addrlen, uint8_t *out);

/* Socket slot state (exch_slot_info, udpdk_types.h:40-47) for the GPU TX slot table. */
int udpdk_slot_table(udpdk_slot_t *slots, uint32_t n_slots);

/* Drop every socket, binding, queue and the interrupt flag without touching the GPU context
 * (test isolation; the reference only resets through process restart). */
void udpdk_host_reset(void);

#ifdef __cplusplus
}
#endif

#endif /* UDPDK_API_H */
