/*
 * port_table.c — raw UDP port -> ordered bindings, and its flattening for the GPU.
 *
 * Semantics follow udpdk_bind_table.c: admission rules of btable_can_bind (:47-89), list order
 * of btable_add_binding (ANY bindings to the head, specific ones to the tail, :119-124),
 * removal of the first binding of a socket (:129-149) and the lowest-free-raw-index search of
 * btable_get_free_port (:33-42). A socket binds at most once (udpdk_syscall.c:201-205), so the
 * list nodes live in the socket slots themselves: no allocator (the reference's shmalloc pools,
 * and their stride bug, SURVEY.md §8 Q2, do not exist here).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "host_state.h"

void h_btable_reset(void)
{
    for (int p = 0; p < 65536; p++) {
        g_udpdk.port_head[p] = -1;
        g_udpdk.port_tail[p] = -1;
        g_udpdk.port_len[p] = 0;
    }
}

static int h_can_bind(uint32_t ip_new, uint32_t port, int opts)
{
    for (int32_t s = g_udpdk.port_head[port]; s >= 0; s = g_udpdk.slots[s].next) {
        const uint32_t ip_oth = g_udpdk.slots[s].ip;
        const int either_any = ip_oth == 0 || ip_new == 0;
        if (ip_oth != ip_new && !either_any)
            continue;                           /* different specific addresses never clash  */
        if (ip_oth != ip_new && (ip_oth == 0 || ip_new != 0) &&
            (opts & (H_SO_REUSEADDR | H_SO_REUSEPORT)))
            continue;                           /* ANY vs specific with the new socket reusing */
        if (ip_oth == ip_new && ip_new != 0 && (opts & H_SO_REUSEPORT) &&
            g_udpdk.slots[s].reuse_port)
            continue;                           /* same specific address, both REUSEPORT      */
        return 0;
    }
    return 1;
}

int h_btable_add(int sockfd, uint32_t ip, uint32_t port, int opts)
{
    port &= 0xFFFFu;
    if (!h_can_bind(ip, port, opts)) return -1;
    struct h_slot *sl = &g_udpdk.slots[sockfd];
    sl->reuse_addr = (opts & H_SO_REUSEADDR) != 0;
    sl->reuse_port = (opts & H_SO_REUSEPORT) != 0;
    sl->ip = ip;
    if (ip == 0) {                               /* INADDR_ANY: list head */
        sl->prev = -1;
        sl->next = g_udpdk.port_head[port];
        if (sl->next >= 0) g_udpdk.slots[sl->next].prev = sockfd;
        else g_udpdk.port_tail[port] = sockfd;
        g_udpdk.port_head[port] = sockfd;
    } else {                                     /* specific address: list tail */
        sl->next = -1;
        sl->prev = g_udpdk.port_tail[port];
        if (sl->prev >= 0) g_udpdk.slots[sl->prev].next = sockfd;
        else g_udpdk.port_head[port] = sockfd;
        g_udpdk.port_tail[port] = sockfd;
    }
    g_udpdk.port_len[port]++;
    g_udpdk.version++;
    return 0;
}

void h_btable_del(int sockfd, uint32_t port)
{
    port &= 0xFFFFu;
    for (int32_t s = g_udpdk.port_head[port]; s >= 0; s = g_udpdk.slots[s].next) {
        if (s != sockfd) continue;
        struct h_slot *sl = &g_udpdk.slots[s];
        if (sl->prev >= 0) g_udpdk.slots[sl->prev].next = sl->next;
        else g_udpdk.port_head[port] = sl->next;
        if (sl->next >= 0) g_udpdk.slots[sl->next].prev = sl->prev;
        else g_udpdk.port_tail[port] = sl->prev;
        sl->prev = sl->next = -1;
        g_udpdk.port_len[port]--;
        g_udpdk.version++;
        return;
    }
}

int h_btable_free_port(void)
{
    for (int p = 0; p < 65536; p++)
        if (g_udpdk.port_head[p] < 0) return p;
    return -1;
}

/* ---- snapshot ----------------------------------------------------------------------------- */
static uint32_t        *s_first;
static uint16_t        *s_count;
static udpdk_binding_t *s_binds;
static udpdk_slot_t    *s_slots;

int udpdk_btable_snapshot(udpdk_bind_snapshot_t *snap, int compat)
{
    if (!snap) { errno = EINVAL; return -1; }
    if (!s_first) {
        s_first = calloc(65536, sizeof(uint32_t));
        s_count = calloc(65536, sizeof(uint16_t));
        s_binds = calloc(UDPDK_MAX_SOCKETS, sizeof(udpdk_binding_t));
        s_slots = calloc(UDPDK_MAX_SOCKETS, sizeof(udpdk_slot_t));
        if (!s_first || !s_count || !s_binds || !s_slots) { errno = ENOMEM; return -1; }
    }
    uint32_t nb = 0;
    int32_t max_sock = 0;
    for (uint32_t p = 0; p < 65536; p++) {
        s_first[p] = nb;
        s_count[p] = 0;
        for (int32_t s = g_udpdk.port_head[p]; s >= 0; s = g_udpdk.slots[s].next) {
            const struct h_slot *sl = &g_udpdk.slots[s];
            s_binds[nb].ip = sl->ip;
            s_binds[nb].sockfd = s;
            s_binds[nb].reuse = (sl->reuse_addr || sl->reuse_port) ? 1u : 0u;
            if (s > max_sock) max_sock = s;
            nb++;
            s_count[p]++;
        }
    }
    memset(snap, 0, sizeof(*snap));
    snap->port_first = s_first;
    snap->port_count = s_count;
    snap->binds = s_binds;
    snap->n_binds = nb;
    snap->lane_mask = compat ? 0xFFu : 0xFFFFFFFFu;
    snap->n_lanes = compat ? 256u : (uint32_t)max_sock + 1u;
    udpdk_slot_table(s_slots, UDPDK_MAX_SOCKETS);
    snap->slots = s_slots;
    snap->n_slots = UDPDK_MAX_SOCKETS;
    snap->version = g_udpdk.version;
    return 0;
}
