/*
 * udpdk_oracle_rss.c — TEST INFRASTRUCTURE ONLY (see udpdk_oracle.h).
 *
 * Receive-side scaling restated. The reference asks for ETH_MQ_RX_RSS with
 * one RX ring (udpdk_init.c:112-137), so the NIC's hash never selects anything there; this is the
 * behaviour a multi-queue port gives: the Toeplitz hash over the IPv4 (+ UDP) tuple (the
 * published algorithm; pinned by the Microsoft RSS verification suite's IPv4 vectors in
 * tests/golden/rss_vectors.json) and the redirection table, then each queue's frames in arrival
 * order (what each queue's poller would receive from rte_eth_rx_burst).
 */
#include <stdint.h>
#include <string.h>

#include "udpdk_oracle.h"

/* Toeplitz: for every set bit i (MSB first) of the input, XOR the key bits [i, i + 32). */
uint32_t oracle_toeplitz(const uint8_t key[40], const uint8_t *data, uint32_t len)
{
    uint32_t h = 0;
    uint32_t win = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) | ((uint32_t)key[2] << 8) | key[3];
    for (uint32_t i = 0; i < len; ++i) {
        for (int b = 7; b >= 0; --b) {
            if ((data[i] >> b) & 1u) h ^= win;
            /* slide the window one bit: bring in key bit 32 + 8 i + (7 - b) */
            const uint32_t nb = 32u + 8u * i + (uint32_t)(7 - b);
            const uint32_t kbit = nb < 320u ? (key[nb >> 3] >> (7u - (nb & 7u))) & 1u : 0u;
            win = (win << 1) | kbit;
        }
    }
    return h;
}

int oracle_rss(const uint8_t key[40], uint32_t hash_types, const uint16_t *reta, uint32_t reta_size,
               uint32_t n_queues, const uint8_t *frames, uint64_t frames_bytes,
               const uint32_t *offset, const uint16_t *length, const uint32_t *ptype, uint32_t n,
               uint32_t *hash_out, uint32_t *queue_off, uint32_t *queue_pkt)
{
    uint32_t count[64] = {0};
    if (n_queues == 0 || n_queues > 64) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t off = offset[i], len = length[i];
        uint32_t h = 0;
        if ((uint64_t)off + len <= frames_bytes && len >= 34) {
            const uint8_t *f = frames + off;
            /* the rx_classify IPv4 gate: ptype given, else derived from ether_type */
            const uint32_t pt = ptype ? ptype[i] : ((f[12] == 0x08 && f[13] == 0x00) ? 0x211u : 0x1u);
            if (pt & 0x10u) {
                const uint16_t ff = (uint16_t)((f[20] << 8) | f[21]);
                const int frag = (ff & 0x3FFFu) != 0;
                const int udp4 = !frag && f[23] == 17 && len >= 38 && (hash_types & 2u);
                if (udp4) h = oracle_toeplitz(key, f + 26, 12);
                else if (hash_types & 1u) h = oracle_toeplitz(key, f + 26, 8);
            }
        }
        hash_out[i] = h;
        count[reta[h & (reta_size - 1)]]++;
    }
    queue_off[0] = 0;
    for (uint32_t q = 0; q < n_queues; ++q) queue_off[q + 1] = queue_off[q] + count[q];
    uint32_t pos[64];
    memcpy(pos, queue_off, n_queues * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i) queue_pkt[pos[reta[hash_out[i] & (reta_size - 1)]]++] = i;
    return 0;
}
