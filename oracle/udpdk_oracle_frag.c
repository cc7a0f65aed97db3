/*
 * udpdk_oracle_frag.c — TEST INFRASTRUCTURE ONLY (see udpdk_oracle.h).
 *
 * CPU restatement of the RX reassembly step of the reference poller (udpdk_poller.c:338-361:
 * rte_ipv4_frag_pkt_is_fragmented -> rte_ipv4_frag_reassemble_packet(tbl, dr, m, tms, ip_hdr)
 * on the table made by rte_ip_frag_table_create(NUM_FLOWS_DEF, IP_FRAG_TBL_BUCKET_ENTRIES,
 * NUM_FLOWS_MAX, frag_cycles, ...), udpdk_poller.c:130, udpdk_constants.h:31-38).
 *
 * The table code is DPDK 20.05 lib/librte_ip_frag (rte_ipv4_reassembly.c, ip_frag_internal.c,
 * ip_frag_common.h), which is not in the container (deps/dpdk is an empty submodule); this is a
 * restatement of its published algorithm, pinned by the properties in tests/test_reasm_oracle.py
 * (round trips through the TX fragmentation restatement, hand-derived scenarios) -- "parity
 * unpinned" against DPDK itself.
 *
 *   key        = (8 bytes src_addr|dst_addr, packet_id), the packet_id as a u32
 *   placement  = ipv4_frag_hash: v = crc32c(crc32c(crc32c(0xeaad8405, src), dst), id) (the
 *                SSE4.2 instruction: no pre/post inversion), sig1 = v, sig2 = (v << 7) + (v >> 14);
 *                the two candidate buckets start at entry (sig & entry_mask), entry_mask =
 *                (entries - 1) & ~(bucket_entries - 1), entries = align32pow2(buckets * assoc)
 *   lookup     = ip_frag_lookup: scan p1[i], p2[i] for i < assoc; a key match wins, else the
 *                first empty and the first expired (start + max_cycles < tms) slot are noted
 *   find       = ip_frag_find: match + expired -> free its fragments and restart it at tms
 *                (ip_frag_tbl_reuse: the entry moves to the LRU list's tail); no match -> a
 *                stale slot is freed and used, else an empty one, but an empty one only while
 *                use_entries < max_entries: at the limit the LRU list's head (the entry added or
 *                reused longest ago) is deleted if it has expired, else the fragment is dropped
 *                (fail_nospace); no slot -> NULL (dropped). use_entries counts valid entries
 *                (ip_frag_tbl_add / _del, ip_frag_inuse after a flow ends). The reference's table
 *                has 4096 x 16 = 65536 entries and max_entries = NUM_FLOWS_MAX = 65535.
 *   process    = ip_frag_process: frag_size += len; ofs 0 -> slot 0 (dup -> error); MF clear ->
 *                total_size = ofs + len, slot 1 (dup -> error); else slot last_idx++ (< 4, else
 *                error). frag_size < total_size: wait; == with slot 0 present: reassemble
 *                (ipv4_frag_reassemble's backward chain walk; a hole -> error); otherwise error.
 *                Any error frees the flow's fragments; the entry is invalidated after an error or
 *                a reassembly.
 *   output     = the first fragment's 34 header bytes + the fragments' IPv4 payloads at their
 *                offsets; total_length = total_size + 20, fragment_offset keeps DF only
 *                (ipv4_frag_reassemble), and the header checksum: DPDK writes 0 ("TODO must fix
 *                the IP header checksum", poller.c:358), kept with the DPDK flag; by default the
 *                RFC 1071 value is written.
 *
 * Divergences: l3_len is 20 as the poller sets it (poller.c:346); a fragment whose
 * IPv4 total_length reaches past its frame, or whose data would end past the table's datagram
 * capacity, is dropped (DPDK would chain the short mbuf); Ethernet padding after a fragment's IP
 * payload is not carried into the datagram (DPDK chains whole mbuf data).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "udpdk_oracle.h"

#define OF_MAX_FRAG 4u            /* RTE_LIBRTE_IP_FRAG_MAX_FRAG */
#define OF_FIRST 0u
#define OF_LAST 1u
#define OF_MIN 2u

struct of_frag {
    uint32_t ofs, len;
    uint8_t *data;                /* the fragment's IPv4 payload (len bytes), NULL: empty slot */
    uint8_t  hdr[34];             /* Ethernet + IPv4 header of the frame (slot 0 uses it)      */
    int      this_call;           /* arrived during the current oracle_reassemble call         */
};

struct of_entry {
    uint32_t src, dst, id;
    int      valid;               /* key_len != 0                                              */
    uint64_t start;
    uint64_t lru;                 /* position in the LRU list: the table's add/reuse counter   */
    uint32_t frag_size, total_size, last_idx;
    struct of_frag frags[OF_MAX_FRAG];
};

struct oracle_ftable {
    uint32_t entries, assoc, mask, max_dgram;
    uint32_t max_entries, use_entries, flags;
    uint64_t max_cycles, lru_seq;
    struct of_entry *e;
};

static uint32_t crc32c_u32(uint32_t crc, uint32_t v)
{
    crc ^= v;
    for (int i = 0; i < 32; ++i) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    return crc;
}

uint32_t oracle_frag_hash(uint32_t src, uint32_t dst, uint32_t id, uint32_t *sig2)
{
    uint32_t v = crc32c_u32(0xeaad8405u, src);
    v = crc32c_u32(v, dst);
    v = crc32c_u32(v, id);
    *sig2 = (v << 7) + (v >> 14);
    return v;
}

oracle_ftable *oracle_ftable_new(uint32_t bucket_num, uint32_t bucket_entries,
                                 uint64_t max_cycles, uint32_t max_dgram, uint32_t max_entries,
                                 uint32_t flags)
{
    uint64_t n = (uint64_t)bucket_num * bucket_entries, p = 1;
    while (p < n) p <<= 1;
    if (!bucket_entries || (bucket_entries & (bucket_entries - 1)) || p > (1u << 24)) return NULL;
    if (max_entries > p) return NULL;                /* rte_ip_frag_table_create: EINVAL */
    oracle_ftable *t = calloc(1, sizeof(*t));
    if (!t) return NULL;
    t->entries = (uint32_t)p;
    t->assoc = bucket_entries;
    t->mask = (t->entries - 1) & ~(bucket_entries - 1);
    t->max_cycles = max_cycles;
    t->max_dgram = max_dgram;
    t->max_entries = max_entries ? max_entries : t->entries;
    t->flags = flags;
    t->e = calloc(t->entries, sizeof(struct of_entry));
    if (!t->e) { free(t); return NULL; }
    return t;
}

static void of_free_frags(struct of_entry *e)
{
    for (uint32_t k = 0; k < OF_MAX_FRAG; ++k) {
        free(e->frags[k].data);
        e->frags[k].data = NULL;
    }
}

void oracle_ftable_free(oracle_ftable *t)
{
    if (!t) return;
    for (uint32_t i = 0; i < t->entries; ++i) of_free_frags(&t->e[i]);
    free(t->e);
    free(t);
}

static void of_reset(struct of_entry *e, uint64_t tms)      /* ip_frag_reset */
{
    e->start = tms;
    e->total_size = UINT32_MAX;
    e->frag_size = 0;
    e->last_idx = OF_MIN;
    for (uint32_t k = 0; k < OF_MAX_FRAG; ++k) e->frags[k].len = e->frags[k].ofs = 0;
}

static int of_expired(const oracle_ftable *t, const struct of_entry *e, uint64_t tms)
{
    return t->max_cycles + e->start < tms;
}

static void of_del(oracle_ftable *t, struct of_entry *e)      /* ip_frag_tbl_del / ip_frag_inuse */
{
    of_free_frags(e);
    e->valid = 0;
    t->use_entries--;
}

/* TAILQ_FIRST(&tbl->lru): the valid entry added or reused longest ago. */
static struct of_entry *of_lru_head(oracle_ftable *t)
{
    struct of_entry *h = NULL;
    for (uint32_t i = 0; i < t->entries; ++i)
        if (t->e[i].valid && (!h || t->e[i].lru < h->lru)) h = &t->e[i];
    return h;
}

/* ip_frag_find (ip_frag_lookup inlined). */
static struct of_entry *of_find(oracle_ftable *t, uint32_t src, uint32_t dst, uint32_t id,
                                uint64_t tms, uint64_t *st)
{
    uint32_t sig2, sig1 = oracle_frag_hash(src, dst, id, &sig2);
    struct of_entry *p1 = t->e + (sig1 & t->mask), *p2 = t->e + (sig2 & t->mask);
    struct of_entry *empty = NULL, *old = NULL;
    for (uint32_t i = 0; i < t->assoc; ++i) {
        struct of_entry *c[2] = {p1 + i, p2 + i};
        for (int h = 0; h < 2; ++h) {
            struct of_entry *q = c[h];
            if (q->valid && q->src == src && q->dst == dst && q->id == id) {
                if (of_expired(t, q, tms)) {                 /* ip_frag_tbl_reuse */
                    st[ORACLE_RS_EXPIRED]++;
                    of_free_frags(q);
                    of_reset(q, tms);
                    q->lru = t->lru_seq++;
                }
                return q;
            }
            if (!q->valid) empty = empty ? empty : q;
            else if (of_expired(t, q, tms)) old = old ? old : q;
        }
    }
    struct of_entry *use = NULL;
    if (old) {                                               /* ip_frag_tbl_del */
        st[ORACLE_RS_EXPIRED]++;
        of_del(t, old);
        use = old;
    } else if (empty && t->use_entries >= t->max_entries) {
        struct of_entry *lru = of_lru_head(t);
        if (lru && of_expired(t, lru, tms)) {                /* the LRU head has expired */
            st[ORACLE_RS_EXPIRED]++;
            of_del(t, lru);
            use = empty;
        }                                                    /* else fail_nospace */
    } else {
        use = empty;
    }
    if (!use) return NULL;
    use->valid = 1;                                          /* ip_frag_tbl_add */
    use->src = src; use->dst = dst; use->id = id;
    of_reset(use, tms);
    use->lru = t->lru_seq++;
    t->use_entries++;
    return use;
}

/* ipv4_frag_reassemble's chain walk: 1 if the fragments chain from the last back to the first. */
static int of_chain_ok(const struct of_entry *e)
{
    const uint32_t first_len = e->frags[OF_FIRST].len;
    const uint32_t n = e->last_idx - 1;
    uint32_t ofs = e->frags[OF_LAST].ofs, curr = OF_LAST;
    while (ofs != first_len) {
        const uint32_t prev = curr;
        for (uint32_t i = n; i != OF_FIRST && ofs != first_len; i--) {
            if (e->frags[i].ofs + e->frags[i].len == ofs) {
                curr = i;
                ofs = e->frags[i].ofs;
            }
        }
        if (curr == prev) return 0;                          /* hole */
    }
    return 1;
}

static uint16_t of_ipcksum(const uint8_t *h)
{
    uint32_t s = 0;
    for (int i = 0; i < 20; i += 2) s += (uint32_t)h[i] | ((uint32_t)h[i + 1] << 8);
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    return (uint16_t)~s;
}

int64_t oracle_reassemble(oracle_ftable *t, const uint8_t *frames, uint64_t frames_bytes,
                          const uint32_t *offset, const uint16_t *length, const uint32_t *meta,
                          uint32_t n, uint64_t tms, uint8_t *out, uint64_t out_cap,
                          uint32_t *out_off, uint16_t *out_len, uint32_t *out_origin,
                          uint32_t out_max, uint64_t stats[ORACLE_RS_N])
{
    uint32_t n_out = 0;
    uint64_t pos = 0;
    for (uint32_t i = 0; i < t->entries; ++i)
        for (uint32_t k = 0; k < OF_MAX_FRAG; ++k) t->e[i].frags[k].this_call = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if ((meta[i] & 0xFu) != 2u) continue;                /* FRAG verdicts only */
        stats[ORACLE_RS_FRAGS]++;
        const uint8_t *f = frames + offset[i];
        const uint32_t flen = length[i];
        if ((uint64_t)offset[i] + flen > frames_bytes || flen < 34) { stats[ORACLE_RS_DROP_SHORT]++; continue; }
        const uint8_t *ip = f + 14;
        const int32_t ip_len = (int32_t)((ip[2] << 8) | ip[3]) - 20;  /* l3_len = 20, poller.c:346 */
        if (ip_len <= 0) { stats[ORACLE_RS_DROP_LEN]++; continue; }
        const uint32_t ff = (uint32_t)((ip[6] << 8) | ip[7]);
        const uint32_t ofs = (ff & 0x1FFFu) * 8u, mf = ff & 0x2000u;
        if (34u + (uint32_t)ip_len > flen || ofs + (uint32_t)ip_len > t->max_dgram) {
            stats[ORACLE_RS_DROP_SHORT]++;
            continue;
        }
        uint32_t src, dst;
        memcpy(&src, ip + 12, 4);
        memcpy(&dst, ip + 16, 4);
        const uint32_t id = (uint32_t)(ip[4] | (ip[5] << 8));
        struct of_entry *e = of_find(t, src, dst, id, tms, stats);
        if (!e) { stats[ORACLE_RS_NO_SPACE]++; continue; }
        /* ip_frag_process */
        const uint32_t len = (uint32_t)ip_len;
        uint32_t idx;
        e->frag_size += len;
        if (ofs == 0) {
            idx = e->frags[OF_FIRST].data == NULL ? OF_FIRST : UINT32_MAX;
        } else if (!mf) {
            e->total_size = ofs + len;
            idx = e->frags[OF_LAST].data == NULL ? OF_LAST : UINT32_MAX;
        } else if ((idx = e->last_idx) < OF_MAX_FRAG) {
            e->last_idx++;
        }
        if (idx >= OF_MAX_FRAG) {
            stats[ORACLE_RS_ERRORS]++;
            of_del(t, e);
            continue;
        }
        struct of_frag *s = &e->frags[idx];
        s->ofs = ofs;
        s->len = len;
        s->data = malloc(len);
        if (!s->data) return -1;
        memcpy(s->data, ip + 20, len);
        memcpy(s->hdr, f, 34);
        s->this_call = 1;
        if (e->frag_size < e->total_size) continue;
        if (e->frag_size == e->total_size && e->frags[OF_FIRST].data && of_chain_ok(e)) {
            const uint32_t fl = 34u + e->total_size;
            const uint64_t at = (pos + 15u) & ~15ull;
            if (n_out == out_max || at + fl > out_cap) return -1;
            uint8_t *o = out + at;
            memcpy(o, e->frags[OF_FIRST].hdr, 34);
            const uint32_t tl = e->total_size + 20u;
            o[16] = (uint8_t)(tl >> 8); o[17] = (uint8_t)tl;
            o[20] &= 0x40u; o[21] = 0;                       /* DF only */
            o[24] = o[25] = 0;
            if (!(t->flags & 1u)) {                          /* else DPDK's 0 (poller.c:358) */
                const uint16_t ck = of_ipcksum(o + 14);
                memcpy(o + 24, &ck, 2);
            }
            for (uint32_t k = 0; k < e->last_idx; ++k)
                if (e->frags[k].data) memcpy(o + 34 + e->frags[k].ofs, e->frags[k].data, e->frags[k].len);
            out_off[n_out] = (uint32_t)at;
            out_len[n_out] = (uint16_t)fl;
            out_origin[n_out] = i;
            n_out++;
            pos = at + fl;
            stats[ORACLE_RS_DONE]++;
        } else {
            const int sized = e->frag_size == e->total_size && e->frags[OF_FIRST].data;
            stats[sized ? ORACLE_RS_HOLES : ORACLE_RS_ERRORS]++;
        }
        of_del(t, e);
    }
    for (uint32_t i = 0; i < t->entries; ++i)
        if (t->e[i].valid)
            for (uint32_t k = 0; k < OF_MAX_FRAG; ++k)
                if (t->e[i].frags[k].data && t->e[i].frags[k].this_call) stats[ORACLE_RS_STORED]++;
    return n_out;
}
