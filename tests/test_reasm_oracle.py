"""CPU checks of the RX reassembly restatement (oracle_reassemble: the poller's
rte_ipv4_frag_reassemble_packet path, udpdk_poller.c:338-361, DPDK 20.05 restated).

DPDK is not in the container and the reference has no fragment fixtures, so the restatement is
pinned by (1) round trips through the TX fragmentation restatement (what the reference sends, the
reference reassembles: the datagram comes back byte-identical) and (2) hand-derived scenarios
for each table outcome; bit-level parity with DPDK itself is unpinned."""
import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi
from reasm_util import batch, frames_of, ip_frame, raw_ip, split, udp_datagram, verdicts

SRC = raw_ip("172.31.100.2")
DST = raw_ip("172.31.100.1")


def _run(t, frames, tms=0, pad=True):
    buf, off, ln = batch(frames, pad=pad)
    meta = verdicts(buf, off, ln)
    out, oo, ol, og, st = t.reassemble(buf, off, ln, meta, tms)
    return frames_of(out, oo, ol), og.tolist(), st


def _same_but_cksum(a, b):
    return a[:24] == b[:24] and a[26:] == b[26:]


@pytest.mark.parametrize("mtu", [1500, 1020, 572])
def test_tx_fragments_reassemble_to_the_sent_frame(mtu):
    rng = np.random.default_rng(mtu)
    t = O.FragTable()
    sent, frags = [], []
    sizes = [L for L in [1473, 2006, 2952, 2953, 5000, 5911, 8000] if L + 8 <= 4 * (mtu - 20)]
    for k, L in enumerate(sizes):
        pay = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        fr = O.tx_frame(O_MAC[0], O_MAC[1], SRC, 1, 0, 0x1027, DST, 0x1127, pay)
        fs = O.tx_fragment(fr, mtu)
        # distinct ids so the flows do not collide (udpdk_sendto always sends id 0)
        fs = [f[:18] + bytes([k, 0]) + f[20:] for f in fs]
        sent.append(fr[:18] + bytes([k, 0]) + fr[20:])
        frags.append(fs)
    order = [f for fs in frags for f in fs]
    rng.shuffle(order)
    got, origin, st = _run(t, order)
    assert len(sent) >= 2
    assert st["done"] == len(sent) and st["errors"] == st["holes"] == st["stored"] == 0
    by_id = {g[18]: g for g in got}
    for k, fr in enumerate(sent):
        if True:
            assert _same_but_cksum(by_id[k], fr)
            s = sum(by_id[k][14 + i] | (by_id[k][15 + i] << 8) for i in range(0, 20, 2))
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            assert s == 0xFFFF
    assert origin == sorted(origin)            # completion order = arrival order of the last piece


O_MAC = (bytes.fromhex("6805ca95f8ec"), bytes.fromhex("6805ca95fa64"))


def test_short_fragment_frames():
    """An unpadded frame of 34-41 B holds a whole IPv4 header but not a UDP one: a fragment is
    handed to reassembly on its IPv4 header alone (poller.c:338-361: rte_ipv4_frag_pkt_is_fragmented
    before any UDP field is read), anything else is TRUNC, and a 33 B frame is TRUNC either way.
    Datagrams whose last fragment carries 1-7 bytes then come back whole."""
    d = udp_datagram(0x1027, 0x1127, bytes(range(19)))          # 27 B: fragments of 8, 8, 8 + 3
    fs = split(SRC, DST, 7, d, [8, 8, 11])
    assert [len(f) for f in fs] == [42, 42, 45]
    fs = split(SRC, DST, 7, d, [8, 16, 3])
    assert len(fs[2]) == 37
    whole = ip_frame(SRC, DST, 8, 0, b"\0" * 5, False)           # 39 B, not a fragment
    buf, off, ln = batch(fs + [whole, fs[2][:33]], pad=False)
    v = verdicts(buf, off, ln) & 0xF
    assert v.tolist() == [abi.V_FRAG] * 3 + [abi.V_TRUNC, abi.V_TRUNC]
    got, _, st = _run(O.FragTable(), fs, pad=False)
    assert st["done"] == 1 and got[0][34:] == d
    for L in (1473, 1474, 1479, 2953, 2959):                     # last pieces of 1-7 bytes
        pay = bytes(range(256)) * (L // 256) + bytes(L % 256)
        fr = O.tx_frame(O_MAC[0], O_MAC[1], SRC, 1, 0, 0x1027, DST, 0x1127, pay)
        pieces = O.tx_fragment(fr, 1500)
        assert 35 <= len(pieces[-1]) <= 41
        got, _, st = _run(O.FragTable(), pieces, pad=False)
        assert st["done"] == 1 and _same_but_cksum(got[0], fr)


def test_in_and_out_of_order_and_across_calls():
    t = O.FragTable()
    d = udp_datagram(0x1027, 0x1127, bytes(range(200)) * 10)        # 2008 B IP payload
    fs = split(SRC, DST, 7, d, [800, 800, 408])
    got, origin, st = _run(t, [fs[2], fs[0]])
    assert got == [] and st["stored"] == 2
    got, origin, st = _run(t, [ip_frame(SRC, DST, 9, 0, b"x" * 8, True), fs[1]])
    assert len(got) == 1 and origin == [1] and st["done"] == 1
    assert got[0][34:] == d and (got[0][16] << 8 | got[0][17]) == 20 + len(d)
    assert got[0][20] == 0 and got[0][21] == 0


def test_df_kept_mf_cleared():
    t = O.FragTable()
    d = udp_datagram(1, 2, b"a" * 40)
    f0 = ip_frame(SRC, DST, 3, 0, d[:16], True, df=True)
    f1 = ip_frame(SRC, DST, 3, 16, d[16:], False, df=True)
    got, _, st = _run(t, [f0, f1])
    assert st["done"] == 1 and got[0][20] == 0x40 and got[0][21] == 0


def test_duplicate_first_last_and_too_many():
    t = O.FragTable()
    d = udp_datagram(1, 2, b"b" * 56)                                 # 64 B
    fs = split(SRC, DST, 1, d, [16, 16, 16, 16])
    got, _, st = _run(t, [fs[0], fs[0], fs[1], fs[2], fs[3]])
    # the duplicate first errors the flow out; fs[1..3] start a new flow that lacks a first
    assert got == [] and st["errors"] == 1 and st["stored"] == 3
    t = O.FragTable()
    fs5 = split(SRC, DST, 2, d, [8, 8, 16, 16, 16])                   # 5 fragments > 4
    got, _, st = _run(t, fs5)
    assert got == [] and st["errors"] == 1
    t = O.FragTable()
    got, _, st = _run(t, [fs[3], fs[3]])                              # duplicate last
    assert st["errors"] == 1 and st["stored"] == 0


def test_hole_and_size_mismatch():
    t = O.FragTable()
    p = bytes(range(32))
    first = ip_frame(SRC, DST, 4, 0, p[:8], True)
    a = ip_frame(SRC, DST, 4, 16, p[16:24], True)
    b = ip_frame(SRC, DST, 4, 16, p[16:24], True)
    last = ip_frame(SRC, DST, 4, 24, p[24:], False)
    got, _, st = _run(t, [first, a, b, last])                         # sizes add up, 8..16 missing
    assert got == [] and st["holes"] == 1
    t = O.FragTable()
    big = ip_frame(SRC, DST, 5, 8, p[8:32], True)
    got, _, st = _run(t, [ip_frame(SRC, DST, 5, 0, p[:16], True), big,
                          ip_frame(SRC, DST, 5, 24, p[24:], False)])   # overlap: 48 > 32
    assert got == [] and st["errors"] == 1


def test_expiry_and_stale_slot_reuse():
    t = O.FragTable(bucket_num=1, bucket_entries=2, max_cycles=100)
    d = udp_datagram(1, 2, b"c" * 24)                                 # 32 B
    fa = split(SRC, DST, 10, d, [16, 16])
    fb = split(SRC, DST, 11, d, [16, 16])
    fc = split(SRC, DST, 12, d, [16, 16])
    _, _, st = _run(t, [fa[0], fb[0]], tms=0)
    assert st["stored"] == 2
    _, _, st = _run(t, [fc[0]], tms=50)                                # both slots busy, alive
    assert st["no_space"] == 1
    got, _, st = _run(t, [fa[1]], tms=101)                             # fa expired: restarted
    assert got == [] and st["expired"] == 1 and st["stored"] == 1
    got, _, st = _run(t, [fc[0], fc[1]], tms=102)                      # fb stale -> slot reused
    assert len(got) == 1 and got[0][34:] == d and st["expired"] == 1


def test_bad_lengths_dropped():
    t = O.FragTable()
    f = bytearray(ip_frame(SRC, DST, 6, 0, b"z" * 16, True))
    f[16:18] = (20).to_bytes(2, "big")                                 # total_length 20: no data
    g = bytearray(ip_frame(SRC, DST, 6, 0, b"z" * 16, True))
    g[16:18] = (200).to_bytes(2, "big")                                # past the frame
    _, _, st = _run(t, [bytes(f), bytes(g)])
    assert st["frags"] == 2 and st["drop_len"] == 1 and st["drop_short"] == 1


def test_hash_is_dpdk_crc32c():
    # crc32c of 4 zero bytes from a zero seed is 0 for the raw instruction form; the chain below
    # is the restated ipv4_frag_hash and must be deterministic and spread ids over buckets
    s = {O.frag_hash(SRC, DST, i)[0] & 0xFFF0 for i in range(256)}
    assert len(s) > 200
    s1, s2 = O.frag_hash(SRC, DST, 0)
    assert s2 == ((s1 << 7) + (s1 >> 14)) & 0xFFFFFFFF


def test_scenario_covers_every_outcome():
    from reasm_util import scenario
    t = O.FragTable(bucket_num=256, max_cycles=25)
    tot = {}
    for frames, tms in scenario(5):
        _, _, st = _run(t, frames, tms)
        for k, v in st.items():
            tot[k] = tot.get(k, 0) + v
    for k in ("frags", "errors", "holes", "expired", "done", "stored"):
        assert tot[k] > 0, (k, tot)


def _buckets(pid, bucket_num, assoc):
    mask = (bucket_num * assoc - 1) & ~(assoc - 1)
    s1, s2 = O.frag_hash(SRC, DST, pid)
    return {(s1 & mask) // assoc, (s2 & mask) // assoc}


def test_max_entries_lru_rule():
    """ip_frag_find at use_entries == max_entries (DPDK 20.05, restated): a new flow with a free
    slot in its buckets is added only after the LRU list's head (the entry added longest ago) is
    deleted for having expired; otherwise the fragment is dropped (no space). Flow d is chosen
    with buckets no other flow uses, so the stale-slot path cannot be what frees it a slot."""
    B, A = 64, 4
    a, b, c = 21, 22, 23
    used = _buckets(a, B, A) | _buckets(b, B, A) | _buckets(c, B, A)
    d = next(p for p in range(100, 10000) if not (_buckets(p, B, A) & used))
    t = O.FragTable(bucket_num=B, bucket_entries=A, max_cycles=10, max_entries=3)
    dg = udp_datagram(1, 2, b"q" * 24)                                 # 32 B: 2 fragments
    fa, fb, fc, fd = (split(SRC, DST, p, dg, [16, 16]) for p in (a, b, c, d))
    _, _, st = _run(t, [fa[0]], tms=0)
    assert st["stored"] == 1
    _, _, st = _run(t, [fb[0], fc[0]], tms=5)
    assert st["stored"] == 2                                          # 3 entries in use
    _, _, st = _run(t, [fd[0]], tms=9)                                # head a alive: no space
    assert st["no_space"] == 1 and st["stored"] == 0
    _, _, st = _run(t, [fd[0]], tms=11)                               # head a expired: deleted
    assert st["expired"] == 1 and st["stored"] == 1 and st["no_space"] == 0
    got, _, st = _run(t, [fb[1], fa[1]], tms=12)                      # b completes; a starts anew
    assert len(got) == 1 and got[0][34:] == dg
    assert st["done"] == 1 and st["stored"] == 1 and st["expired"] == 0
    got, _, st = _run(t, [fd[1]], tms=13)
    assert len(got) == 1 and st["done"] == 1
    # without the limit (max_entries = 0: the entry count) the first fd[0] is simply stored
    t2 = O.FragTable(bucket_num=B, bucket_entries=A, max_cycles=10)
    _run(t2, [fa[0]], tms=0)
    _run(t2, [fb[0], fc[0]], tms=5)
    _, _, st = _run(t2, [fd[0]], tms=9)
    assert st["stored"] == 1 and st["no_space"] == 0
    with pytest.raises(ValueError):
        O.FragTable(bucket_num=B, bucket_entries=A, max_entries=B * A + 1)


def test_reassembled_checksum_dpdk_mode():
    """flags = UDPDK_FRAG_CKSUM_DPDK: the header checksum is left 0 as ipv4_frag_reassemble writes
    it (the reference's "TODO must fix the IP header checksum", udpdk_poller.c:355-360); every
    other byte equals the default mode's output, whose checksum is the RFC 1071 value."""
    dg = udp_datagram(1, 2, bytes(range(200)))
    fr = split(SRC, DST, 31, dg, [104, 104])
    g0, _, _ = _run(O.FragTable(), fr)
    g1, _, _ = _run(O.FragTable(flags=1), fr)
    assert len(g0) == len(g1) == 1
    assert g1[0][24:26] == b"\0\0" and g0[0][24:26] != b"\0\0"
    assert _same_but_cksum(g0[0], g1[0])
