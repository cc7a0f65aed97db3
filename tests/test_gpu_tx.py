"""TX parity: udpdk_gpu_tx_build against the oracle's restatement of udpdk_sendto and the
survey's golden vectors; frames packed back to back at arbitrary alignment."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi

pytestmark = pytest.mark.gpu

SRC_MAC = bytes.fromhex("6805ca95f8ec")
DST_MAC = bytes.fromhex("6805ca95fa64")
SRC_IP = abi.raw_ip("172.31.100.2")


def _tx_gpu(ctx, slots, sock, dst_ip, dst_port, payloads, frame_off, frames_cap, mtu=None, exact=False):
    """exact: payload_bytes ends at the last payload's last byte and the payload allocation is
    exactly payload_bytes + UDPDK_GPU_FRAMES_TAILROOM (the contract of udpdk_tx_batch_t)."""
    n = len(payloads)
    pay_off = np.zeros(n, np.uint32)
    pos = 0
    for i, p in enumerate(payloads):
        pay_off[i] = pos
        pos += len(p) + int(i % 3)                       # unaligned payload starts
    if exact:
        pos = int(pay_off[-1]) + len(payloads[-1])
    pay = np.zeros(pos + (abi.FRAMES_TAILROOM if exact else 256), np.uint8)
    for i, p in enumerate(payloads):
        pay[pay_off[i]:pay_off[i] + len(p)] = np.frombuffer(p, np.uint8)
    lens = np.array([len(p) for p in payloads], np.uint16)
    hs = abi.snapshot_from_lists({}, 1, slots=slots)
    ctx.upload_snapshot(hs)
    bufs = [ctx.upload(pay), ctx.upload(pay_off), ctx.upload(lens), ctx.upload(np.array(sock, np.int32)),
            ctx.upload(np.array(dst_ip, np.uint32)), ctx.upload(np.array(dst_port, np.uint16)),
            ctx.upload(np.array(frame_off, np.uint32))]
    out = ctx.alloc(frames_cap)
    abi.lib().udpdk_gpu_memset(ctx.handle, C.c_void_p(out.ptr), 0xEE, frames_cap)
    cfg = abi.TxConfig((C.c_uint8 * 6)(*SRC_MAC), (C.c_uint8 * 6)(*DST_MAC), SRC_IP)
    bt = abi.TxBatch(bufs[0].ptr, pos, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, bufs[4].ptr, bufs[5].ptr, n)
    ot = abi.TxOut(out.ptr, frames_cap, bufs[6].ptr)
    if mtu is None:
        rc = abi.lib().udpdk_gpu_tx_build(ctx.handle, C.byref(cfg), C.byref(bt), C.byref(ot))
    else:
        rc = abi.lib().udpdk_gpu_tx_build_mtu(ctx.handle, C.byref(cfg), C.byref(bt), C.byref(ot), mtu)
    assert rc == 0
    res = ctx.download(out, np.uint8, frames_cap)
    for b in bufs + [out]:
        b.free()
    return res


def test_tx_random_batch(gpu_ctx):
    rng = np.random.default_rng(3)
    n_slots = 64
    slots = []
    for s in range(n_slots):
        kind = s % 3
        if kind == 0:
            slots.append((0, int(rng.integers(0, 65536)), 1))                      # bound ANY
        elif kind == 1:
            slots.append((int(rng.integers(1, 2**32)), int(rng.integers(0, 65536)), 1))  # specific
        else:
            slots.append((int(rng.integers(1, 2**32)), int(rng.integers(0, 65536)), 0))  # unbound
    n = 3000
    lens = rng.integers(0, 1459, n)
    lens[:20] = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 15, 16, 17, 1457, 1458, 31, 32, 33, 100]
    payloads = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    sock = rng.integers(0, n_slots, n)
    dip = rng.integers(0, 2**32, n, dtype=np.uint64)
    dport = rng.integers(0, 65536, n)
    # back-to-back frames starting at offset 5 (frame boundaries share 16-byte chunks)
    fo = np.zeros(n, np.uint32)
    pos = 5
    for i in range(n):
        fo[i] = pos
        pos += int(lens[i]) + 42
    cap = pos + 64
    res = _tx_gpu(gpu_ctx, slots, sock, dip, dport, payloads, fo, cap)
    assert np.all(res[:5] == 0xEE) and np.all(res[pos:pos + 32] == 0xEE)
    for i in range(n):
        ip, port, bound = slots[sock[i]]
        want = O.tx_frame(SRC_MAC, DST_MAC, SRC_IP, bound, ip, port, int(dip[i]), int(dport[i]), payloads[i])
        got = res[fo[i]:fo[i] + len(want)].tobytes()
        assert got == want, f"frame {i} len {lens[i]} off {fo[i]}"


@pytest.mark.parametrize("gap", [0, 3])
def test_tx_small_frames(gpu_ctx, gap):
    """Waves whose frames are all <= 80 bytes take the lane-per-frame path (tx_small): every
    payload length 0-38 at odd payload and frame offsets, frames back to back (gap 0: frame ends
    share 16-byte pieces with the next frame) or with 3 untouched bytes between them; some waves
    carry one larger frame (the chunk-sweep path) and some lanes an invalid socket (no frame)."""
    rng = np.random.default_rng(11 + gap)
    slots = [(0, 10000, 1), (abi.raw_ip("10.1.2.3"), 5353, 1), (abi.raw_ip("10.9.9.9"), 7, 0)]
    n = 64 * 40 + 17
    lens = rng.integers(0, 39, n)
    lens[:39] = np.arange(39)
    for g in range(0, n // 64, 3):                     # every third wave: one 300-byte frame
        lens[g * 64 + int(rng.integers(0, 64))] = 300
    payloads = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    sock = rng.integers(0, 3, n)
    sock[rng.integers(0, n, 20)] = 7                    # out of range: nothing written
    dip = rng.integers(0, 2**32, n, dtype=np.uint64)
    dport = rng.integers(0, 65536, n)
    fo = np.zeros(n, np.uint32)
    pos = 7
    for i in range(n):
        fo[i] = pos
        pos += int(lens[i]) + 42 + gap
    cap = pos + 64
    res = _tx_gpu(gpu_ctx, slots, sock, dip, dport, payloads, fo, cap)
    want_buf = np.full(cap, 0xEE, np.uint8)
    for i in range(n):
        if sock[i] >= len(slots):
            continue
        ip, port, bound = slots[sock[i]]
        want = O.tx_frame(SRC_MAC, DST_MAC, SRC_IP, bound, ip, port, int(dip[i]), int(dport[i]), payloads[i])
        want_buf[fo[i]:fo[i] + len(want)] = np.frombuffer(want, np.uint8)
    bad = np.nonzero(res != want_buf)[0]
    assert bad.size == 0, f"first differing byte {bad[0]} (frame {np.searchsorted(fo, bad[0], 'right') - 1})"


@pytest.mark.parametrize("start", [0, 1, 2, 3])
def test_tx_payload_ends_at_payload_bytes(gpu_ctx, start):
    """The batch's last payload ends exactly at payload_bytes at every dword alignment, lengths
    1-40 (so its last bytes come from a dword that ends past payload_bytes), the allocation being
    exactly payload_bytes + tailroom: every byte is copied (udpdk_tx_drain packs payloads like
    this; a range rounded to 16 bytes returned those dwords as zeros)."""
    for last in range(1, 41):
        payloads = [bytes(range(1, 1 + start))] if start else []
        payloads += [bytes((7 * k + last) & 0xFF or 1 for k in range(last))]
        n = len(payloads)
        fo = np.cumsum([0] + [len(p) + 42 for p in payloads[:-1]]).astype(np.uint32)
        cap = int(fo[-1]) + len(payloads[-1]) + 42 + 64
        res = _tx_gpu(gpu_ctx, [(0, 10000, 1)], [0] * n, [abi.raw_ip("10.0.0.9")] * n, [4242] * n,
                      payloads, fo, cap, exact=True)
        for i, p in enumerate(payloads):
            want = O.tx_frame(SRC_MAC, DST_MAC, SRC_IP, 1, 0, 10000, abi.raw_ip("10.0.0.9"), 4242, p)
            got = res[fo[i]:fo[i] + len(want)].tobytes()
            assert got == want, (start, last, i)


def test_tx_golden_vectors(gpu_ctx):
    with open(os.path.join(os.path.dirname(__file__), "golden", "tx_vectors.json")) as f:
        g = json.load(f)
    slots = [(0, abi.raw_port(10000), 1), (abi.raw_ip("10.1.2.3"), abi.raw_port(5353), 1),
             (0, 0, 1), (0, 1, 1)]    # s2/s3 after auto-bind to raw ports 0 and 1 (V4, V5)
    vs = g["vectors"]
    payloads = [bytes((i * 7 + 3) & 0xFF for i in range(v["send"]["len"])) for v in vs]
    fo = np.cumsum([0] + [len(p) + 42 for p in payloads[:-1]]).astype(np.uint32)
    res = _tx_gpu(gpu_ctx, slots, [v["send"]["sock"] for v in vs],
                  [abi.raw_ip(v["send"]["dst"]) for v in vs],
                  [abi.raw_port(v["send"]["port"]) for v in vs], payloads, fo,
                  int(fo[-1]) + len(payloads[-1]) + 42 + 64)
    for i, v in enumerate(vs):
        fr = res[fo[i]:fo[i] + v["pkt_len"]].tobytes()
        assert fr[:42].hex() == v["hdr"], v["id"]
        assert fr[42:] == payloads[i]


@pytest.mark.parametrize("mtu", [1500, 1020])
def test_tx_fragmentation(gpu_ctx, mtu):
    """udpdk_gpu_tx_build_mtu against the poller's fragmentation restated (oracle_tx_fragment):
    unfragmented, single-'fragment' (pkt_len in (mtu, mtu + 14]), 2-fragment and 45-fragment
    datagrams mixed, frames back to back from an unaligned start."""
    rng = np.random.default_rng(11)
    slots = [(0, abi.raw_port(10000), 1), (abi.raw_ip("10.1.2.3"), abi.raw_port(5353), 1)]
    n = 700
    lens = rng.integers(0, 4000, n)
    lens[:16] = [0, 1, mtu - 42, mtu - 41, mtu - 28, mtu - 27, 2006, 2952, 2953, 65507, 8, 9,
                 mtu - 29, 2 * (mtu - 20) - 8, 2 * (mtu - 20) - 7, 1458]
    lens[rng.integers(16, n, 5)] = rng.integers(20000, 65508, 5)
    payloads = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    sock = rng.integers(0, 2, n)
    dip = rng.integers(0, 2**32, n, dtype=np.uint64)
    dport = rng.integers(0, 65536, n)
    fo = np.zeros(n, np.uint32)
    pos = 3
    for i in range(n):
        fo[i] = pos
        pos += int(abi.lib().udpdk_gpu_tx_span(int(lens[i]), mtu, None))
    cap = pos + 64
    res = _tx_gpu(gpu_ctx, slots, sock, dip, dport, payloads, fo, cap, mtu=mtu)
    assert np.all(res[:3] == 0xEE) and np.all(res[pos:pos + 32] == 0xEE)
    for i in range(n):
        ip, port, bound = slots[sock[i]]
        frame = O.tx_frame(SRC_MAC, DST_MAC, SRC_IP, bound, ip, port, int(dip[i]), int(dport[i]),
                           payloads[i])
        want = b"".join(O.tx_fragment(frame, mtu))
        got = res[fo[i]:fo[i] + len(want)].tobytes()
        assert got == want, f"datagram {i} len {lens[i]}"

