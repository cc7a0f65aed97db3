"""The reference's socket surface over the GPU datapath (udpdk_api.h, -m gpu):

* TX: udpdk_sendto queues, udpdk_tx_drain builds the frames on the GPU in the poller's order
  (udpdk_poller.c:453-514) — the §8.G golden vectors V1-V5, the fragmentation of datagrams
  longer than the MTU against the oracle's restatement, the per-socket burst order, partial drains;
* RX: udpdk_poll_rx admits each socket's deliveries per burst of 128 frames, all-or-nothing
  (flush_rx_queue, :274-292), into rings recvfrom reads, with payloads gathered on the GPU;
* both halves driven by the poller thread against the built-in loopback port, while the test
  thread calls sendto / recvfrom (SP/SC rings across threads)."""
import ctypes as C
import json
import os
import threading

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SRC_MAC, DST_MAC, SRC_IP = "68:05:ca:95:f8:ec", "68:05:ca:95:fa:64", "172.31.100.2"


@pytest.fixture()
def api(tmp_path, host_api, request):
    """udpdk_init over a test ini; indirect parametrization sets [gpu] poll_threads (an int) or
    adds [gpu] lines (a str)."""
    param = getattr(request, "param", None)
    threads = param if isinstance(param, int) else None
    extra = param if isinstance(param, str) else ""
    ini = tmp_path / "udpdk.ini"
    ini.write_text(f"[port0]\nmac_addr = {SRC_MAC}\nip_addr = {SRC_IP}\n"
                   f"[port0_dst]\nmac_addr = {DST_MAC}\n"
                   "[gpu]\ndevice = 0\nmax_frames = 65536\nmax_lanes = 64\n"
                   "frag_buckets = 64\nfrag_bucket_entries = 16\nfrag_max_dgram = 16384\n"
                   + (f"poll_threads = {threads}\n" if threads else "") + extra)
    L = abi.lib()
    argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
    assert L.udpdk_init(3, argv) == 0
    yield host_api
    L.udpdk_cleanup()


def _payload(n, seed=0):
    return bytes(np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8))


def _tx_expected(slot_ip, slot_port, dst, port, payload, mtu=1500):
    fr = O.tx_frame(bytes.fromhex(SRC_MAC.replace(":", "")), bytes.fromhex(DST_MAC.replace(":", "")),
                    abi.raw_ip(SRC_IP), 1, slot_ip, slot_port, abi.raw_ip(dst), abi.raw_port(port), payload)
    return O.tx_fragment(fr, mtu) if len(fr) > mtu else [fr]


def test_tx_golden_vectors_through_sendto(api):
    """§8.G V1-V5 (the reference's udpdk_sendto output) through sendto -> tx_drain on the GPU."""
    with open(os.path.join(HERE, "tx_vectors.json")) as f:
        g = json.load(f)
    cfg = g["config"]
    for v in g["vectors"]:
        api.reset()
        api.config_set(bytes.fromhex(cfg["src_mac"]), bytes.fromhex(cfg["dst_mac"]), cfg["src_ip"])
        for step in v["setup"]:
            if step[0] == "socket":
                assert api.socket() >= 0
            elif step[0] == "bind":
                assert api.bind(step[1], step[2], step[3]) == 0
            elif step[0] == "autobind":
                assert api.sendto(step[1], b"x", "172.31.100.1", 10001) == 1
                assert len(api.tx_drain()) == 1
        pl = bytes((i * 7 + 3) & 0xFF for i in range(v["send"]["len"]))
        assert api.sendto(v["send"]["sock"], pl, v["send"]["dst"], v["send"]["port"]) == len(pl)
        frames = api.tx_drain()
        assert len(frames) == 1, v["id"]
        assert len(frames[0]) == v["pkt_len"], v["id"]
        assert frames[0][:42].hex() == v["hdr"], v["id"]
        assert frames[0][42:] == pl, v["id"]


@pytest.mark.parametrize("mtu", [1500, 1020])
def test_tx_fragmentation_through_sendto(api, mtu):
    """Datagrams around and far past the MTU: the poller fragments frames longer than the MTU
    (pkt_len > IPV4_MTU_DEFAULT, poller.c:461-501); frames equal the oracle's restatement."""
    assert abi.lib().udpdk_config_mtu(mtu) == 0
    s = api.socket()
    assert api.bind(s, "10.1.2.3", 5353) == 0
    lens = [0, 1, 1458, 1459, 1472, 1473, 2000, 2006, 2007, 8000, 65507]
    want = []
    for i, n in enumerate(lens):
        pl = _payload(n, i)
        assert api.sendto(s, pl, "172.31.100.1", 10001) == n
        want += _tx_expected(abi.raw_ip("10.1.2.3"), abi.raw_port(5353), "172.31.100.1", 10001, pl, mtu)
    got = api.tx_drain(max_frames=4096, cap=1 << 21)
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a == b, i
    assert api.tx_pending() == 0


def _poller_drain(q, max_frames, nfrag):
    """Model of one udpdk_tx_drain call: the poller's TX loop (udpdk_poller.c:452-507) from
    socket 0 with an empty burst: sockets in index order, each dequeued while the burst holds
    < 128 frames, flush at >= 128, repeated until the rings are empty or the next datagram's
    frames would pass max_frames. Mutates q."""
    order, burst, frames = [], 0, 0
    while any(q.values()):
        for s in sorted(q):
            while burst < 128 and q[s]:
                nf = nfrag(q[s][0])
                if frames + nf > max_frames:
                    return order
                order.append((s, q[s].pop(0)))
                burst += nf
                frames += nf
            if burst >= 128:
                burst = 0
        burst = 0
    return order


def test_tx_poller_order_and_partial_drains(api):
    socks = [api.socket() for _ in range(3)]
    for i, s in enumerate(socks):
        assert api.bind(s, "0.0.0.0", 20000 + i) == 0
    queues = {s: [] for s in socks}
    rng = np.random.default_rng(3)
    for k in range(600):
        s = socks[int(rng.integers(0, 3))]
        n = int(rng.choice([10, 100, 3000]))               # 3000 B -> 3 fragments at MTU 1500
        pl = bytes([s, k & 0xFF, k >> 8]) + b"\0" * (n - 3)
        assert api.sendto(s, pl, "172.31.100.1", 10001) == n
        queues[s].append((k, n))
    span = abi.lib().udpdk_gpu_tx_span

    def nf(item):
        c = C.c_uint32()
        span(item[1], 1500, C.byref(c))
        return c.value
    q = {s: list(v) for s, v in queues.items()}
    want, got = [], []
    while api.tx_pending():
        frames = api.tx_drain(max_frames=97, cap=1 << 20)     # partial drains: whole datagrams only
        assert frames and len(frames) <= 97
        want += _poller_drain(q, 97, nf)
        got += frames
    # first fragment (or the frame) of each datagram names its socket and sequence number
    firsts = [f for f in got if (int.from_bytes(f[20:22], "big") & 0x1FFF) == 0]
    seq = [(f[42], f[43] | f[44] << 8) for f in firsts]
    assert seq == [(s, k) for s, (k, _) in want]
    assert len(got) == sum(nf(it) for v in queues.values() for it in v)


def _rx_batch(ports, size=64, seed=5):
    b = F.build_frames(np.full(len(ports), size, np.uint32), np.asarray(ports, np.uint32), seed)
    return b


def _poll(b):
    st = abi.RxStats()
    rc = abi.lib().udpdk_poll_rx(b.frames.ctypes.data, b.frames_bytes, b.offset.ctypes.data,
                                 b.length.ctypes.data, None, b.n, C.byref(st))
    assert rc == 0
    return st


def _admitted(idx, room):
    """flush_rx_queue's model: per burst of 128 frame indices, all-or-nothing into the ring."""
    acc = []
    for burst in range(0, (max(idx) if idx else 0) + 128, 128):
        grp = [i for i in idx if burst <= i < burst + 128]
        if grp and len(grp) <= room:
            acc += grp
            room -= len(grp)
    return acc


@pytest.mark.parametrize("api", [1, 3, 8, 32, "poll_threads = 3\npoll_chunk_mb = 1\npoll_chunk_min_avg = 0\n"], indirect=True)
def test_rx_many_sockets_over_poll_threads(api):
    """40 sockets, Zipf-skewed destination ports, some rings partly full before the poll: the
    admission and ring publication split the sockets over 1, 3, 8 or 32 threads (sockets
    straddle the parts' boundaries; at 32 most parts hold one socket or none, the Zipf head
    filling several parts' share alone) and every socket still gets exactly its admitted
    bursts, in order. (poll_chunk_mb = 1: the pipelined poll, the batch cut into chunks.)"""
    ns = 40
    socks = [api.socket() for _ in range(ns)]
    for k, s in enumerate(socks):
        assert api.bind(s, "0.0.0.0", 11000 + k) == 0
    pre = {0: 1500, 3: 2000, 7: 300}
    for k, m in pre.items():
        _poll(_rx_batch([11000 + k] * m, seed=10 + k))
    rng = np.random.default_rng(21)
    ports = 11000 + np.minimum(rng.zipf(1.3, 30000) - 1, ns - 1)
    b = _rx_batch(ports, size=int(rng.integers(60, 300)), seed=3)
    _poll(b)
    L = abi.lib()
    for k, s in enumerate(socks):
        idx = [int(i) for i in np.nonzero(ports == 11000 + k)[0]]
        want = _admitted(idx, 2047 - pre.get(k, 0))
        for _ in range(pre.get(k, 0)):
            assert api.recvfrom(s, 4096)[0] > 0
        for i in want:
            n, data, _ = api.recvfrom(s, 4096)
            o, ln = int(b.offset[i]), int(b.length[i])
            assert data == bytes(b.frames[o + 42:o + ln]), (k, i)
    L.udpdk_interrupt(0)
    assert all(api.recvfrom(s, 64)[0] == -1 for s in socks)


@pytest.mark.parametrize("api", [None, 3, "poll_threads = 3\nhost_copy_min = 1\n"], indirect=True)
def test_rx_burst_admission_and_payloads(api):
    """A socket gets more deliveries in one poll than its ring holds, with the ring partly full:
    each burst of 128 frames is admitted whole or dropped whole (poller.c:287-290); payloads and
    source addresses come from the GPU gather, or (host_copy_min = 1) from the host copy out of
    the caller's frames."""
    s0, s1 = api.socket(), api.socket()
    assert api.bind(s0, "0.0.0.0", 10001) == 0 and api.bind(s1, "0.0.0.0", 10002) == 0
    pre = _rx_batch([10001] * 700, seed=1)
    _poll(pre)
    rng = np.random.default_rng(9)
    ports = np.where(rng.random(6000) < 0.7, 10001, 10002)
    b = _rx_batch(ports, size=int(rng.integers(60, 200)), seed=2)
    _poll(b)
    # model: ring room 2047 - 700; bursts = frame index // 128
    room, acc0 = 2047 - 700, []
    idx0 = np.nonzero(ports == 10001)[0]
    for burst in range(0, 6000, 128):
        grp = [int(i) for i in idx0 if burst <= i < burst + 128]
        if len(grp) <= room:
            acc0 += grp
            room -= len(grp)
    idx1 = [int(i) for i in np.nonzero(ports == 10002)[0]]
    acc1 = []
    room1 = 2047
    for burst in range(0, 6000, 128):
        grp = [i for i in idx1 if burst <= i < burst + 128]
        if len(grp) <= room1:
            acc1 += grp
            room1 -= len(grp)

    def payload(batch, i):
        o, n = int(batch.offset[i]), int(batch.length[i])
        return bytes(batch.frames[o + 42:o + n])
    for i in range(700):
        n, data, addr = api.recvfrom(s0, 4096)
        assert data == payload(pre, i) and addr == ("172.31.100.2", 10000)
    for i in acc0:
        n, data, _ = api.recvfrom(s0, 4096)
        assert data == payload(b, i), i
    for i in acc1:
        n, data, _ = api.recvfrom(s1, 4096)
        assert data == payload(b, i), i
    # nothing else is queued: a non-blocking probe through the interrupt flag
    L = abi.lib()
    L.udpdk_interrupt(0)
    assert api.recvfrom(s0, 64)[0] == -1 and api.recvfrom(s1, 64)[0] == -1
    assert len(acc0) < len(idx0)                          # the model really dropped bursts


def test_two_threads_poller_and_app_over_loopback(api):
    """udpdk_port_attach starts the poller thread (TX drain -> port -> RX poll); the test thread
    only calls sendto and recvfrom, as an application on the reference would."""
    L = abi.lib()
    ops = abi.PortOps()
    assert L.udpdk_port_loopback(C.byref(ops)) == 0
    ops.batch_frames = 512
    a, b = api.socket(), api.socket()
    assert api.bind(a, "0.0.0.0", 10000) == 0 and api.bind(b, "0.0.0.0", 10001) == 0
    assert L.udpdk_port_attach(C.byref(ops)) == 0
    watchdog = threading.Timer(60.0, L.udpdk_interrupt, [0])   # a hang ends as EINTR
    watchdog.start()
    try:
        sent = []
        for k in range(3000):
            pl = _payload(int(k % 1400) + 1, k)
            while api.sendto(a, pl, SRC_IP, 10001) < 0:      # TX ring full: the poller drains it
                assert api.errno() == 105                     # ENOBUFS
            sent.append(pl)
            if k % 500 == 499:                                # let the consumer keep up
                for want in sent[k - 499:k + 1]:
                    n, data, addr = api.recvfrom(b, 2048)
                    assert n == len(want) and data == want and addr == (SRC_IP, 10000)
        # fragmented on TX (4 fragments at MTU 1500), reassembled on RX; DPDK's table takes at
        # most RTE_LIBRTE_IP_FRAG_MAX_FRAG = 4 fragments per datagram, so a larger one would be
        # dropped there as in the reference
        big = _payload(5000, 77)
        assert api.sendto(a, big, SRC_IP, 10001) == 5000
        n, data, addr = api.recvfrom(b, 16384)
        assert n == 5000 and data == big and addr == (SRC_IP, 10000)
    finally:
        watchdog.cancel()
        assert L.udpdk_port_detach() == 0


def test_autobind_sendto_while_poller_runs(api):
    """A sendto that auto-binds its socket (or a close + socket + bind) while the poller thread
    drains TX: every frame carries the source port the socket had when its datagram was queued,
    never the slot row of the previous owner or of the unbound socket (udpdk_tx_drain takes the
    TX lock before it releases the table lock that covers its slot-table refresh)."""
    L = abi.lib()
    ops = abi.PortOps()
    assert L.udpdk_port_loopback(C.byref(ops)) == 0
    ops.batch_frames = 256
    rcv, hold = api.socket(), api.socket()
    assert api.bind(rcv, "0.0.0.0", 10001) == 0
    assert api.bind(hold, "0.0.0.0", 0) == 0         # raw port 0 taken: auto-bind gets raw 1 (256)
    assert L.udpdk_port_attach(C.byref(ops)) == 0
    watchdog = threading.Timer(60.0, L.udpdk_interrupt, [0])
    watchdog.start()
    try:
        for k in range(400):
            s = api.socket()
            want = 256
            if k % 2:
                want = 12000 + k
                assert api.bind(s, "0.0.0.0", want) == 0
            pl = bytes([k & 0xFF, k >> 8]) * 4
            assert api.sendto(s, pl, SRC_IP, 10001) == 8
            n, data, addr = api.recvfrom(rcv, 64)
            assert (n, data, addr) == (8, pl, (SRC_IP, want)), k
            assert api.close(s) == 0
    finally:
        watchdog.cancel()
        assert L.udpdk_port_detach() == 0


@pytest.mark.parametrize("api", ["slab_bytes_max = 606208\nslab_count_max = 2\n"], indirect=True)
def test_slab_budget_drops_polls_like_an_exhausted_pool(api):
    """Payload slabs are pinned host memory held until every datagram in them is received: with
    the budget at two slabs, a third poll while both are held is dropped whole (rx_nobufs, as
    rte_eth_rx_burst returns nothing from an exhausted mempool); once one slab's datagrams are
    read it is reused. Slab footprint here: 4096 slots x 64 B + 10 B per slot = 303,104 B."""
    socks = [api.socket() for _ in range(4)]
    for k, s in enumerate(socks):
        assert api.bind(s, "0.0.0.0", 10001 + k) == 0
    batches = [_rx_batch([10001 + k] * 1000, seed=40 + k) for k in range(4)]
    _poll(batches[0])
    _poll(batches[1])
    assert api.rx_nobufs() == 0
    _poll(batches[2])                                   # both slabs held: dropped
    assert api.rx_nobufs() == 1000
    for i in range(1000):
        n, data, _ = api.recvfrom(socks[0], 2048)
        o, ln = int(batches[0].offset[i]), int(batches[0].length[i])
        assert data == bytes(batches[0].frames[o + 42:o + ln])
    _poll(batches[3])                                   # slab 0 is free again
    assert api.rx_nobufs() == 1000
    for k in (1, 3):
        for i in range(1000):
            n, data, _ = api.recvfrom(socks[k], 2048)
            o, ln = int(batches[k].offset[i]), int(batches[k].length[i])
            assert data == bytes(batches[k].frames[o + 42:o + ln])
    abi.lib().udpdk_interrupt(0)
    assert api.recvfrom(socks[2], 64)[0] == -1          # the dropped poll left nothing queued


def test_tx_datagram_larger_than_any_drain_is_dropped(api):
    """A queued datagram that needs more frames than the drain's limit (8000 B = 6 fragments at
    MTU 1500, max_frames 4) can never be carried: it is dropped and counted instead of blocking
    its socket's ring forever; the datagrams behind it still go out."""
    s = api.socket()
    assert api.bind(s, "0.0.0.0", 10000) == 0
    assert api.sendto(s, _payload(8000, 1), "172.31.100.1", 10001) == 8000
    small = _payload(100, 2)
    assert api.sendto(s, small, "172.31.100.1", 10001) == 100
    frames = api.tx_drain(max_frames=4, cap=1 << 16)
    assert api.tx_dropped() == 1 and api.tx_pending() == 0
    assert len(frames) == 1 and frames[0][42:] == small


@pytest.mark.parametrize("api", ["poll_chunk_mb = 1\npoll_chunk_min_avg = 0\nslab_count_max = 3\n"], indirect=True)
def test_chunked_poll_slab_budget_keeps_payloads(api):
    """The pipelined poll (1 MiB chunks) over direct datagrams to 8 sockets and 2-fragment ones
    to a ninth, with the slab budget at three: the first chunk holds two slabs (direct and
    reassembled payloads), so a later chunk gets at most one of its two and is dropped whole
    (it used to drop after queueing its direct gather, which then raced the next
    chunk's use of the same buffers). Every datagram a socket receives is byte-identical to one
    sent to it, in send order; the dropped ones are counted in rx_nobufs."""
    ports = list(range(10002, 10010))
    socks = {p: api.socket() for p in [10001] + ports}
    for p, s in socks.items():
        assert api.bind(s, "0.0.0.0", p) == 0
    rng = np.random.default_rng(61)
    nd, nfr, L = 3000, 700, 2910
    direct = F.build_frames(np.full(nd, 1000, np.uint32), rng.choice(ports, nd).astype(np.uint32), 62)
    frag = F.frag_batch(nfr, L, 1500, seed=63)
    whole = F.build_frames(np.full(nfr, L + 42, np.uint32), np.full(nfr, 10001, np.uint32), 63)
    order = rng.permutation(np.r_[np.zeros(nd, int), np.ones(nfr, int)])
    buf, offs, lens = bytearray(), [], []
    sent = {p: [] for p in socks}
    di = fi = 0
    for kind in order:
        if kind == 0:
            o, ln = int(direct.offset[di]), int(direct.length[di])
            port = int(direct.frames[o + 36]) << 8 | int(direct.frames[o + 37])
            sent[port].append(bytes(direct.frames[o + 42:o + ln]))
            offs.append(len(buf)), lens.append(ln)
            buf += bytes(direct.frames[o:o + ln])
            di += 1
        else:
            for j in (2 * fi, 2 * fi + 1):
                o, ln = int(frag.offset[j]), int(frag.length[j])
                offs.append(len(buf)), lens.append(ln)
                buf += bytes(frag.frames[o:o + ln])
            sent[10001].append(bytes(whole.frames[fi * (L + 42) + 42:(fi + 1) * (L + 42)]))
            fi += 1
    fr = np.zeros(len(buf) + 256, np.uint8)
    fr[:len(buf)] = np.frombuffer(bytes(buf), np.uint8)
    b = F.Batch(fr, np.array(offs, np.uint32), np.array(lens, np.uint16), len(buf))
    _poll(b)
    dropped = api.rx_nobufs()
    assert dropped > 0
    abi.lib().udpdk_interrupt(0)                       # recvfrom returns -1 once a ring is empty
    got = 0
    for p, s in socks.items():
        want = {d: i for i, d in enumerate(sent[p])}
        last = -1
        while True:
            n, data, _ = api.recvfrom(s, 4096)
            if n < 0:
                break
            assert data in want, (p, n)
            assert want[data] > last, p
            last = want[data]
            got += 1
    assert got + dropped == nd + nfr
