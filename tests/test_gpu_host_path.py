"""The reference's socket surface end to end on the GPU: udpdk_init (config file), bind,
udpdk_poll_rx (the poller's RX half: GPU classify/demux, device reassembly of IPv4 fragments,
per-socket rings in the reference's order) and udpdk_recvfrom; a reassembled datagram arrives at
the position of the fragment that completed it (udpdk_poller.c:338-412), across poll calls."""
import ctypes as C

import numpy as np
import pytest

from reasm_util import batch, ip_frame, raw_ip, split, udp_datagram
from udpdk_amd import abi

pytestmark = pytest.mark.gpu


def _port(p):
    return int.from_bytes(p.to_bytes(2, "big"), "little")


@pytest.mark.parametrize("threads", [None, 2])
def test_poll_rx_delivers_reassembled_datagrams_in_order(tmp_path, host_api, threads):
    """(threads = 2: each socket's admission, with its reassembled datagrams merged in, runs on
    its own thread of the poll pool)"""
    ini = tmp_path / "udpdk.ini"
    ini.write_text("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n"
                   "[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n"
                   "[gpu]\ndevice = 0\nmax_frames = 65536\nmax_lanes = 16\n"
                   "frag_buckets = 16\nfrag_bucket_entries = 16\nfrag_max_dgram = 16384\n"
                   + (f"poll_threads = {threads}\n" if threads else ""))
    L = abi.lib()
    argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
    assert L.udpdk_init(3, argv) == 0
    try:
        s0, s1 = host_api.socket(), host_api.socket()
        assert host_api.bind(s0, "0.0.0.0", 10001) == 0
        assert host_api.bind(s1, "0.0.0.0", 10002) == 0
        src, dst = raw_ip("10.9.8.7"), raw_ip("172.31.100.1")

        def plain(port, payload, pid):
            return ip_frame(src, dst, pid, 0, udp_datagram(_port(4000), _port(port), payload), False)
        d1 = udp_datagram(_port(4000), _port(10001), bytes(range(256)) * 12)        # 3080 B
        d2 = udp_datagram(_port(4000), _port(10002), bytes(range(100, 200)) * 20)   # 2008 B
        f1 = split(src, dst, 77, d1, [1480, 1480, 120])
        f2 = split(src, dst, 78, d2, [1480, 528])
        b1 = [plain(10001, b"A" * 10, 1), f1[2], plain(10002, b"B" * 20, 2), f1[0],
              plain(10001, b"C" * 30, 3), f2[1]]
        b2 = [f1[1], plain(10001, b"D" * 40, 4), f2[0], plain(10002, b"E" * 50, 5)]
        for fr in (b1, b2):
            buf, off, ln = batch(fr)
            st = abi.RxStats()
            assert L.udpdk_poll_rx(buf.ctypes.data, len(buf) - 64, off.ctypes.data, ln.ctypes.data,
                                   None, len(off), C.byref(st)) == 0
        want0 = [b"A" * 10, b"C" * 30, d1[8:], b"D" * 40]      # d1 completes at b2[0]
        want1 = [b"B" * 20, d2[8:], b"E" * 50]                 # d2 completes at b2[2]
        for s, want in ((s0, want0), (s1, want1)):
            for w in want:
                n, data, addr = host_api.recvfrom(s, 8192)
                assert n == len(w) and data == w, (s, n)
                assert addr == ("10.9.8.7", 4000)
    finally:
        L.udpdk_cleanup()


def test_poll_rx_inplace_reassembly_keeps_aliased_frames(tmp_path, host_api):
    """A burst whose fragments sit back to back (in-place reassembly would close the datagram up
    in the staged buffer) and a direct frame whose descriptor aliases the second fragment's data:
    udpdk_poll_rx only reassembles in place when the burst's frames are disjoint, so the aliased
    frame's payload is delivered as it was received, next to the reassembled datagram.
    A disjoint burst of the same fragments takes the in-place pass and delivers the same."""
    ini = tmp_path / "udpdk.ini"
    ini.write_text("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n"
                   "[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n"
                   "[gpu]\ndevice = 0\nmax_frames = 65536\nmax_lanes = 16\n"
                   "frag_buckets = 16\nfrag_bucket_entries = 16\nfrag_max_dgram = 16384\n")
    L = abi.lib()
    argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
    assert L.udpdk_init(3, argv) == 0
    try:
        s0, s1 = host_api.socket(), host_api.socket()
        assert host_api.bind(s0, "0.0.0.0", 10001) == 0
        assert host_api.bind(s1, "0.0.0.0", 10002) == 0
        src, dst = raw_ip("10.9.8.7"), raw_ip("172.31.100.1")

        def plain(port, payload, pid):
            return ip_frame(src, dst, pid, 0, udp_datagram(_port(4000), _port(port), payload), False)
        for aliased in (True, False):
            inner = plain(10002, bytes(range(40, 100)), 9)          # a whole frame, 102 B
            pay = bytes([0x5A]) * 1500 + inner + bytes([0xA5]) * 1500
            d1 = udp_datagram(_port(4000), _port(10001), pay)
            f1 = split(src, dst, 77 + aliased, d1, [1480, 1480, len(d1) - 2960])
            frames = [plain(10001, b"A" * 10, 1), f1[0], f1[1], f1[2]]
            if not aliased:
                frames.append(inner)
            buf, off, ln = batch(frames)
            if aliased:
                # the inner frame inside fragment 1's data: datagram byte 8 + 1500 = 1508, i.e.
                # 28 bytes into the fragment's data, which starts 34 bytes into its frame
                off = np.append(off, np.uint32(off[2] + 34 + 28))
                ln = np.append(ln, np.uint16(len(inner)))
            st = abi.RxStats()
            assert L.udpdk_poll_rx(buf.ctypes.data, len(buf) - 64, off.ctypes.data, ln.ctypes.data,
                                   None, len(off), C.byref(st)) == 0
            for s, want in ((s0, [b"A" * 10, d1[8:]]), (s1, [bytes(range(40, 100))])):
                for w in want:
                    n, data, addr = host_api.recvfrom(s, 8192)
                    assert n == len(w) and data == w, (aliased, s, n)
                    assert addr == ("10.9.8.7", 4000)
    finally:
        L.udpdk_cleanup()


def _poll_and_drain(tmp_path, host_api, frames, extra):
    """udpdk_init (+ the [gpu] lines `extra`), one udpdk_poll_rx over the packed frames (after a
    pre-fill of socket 1's ring), then every socket drained: ([(len, data, addr)] per socket,
    the poll's counters)."""
    ini = tmp_path / "udpdk.ini"
    ini.write_text("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n"
                   "[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n"
                   "[gpu]\ndevice = 0\nmax_frames = 131072\nmax_lanes = 16\n"
                   "frag_buckets = 1024\nfrag_bucket_entries = 16\nfrag_max_dgram = 16384\n" + extra)
    L = abi.lib()
    argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
    assert L.udpdk_init(3, argv) == 0
    try:
        socks = [host_api.socket() for _ in range(4)]
        for k, s in enumerate(socks):
            assert host_api.bind(s, "0.0.0.0", 10000 + k) == 0
        src, dst = raw_ip("10.9.8.7"), raw_ip("172.31.100.1")
        pre = [ip_frame(src, dst, k, 0, udp_datagram(_port(4000), _port(10001), b"P" * 30), False)
               for k in range(900)]
        stats = []
        for fr in (pre, frames):
            buf, off, ln = batch(fr)
            st = abi.RxStats()
            assert L.udpdk_poll_rx(buf.ctypes.data, len(buf) - 64, off.ctypes.data, ln.ctypes.data,
                                   None, len(off), C.byref(st)) == 0
            stats.append((list(st.counters), st.deliveries))
        L.udpdk_interrupt(0)                    # recvfrom on an empty ring: -1 instead of waiting
        got = []
        for s in socks:
            q = []
            while True:
                n, data, addr = host_api.recvfrom(s, 70000)
                if n < 0:
                    break
                q.append((n, data, addr))
            got.append(q)
        return got, stats
    finally:
        L.udpdk_cleanup()


def test_poll_rx_chunked_equals_one_piece(tmp_path, host_api):
    """The pipelined poll ([gpu] poll_chunk_mb: a large batch cut into chunks at burst boundaries,
    chunk k + 1's RX overlapping chunk k - 1's payload copy) gives every ring exactly what the
    one-piece poll gives it: the same datagrams in the same order, reassembled datagrams whose
    fragments straddle chunk cuts included, and the same bursts dropped where a ring fills (every
    socket gets more than its 2047 entries). poll_chunk_mb = 1 (and poll_chunk_min_avg = 0: its
    frames are short) cuts this ~9 MB batch into 9 chunks; the default polls it in one piece."""
    from reasm_util import scenario
    frames = [f for fs, _ in scenario(11, n_batches=10, flows_per_batch=300, normal_per_batch=1800)
              for f in fs]
    one, st_one = _poll_and_drain(tmp_path, host_api, frames, "")
    chk, st_chk = _poll_and_drain(tmp_path, host_api, frames, "poll_chunk_mb = 1\npoll_chunk_min_avg = 0\n")
    assert st_chk == st_one
    assert [len(q) for q in chk] == [len(q) for q in one]
    assert sum(len(q) for q in one) > 4000 and all(len(q) >= 1000 for q in one)
    for k, (a, b) in enumerate(zip(one, chk)):
        assert a == b, k
    # the rings did fill: fewer datagrams than deliveries
    assert sum(len(q) for q in one) < st_one[1][1] + 900
