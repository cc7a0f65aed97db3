"""The udpdk_api.h socket layer (host C) against the reference semantics: errno values, option
bits, bind admission and list order (cross-checked with the oracle's restated bind table),
auto-bind, close, sendto/tx_drain. CPU only."""
import errno
import socket

import numpy as np

import oracle as O
from udpdk_amd import abi


def test_socket_arguments(host_api):
    assert host_api.socket(socket.AF_INET6) == -1 and host_api.errno() == errno.EAFNOSUPPORT
    assert host_api.socket(typ=socket.SOCK_STREAM) == -1 and host_api.errno() == errno.EPROTONOSUPPORT
    assert host_api.socket(proto=6) == -1 and host_api.errno() == errno.EINVAL
    assert host_api.socket(proto=socket.IPPROTO_UDP) == 0
    assert host_api.socket() == 1
    assert host_api.close(0) == 0
    assert host_api.socket() == 0                     # lowest free slot is reused
    assert host_api.close(7) == -1 and host_api.errno() == errno.EBADF


def test_sockopt_errors(host_api):
    s = host_api.socket()
    assert host_api.setsockopt(s, 6, abi.SO_REUSEADDR, 1) == -1 and host_api.errno() == errno.EINVAL
    assert host_api.setsockopt(s, abi.SOL_SOCKET, 7, 1) == -1 and host_api.errno() == errno.ENOPROTOOPT
    assert host_api.setsockopt(99, abi.SOL_SOCKET, abi.SO_REUSEADDR, 1) == -1
    assert host_api.errno() == errno.EBADF
    assert host_api.getsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT) == (0, 0)
    assert host_api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEADDR, 1) == 0
    assert host_api.getsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEADDR) == (0, 1)
    assert host_api.getsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT) == (0, 1)   # 15 & 2 (Q4)
    assert host_api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEADDR, 0) == 0
    assert host_api.getsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT) == (0, 0)


def test_bind_errors(host_api):
    s = host_api.socket()
    assert host_api.bind(s, "0.0.0.0", 10001, addrlen=8) == -1 and host_api.errno() == errno.EINVAL
    assert host_api.bind(s, "0.0.0.0", 10001) == 0
    assert host_api.bind(s, "0.0.0.0", 10002) == -1 and host_api.errno() == errno.EINVAL
    t = host_api.socket()
    assert host_api.bind(t, "0.0.0.0", 10001) == -1 and host_api.errno() == errno.EADDRINUSE
    assert host_api.close(s) == 0
    assert host_api.bind(t, "0.0.0.0", 10001) == 0    # freed by close


def _replay(host_api, ops, bt):
    """Apply the same bind/close sequence to the product and to the oracle bind table."""
    socks = {}
    for op in ops:
        if op[0] == "bind":
            _, s, ip, port, opts = op
            if s not in socks:
                assert host_api.socket() == s
                socks[s] = None
                if opts:
                    host_api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT if opts == 15 else abi.SO_REUSEADDR, 1)
            rc_p = host_api.bind(s, ip, port)
            rc_o = bt.add(s, abi.raw_ip(ip), abi.raw_port(port), opts)
            assert (rc_p == 0) == (rc_o == 0), op
            socks[s] = port if rc_p == 0 else None


def test_bind_rules_and_order_match_oracle(host_api):
    rng = np.random.default_rng(0)
    ips = ["0.0.0.0", "10.0.0.1", "10.0.0.2"]
    for trial in range(30):
        host_api.reset()
        bt = O.BindTable()
        ops = []
        for s in range(24):
            ops.append(("bind", s, str(rng.choice(ips)), int(rng.integers(5000, 5004)),
                        int(rng.choice([0, 0, 2, 15]))))
        _replay(host_api, ops, bt)
        lists = host_api.port_lists()
        for p in range(65536):
            want = bt.port_list(p)
            got = lists.get(p, [])
            assert [(ip, s, r) for ip, s, r in got] == want, (trial, p)


def test_close_removes_binding_and_version(host_api):
    s = host_api.socket()
    t = host_api.socket()
    host_api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT, 1)
    host_api.setsockopt(t, abi.SOL_SOCKET, abi.SO_REUSEPORT, 1)
    assert host_api.bind(s, "10.0.0.5", 7000) == 0
    assert host_api.bind(t, "10.0.0.5", 7000) == 0
    v0 = host_api.snapshot().version
    assert host_api.port_lists()[abi.raw_port(7000)] == [(abi.raw_ip("10.0.0.5"), 0, 1),
                                                           (abi.raw_ip("10.0.0.5"), 1, 1)]
    assert host_api.close(s) == 0
    assert host_api.port_lists()[abi.raw_port(7000)] == [(abi.raw_ip("10.0.0.5"), 1, 1)]
    assert host_api.snapshot().version > v0


def test_autobind_lowest_raw_port(host_api):
    """Q9: btable_get_free_port walks raw indices, so sendto auto-binds to raw ports 0, 1, ..."""
    a, b = host_api.socket(), host_api.socket()
    assert host_api.sendto(a, b"hi", "9.9.9.9", 53) == 2
    assert host_api.sendto(b, b"hi", "9.9.9.9", 53) == 2
    slots = host_api.slots(2)
    assert slots[0] == (0, 0, 1) and slots[1] == (0, 1, 1)     # ANY, raw port 0 / 1, bound
    snap = host_api.snapshot()
    assert snap.port_count[0] == 1 and snap.port_count[1] == 1
    assert host_api.tx_pending() == 2


def test_sendto_validation_and_queue(host_api):
    """sendto's checks (udpdk_syscall.c:247-276) and its TX ring (EXCH_RING_SIZE, ENOBUFS when
    full, :356-365); the frames are built on the GPU by udpdk_tx_drain (test_gpu_sock_path)."""
    s = host_api.socket()
    assert host_api.bind(s, "0.0.0.0", 10000) == 0
    assert host_api.sendto(s, b"a" * 64, "172.31.100.1", 10001) == 64
    assert host_api.sendto(s, b"b" * 10, "172.31.100.1", 10001, flags=1) == -1
    assert host_api.errno() == errno.EINVAL
    # the poller fragments what exceeds the MTU, so sendto takes any UDP-sized payload
    assert host_api.sendto(s, b"c" * 2000, "172.31.100.1", 10001) == 2000
    assert host_api.sendto(s, b"c" * 65507, "172.31.100.1", 10001) == 65507
    assert host_api.sendto(s, b"c" * 65508, "172.31.100.1", 10001) == -1
    assert host_api.errno() == errno.EMSGSIZE
    assert host_api.sendto(5000, b"x", "1.1.1.1", 1) == -1 and host_api.errno() == errno.ENOTSOCK
    assert host_api.sendto(7, b"x", "1.1.1.1", 1) == -1 and host_api.errno() == errno.EBADF
    assert host_api.tx_pending() == 3
    for i in range(2047 - 3):
        assert host_api.sendto(s, b"q", "172.31.100.1", 10001) == 1
    assert host_api.sendto(s, b"q", "172.31.100.1", 10001) == -1 and host_api.errno() == errno.ENOBUFS
    assert host_api.close(s) == 0
    assert host_api.tx_pending() == 0                 # queued sends die with the socket


def test_tx_drain_needs_gpu_context(host_api):
    if abi.device_count() > 0:
        return
    s = host_api.socket()
    assert host_api.sendto(s, b"x", "1.1.1.1", 1) == 1
    import pytest
    with pytest.raises(abi.UdpdkError):
        host_api.tx_drain()


def test_snapshot_compat_mode(host_api):
    for i in range(300):
        assert host_api.socket() == i
        assert host_api.bind(i, "0.0.0.0", 20000 + i) == 0
    s = host_api.snapshot(compat=True)
    assert s.n_lanes == 256 and s.lane_mask == 0xFF and s.n_binds == 300
    s = host_api.snapshot(compat=False)
    assert s.n_lanes == 300 and s.lane_mask == 0xFFFFFFFF


def test_init_requires_config():
    import ctypes as C
    L = abi.lib()
    argv = (C.c_char_p * 2)(b"prog", None)
    assert L.udpdk_init(1, argv) == -1


def test_close_unblocks_a_blocked_recvfrom(host_api):
    """A recvfrom blocked on an empty ring in another thread (the reference busy-waits,
    udpdk_syscall.c:424-426) returns -1/EBADF when the socket is closed under it, instead of
    reading ring entries close has freed; the slot is reusable afterwards."""
    import threading
    s = host_api.socket()
    assert host_api.bind(s, "0.0.0.0", 10001) == 0
    out = {}

    def reader():
        n, _, _ = host_api.recvfrom(s, 64)
        out["rc"], out["errno"] = n, host_api.errno()    # errno is per thread
    for _ in range(20):
        t = threading.Thread(target=reader)
        t.start()
        t.join(0.02)
        assert t.is_alive()                              # blocked: nothing was queued
        assert host_api.close(s) == 0
        t.join(10)
        assert not t.is_alive() and out == {"rc": -1, "errno": errno.EBADF}
        assert host_api.socket() == s and host_api.bind(s, "0.0.0.0", 10001) == 0
        out.clear()
    # a recvfrom on a closed socket fails at once
    assert host_api.close(s) == 0
    assert host_api.recvfrom(s, 64)[0] == -1 and host_api.errno() == errno.EBADF
