"""Multi-device RX in the library (f4's "RX queues to GPUs"): with
"[gpu] devices = ..." udpdk_init creates one RX shard context per entry, and udpdk_poll_rx splits
each batch into contiguous shards (or, with "dispatch = rss", by each frame's RSS queue, one queue
per device), classifies / demultiplexes / gathers each on its own context from its own pool
thread, and merges the shards' lanes in arrival order before ring admission.
The rings must then equal a single-context session's on the same traffic, fragments included
(their flows straddle shard boundaries and go through the main context's reassembly table).
The box has one GPU, so the shard contexts all sit on device 0; the code path is the same as on
eight devices (each context does hipSetDevice on its own device id)."""
import ctypes as C

import numpy as np
import pytest

from reasm_util import batch, ip_frame, raw_ip, split, udp_datagram
from udpdk_amd import abi

pytestmark = pytest.mark.gpu

SOCK_PORTS = [10001, 10002, 10003, 10004, 10005]


def _port(p):
    return int.from_bytes(p.to_bytes(2, "big"), "little")


def _traffic(seed):
    """Two polls of mixed frames: plain datagrams to five sockets (Zipf-skewed, enough for one
    socket to overflow its ring so whole bursts are dropped), some to unbound ports, and
    fragmented datagrams whose fragments are spread over the batch and over the two polls."""
    rng = np.random.default_rng(seed)
    src, dst = raw_ip("10.9.8.7"), raw_ip("172.31.100.1")
    polls = [[], []]
    pid = 100
    for k in range(2):
        n = 5000
        for i in range(n):
            r = int(min(rng.zipf(1.4), 7)) - 1
            port = SOCK_PORTS[r] if r < 5 else 20000 + r
            pl = rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
            polls[k].append(ip_frame(src, dst, pid & 0xFFFF, 0,
                                     udp_datagram(_port(40000 + (i & 7)), _port(port), pl), False))
            pid += 1
    # 60 fragmented datagrams: fragments at random positions, some completing in the second poll
    for j in range(60):
        port = SOCK_PORTS[j % 5]
        pl = rng.integers(0, 256, int(rng.integers(1500, 4000)), dtype=np.uint8).tobytes()
        d = udp_datagram(_port(4000 + j), _port(port), pl)
        sizes, left = [], len(d)
        while left > 1480:
            sizes.append(1480)
            left -= 1480
        sizes.append(left)
        frs = split(src, dst, 5000 + j, d, sizes)
        rng.shuffle(frs)
        for f in frs:
            k = 1 if (j % 4 == 0 and f is frs[-1]) else 0
            polls[k].insert(int(rng.integers(0, len(polls[k]) + 1)), f)
    return polls


def _session(tmp_path, host_api, gpu_lines, polls):
    ini = tmp_path / "udpdk.ini"
    ini.write_text("[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n"
                   "[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n"
                   "[gpu]\nmax_frames = 65536\nmax_lanes = 64\n"
                   "frag_buckets = 64\nfrag_bucket_entries = 16\nfrag_max_dgram = 16384\n" + gpu_lines)
    L = abi.lib()
    argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
    assert L.udpdk_init(3, argv) == 0
    try:
        devs = (C.c_int * 16)()
        nd = L.udpdk_shard_devices(devs, 16)
        socks = [host_api.socket() for _ in SOCK_PORTS]
        for s, p in zip(socks, SOCK_PORTS):
            assert host_api.bind(s, "0.0.0.0", p) == 0
        stats = []
        for frames in polls:
            buf, off, ln = batch(frames)
            st = abi.RxStats()
            assert L.udpdk_poll_rx(buf.ctypes.data, len(buf) - 64, off.ctypes.data, ln.ctypes.data,
                                   None, len(off), C.byref(st)) == 0
            stats.append((list(st.counters), st.deliveries))
        fr = (C.c_uint32 * 16)()
        L.udpdk_shard_frames.argtypes = [C.c_void_p, C.c_int]
        ns = L.udpdk_shard_frames(fr, 16)
        shard_frames = [fr[i] for i in range(ns)]
        L.udpdk_interrupt(0)
        rings = []
        for s in socks:
            got = []
            while True:
                n, data, addr = host_api.recvfrom(s, 16384)
                if n < 0:
                    break
                got.append((data, addr))
            rings.append(got)
        return nd, [devs[i] for i in range(nd)], stats, rings, shard_frames
    finally:
        L.udpdk_cleanup()


@pytest.mark.parametrize("devices,n_shards,threads", [("0,0", 2, None), ("0,0,0", 3, 2), ("0-0,0,0,0", 4, 1)])
def test_shard_contexts_give_the_single_context_rings(tmp_path, host_api, devices, n_shards, threads):
    polls = _traffic(7)
    extra = f"poll_threads = {threads}\n" if threads else ""
    n1, d1, st1, r1, _ = _session(tmp_path, host_api, "device = 0\n" + extra, polls)
    host_api.reset()
    nk, dk, stk, rk, _ = _session(tmp_path, host_api, f"devices = {devices}\n" + extra, polls)
    assert n1 == 1 and d1 == [0]
    assert nk == n_shards and dk == [0] * n_shards
    assert stk == st1                                  # counters and deliveries, summed over shards
    assert [len(r) for r in rk] == [len(r) for r in r1]
    for a, b in zip(rk, r1):
        assert a == b
    # the traffic exercised what it should: whole bursts dropped on the hottest socket,
    # reassembled datagrams delivered (payloads > 1480 B)
    assert len(r1[0]) < sum(1 for p in polls for f in p if len(f) >= 38 and f[36:38] == _port(10001).to_bytes(2, "little"))
    assert any(len(d) > 1480 for r in r1 for d, _ in r)


@pytest.mark.parametrize("devices,n_shards", [("0,0", 2), ("0,0,0,0", 4)])
def test_rss_dispatch_gives_the_single_context_rings(tmp_path, host_api, gpu_ctx, devices, n_shards):
    """[gpu] dispatch = rss (f4: one RX queue per device, the frame's queue from its Toeplitz
    hash): the rings still equal a single-context session's (lanes merged back in arrival order),
    and each shard took exactly the frames udpdk_gpu_rss puts in its queue (the same hash, key and
    redirection table on the GPU, n_queues = the shard count)."""
    polls = _traffic(11)
    n1, _, st1, r1, _ = _session(tmp_path, host_api, "device = 0\n", polls)
    host_api.reset()
    nk, _, stk, rk, sfr = _session(tmp_path, host_api, f"devices = {devices}\ndispatch = rss\n", polls)
    assert nk == n_shards
    assert stk == st1
    assert [len(r) for r in rk] == [len(r) for r in r1]
    for a, b in zip(rk, r1):
        assert a == b
    # the last poll's split against the GPU RSS kernel's queues for the same frames
    buf, off, ln = batch(polls[-1])
    db = abi.rx_upload(gpu_ctx, buf, off, ln)
    db.frames_bytes = len(buf) - 64
    qoff = abi.rss_run(gpu_ctx, db, abi.rss_conf(n_shards))[1]
    for x in (db.frames, db.offset, db.length):
        x.free()
    want = [int(qoff[q + 1] - qoff[q]) for q in range(n_shards)]
    assert sfr == want and min(want) > 0


def test_devices_key_errors(tmp_path):
    """A malformed devices list fails udpdk_init with EINVAL, a device id the box does not have
    with ENODEV (the main context is created first, on the list's first device)."""
    L = abi.lib()
    for bad, want in (("devices = 1-0\n", 22), ("devices = x\n", 22), ("devices = 0,63\n", 19)):
        ini = tmp_path / "bad.ini"
        ini.write_text("[port0]\nip_addr = 172.31.100.1\n[gpu]\nmax_frames = 4096\nmax_lanes = 8\n" + bad)
        argv = (C.c_char_p * 4)(b"prog", b"-c", str(ini).encode(), None)
        assert L.udpdk_init(3, argv) == -1
        assert abi.HostApi().errno() == want, bad
