"""RX parity: the HIP pipeline (through the C ABI) against the oracle, bit for bit — verdict
words, per-lane delivery lists and counters — on seeded inputs; plus full-size property checks.
"""
import errno

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

IP1, IP9 = "172.31.100.1", "172.31.100.9"


def _rx_both(ctx, batch, lists, n_lanes, lane_mask=0xFFFFFFFF, lane_cap=None):
    hs = abi.snapshot_from_lists(lists, n_lanes, lane_mask)
    ctx.upload_snapshot(hs)
    bt = O.bindtable_from_lists(lists)
    want = O.rx(bt, batch.frames, batch.frames_bytes, batch.offset, batch.length, batch.ptype,
                n_lanes, lane_mask)
    db = abi.rx_upload(ctx, batch.frames, batch.offset, batch.length, batch.ptype)
    db.frames_bytes = batch.frames_bytes
    cap = lane_cap if lane_cap is not None else max(1, batch.n * 4)
    out = abi.rx_alloc_out(ctx, batch.n, n_lanes, cap)
    got = abi.rx_run(ctx, db, out)
    for b in (db.frames, db.offset, db.length, db.ptype, out.meta, out.lane_off, out.lane_pkt):
        if b is not None:
            b.free()
    return want, got


def _assert_same(want, got, ctx=""):
    wm, wl, wp, wc = want
    gm, gl, gp, gc, rc = got
    assert rc == 0, ctx
    bad = np.nonzero(wm != gm)[0]
    assert len(bad) == 0, f"{ctx}: {len(bad)} verdict words differ, first {bad[:5]} " \
                          f"want {[hex(x) for x in wm[bad[:5]]]} got {[hex(x) for x in gm[bad[:5]]]}"
    assert np.array_equal(wl, gl), ctx
    assert np.array_equal(wp, gp), ctx
    assert np.array_equal(wc, gc), f"{ctx}: counters {wc} vs {gc}"


MIXED_LISTS = {
    abi.raw_port(10001): [(0, 0, 0)],
    abi.raw_port(10002): [(abi.raw_ip(IP1), 1, 1), (abi.raw_ip(IP1), 2, 1)],    # REUSEPORT fan-out
    abi.raw_port(10003): [(abi.raw_ip(IP9), 3, 0)],                          # specific, no match
    abi.raw_port(10004): [(0, 4, 1), (abi.raw_ip(IP1), 5, 1)],               # ANY + specific clone
    abi.raw_port(10005): [(0, 6, 0), (abi.raw_ip(IP1), 7, 1)],               # ANY swallows (Q3)
}


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("with_ptype", [False, True])
def test_mixed_batches(gpu_ctx, seed, with_ptype):
    b = F.mixed_batch(seed, 3000, [10001, 10002, 10003, 10004, 10005], [9, 20000, 65535],
                      [IP1, IP9], with_ptype=with_ptype)
    want, got = _rx_both(gpu_ctx, b, MIXED_LISTS, 8)
    _assert_same(want, got, f"seed={seed} ptype={with_ptype}")
    # the batch really covers every verdict class
    assert set(np.unique(abi.meta_verdict(want[0]))) >= {0, 1, 2, 3, 4, 5, 6}


def test_fixture_batch(gpu_ctx):
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "rx_mixed.npz"))
    lists = {}
    for p, ip, s, r in z["lists"]:
        lists.setdefault(int(p), []).append((int(ip), int(s), int(r)))
    fr = np.zeros(len(z["frames"]) + 256, np.uint8)
    fr[:len(z["frames"])] = z["frames"]
    b = F.Batch(fr, z["offset"], z["length"], len(z["frames"]), z["ptype"])
    want, got = _rx_both(gpu_ctx, b, lists, 4)
    _assert_same(want, got, "fixture")
    assert np.array_equal(got[0], z["meta"])
    assert np.array_equal(got[2], z["lane_pkt"])


@pytest.mark.parametrize("seed", [31, 32, 33, 34])
def test_fuzzed_headers_and_descriptors(gpu_ctx, seed):
    """The mixed batch with random header bits flipped in 30 % of the frames (ether_type, IHL,
    flags, protocol, lengths, checksums, ports), 5 % of the offsets moved to any byte (frames
    overlapping, starting mid-frame, at odd offsets or past the batch) and 5 % of the lengths
    replaced by edge values (0, 1, 13, 14, 33, 41-43, 63-65, 2047, 65535): the verdict words,
    lanes and counters equal the oracle's on whatever the bytes say."""
    rng = np.random.default_rng(seed)
    base = F.mixed_batch(seed, 4000, [10001, 10002, 10003, 10004, 10005], [9, 20000, 65535],
                         [IP1, IP9], with_ptype=seed % 2 == 0)
    fr = base.frames.copy()
    for i in rng.choice(base.n, base.n * 3 // 10, replace=False):
        o = int(base.offset[i])
        for _ in range(int(rng.integers(1, 4))):
            pos = o + 12 + int(rng.integers(0, 40))
            if pos < base.frames_bytes:
                fr[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    off = base.offset.astype(np.uint64).copy()
    ln = base.length.astype(np.uint32).copy()
    k = rng.choice(base.n, base.n // 20, replace=False)
    off[k] = rng.integers(0, base.frames_bytes + 5000, len(k))
    k = rng.choice(base.n, base.n // 20, replace=False)
    ln[k] = rng.choice([0, 1, 13, 14, 33, 41, 42, 43, 63, 64, 65, 2047, 65535], len(k))
    b = F.Batch(fr, off.astype(np.uint32), ln.astype(np.uint16), base.frames_bytes, base.ptype)
    want, got = _rx_both(gpu_ctx, b, MIXED_LISTS, 8)
    _assert_same(want, got, f"fuzz seed={seed}")
    assert len(set(abi.meta_verdict(want[0]).tolist())) >= 6


def test_compat_uint8_lanes(gpu_ctx):
    """Compat mode: lanes keyed by (uint8_t)sockfd exactly like exch_slots[(uint8_t)fd]."""
    n = 600
    lists = {abi.raw_port(10000 + i): [(0, i, 0)] for i in range(n)}
    rng = np.random.default_rng(5)
    ports = 10000 + rng.integers(0, n, 20000)
    b = F.build_frames(np.full(len(ports), 64, np.uint32), ports, 9)
    want, got = _rx_both(gpu_ctx, b, lists, 256, 0xFF)
    _assert_same(want, got, "compat")
    assert int(np.sum(abi.meta_sockfd(got[0]) >= 256)) > 0


@pytest.mark.parametrize("n_lanes", [2, 3, 7, 8, 9, 16, 33, 100])
def test_lane_counts_no_fanout(gpu_ctx, n_lanes):
    """Small and odd lane counts on the general path without fan-out (rx_scatterw: wave-total
    scratch, 16-byte LDS zeroing only at lanes % 4 == 0, staging only at tiles <= 2 x lanes), one
    binding per port, frames to bound and unbound ports, several tiles."""
    lists = {abi.raw_port(20000 + i): [(0, i, 0)] for i in range(n_lanes)}
    rng = np.random.default_rng(n_lanes)
    ports = 20000 + rng.integers(0, n_lanes + 2, 9000)        # 2 unbound ports among them
    b = F.build_frames(np.full(len(ports), 64, np.uint32), ports, 9)
    want, got = _rx_both(gpu_ctx, b, lists, n_lanes)
    _assert_same(want, got, f"lanes={n_lanes}")


def test_many_tiles_narrow_scan_columns():
    """8 M frames over 64 lanes in a context sized for 64 lanes: 8192 tiles, so rx_scan_cols
    narrows its columns to 2 lanes per workgroup (32 lane blocks, each with a look-back word;
    words for only max_lanes / 8 blocks were allocated before round 5). Exact against the
    oracle."""
    n, n_lanes = 1 << 23, 64
    ctx = abi.GpuContext(0, max_frames=n, max_lanes=n_lanes)
    try:
        assert abi.geometry(n, n_lanes) == (1024, 8192)
        lists = {abi.raw_port(30000 + i): [(0, i, 0)] for i in range(n_lanes)}
        rng = np.random.default_rng(64)
        ports = 30000 + rng.integers(0, n_lanes, n)
        b = F.build_frames(np.full(n, 64, np.uint32), ports, 11)
        want, got = _rx_both(ctx, b, lists, n_lanes, lane_cap=n)
        _assert_same(want, got, "8M x 64 lanes")
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg,n", [(2, 70001), (3, 20000), (4, 50000), (5, 100000), (1, 4096)])
def test_configs_reduced(gpu_ctx, cfg, n):
    w = F.config_batch(cfg, n=n)
    want, got = _rx_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets)
    _assert_same(want, got, w.name)
    assert int(want[3][abi.V_DELIVERED]) == n


@pytest.mark.parametrize("cfg", [2, 3])
def test_configs_full_size(gpu_ctx, cfg):
    """BASELINE.json sizes (1 M frames): exact against the oracle plus properties."""
    w = F.config_batch(cfg)
    want, got = _rx_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets)
    _assert_same(want, got, w.name)
    meta, loff, pkt = got[0], got[1], got[2]
    assert np.all(abi.meta_verdict(meta) == abi.V_DELIVERED)
    assert np.all(abi.meta_udp(meta) == abi.UDP_OK)
    assert np.all((meta >> 4) & 1)
    assert np.array_equal(pkt, np.arange(w.batch.n, dtype=np.uint32))   # one lane, arrival order


def test_zipf_4096_full(gpu_ctx):
    w = F.config_batch(5)
    want, got = _rx_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets)
    _assert_same(want, got, w.name)
    # stability: every lane is strictly increasing
    loff, pkt = got[1], got[2]
    d = np.diff(pkt.astype(np.int64))
    starts = loff[1:-1].astype(np.int64) - 1
    mask = np.ones(len(d), bool)
    mask[starts[(starts >= 0) & (starts < len(d))]] = False
    assert np.all(d[mask] > 0)


@pytest.mark.parametrize("shard", range(1, 8))
def test_zipf_4096_other_shards(gpu_ctx, shard):
    """Config 5's other shards (seeds 1001-1007: the frames each rank of an 8-GPU run gets),
    at a quarter of the full size: exact against the oracle."""
    w = F.config_batch(5, n=1 << 20, shard=shard)
    want, got = _rx_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets)
    _assert_same(want, got, f"{w.name} shard {shard}")


@pytest.mark.parametrize("seed", [21, 22])
def test_tail_checksums_every_alignment(gpu_ctx, seed):
    """rx_classify sums a datagram's tail (frame bytes [64, end)) from the dword-aligned buffer
    offset at or below offset + 64, subtracting the lead bytes and byte-swapping the sum for odd
    offsets: long datagrams at every offset residue, one byte corrupted in a third of them (in
    the lead bytes 64-67, anywhere in the tail, or the last byte). Exact against the oracle,
    and every corrupted datagram is flagged UDP_BAD, every intact one UDP_OK."""
    rng = np.random.default_rng(seed)
    n = 6000
    sizes = rng.integers(65, 1515, n).astype(np.uint32)
    sizes[:8] = [65, 66, 67, 68, 69, 127, 128, 129]
    src = F.build_frames(sizes, np.full(n, 10001, np.uint32), seed)
    gaps = rng.integers(0, 4, n)
    off = np.zeros(n, np.int64)
    pos = 1
    for i in range(n):
        off[i] = pos
        pos += int(sizes[i]) + int(gaps[i])
    fr = np.zeros(pos + 256, np.uint8)
    for i in range(n):
        fr[off[i]:off[i] + sizes[i]] = src.frames[int(src.offset[i]):int(src.offset[i]) + int(sizes[i])]
    bad = rng.random(n) < 1 / 3
    where = rng.integers(0, 3, n)
    for i in np.nonzero(bad)[0]:
        L = int(sizes[i])
        k = {0: 64 + int(rng.integers(0, min(4, L - 64))), 1: int(rng.integers(64, L)), 2: L - 1}[int(where[i])]
        fr[off[i] + k] ^= 0x5A
    b = F.Batch(fr, off.astype(np.uint32), sizes.astype(np.uint16), pos)
    want, got = _rx_both(gpu_ctx, b, {abi.raw_port(10001): [(0, 0, 0)]}, 1)
    _assert_same(want, got, f"seed={seed}")
    assert set(np.unique(off % 4)) == {0, 1, 2, 3}
    udp = abi.meta_udp(got[0])
    assert np.all(udp[bad] == abi.UDP_BAD) and np.all(udp[~bad] == abi.UDP_OK)


def test_edge_sizes(gpu_ctx):
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    for n in [1, 63, 64, 65, 1023, 1024, 1025, 4097]:
        b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), n)
        want, got = _rx_both(gpu_ctx, b, lists, 1)
        _assert_same(want, got, f"n={n}")


@pytest.mark.parametrize("drops", [(), (0,), (5,), (9,), (3, 7), ("all", 3)])
def test_single_lane_speculation(gpu_ctx, drops):
    """Single lane, 1024-frame tiles: rx_classify writes each tile's entries where they belong if
    every earlier tile delivered all its frames, and rx_compact1 keeps them up to the first tile
    that did not (flagged per call) and rewrites the rest. Ten tiles plus a partial one; frames
    dropped (unbound port) in the listed tiles, or a whole tile; each case runs after a call with
    every frame delivered, so a stale flag from an earlier call would show."""
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    n = 10 * 1024 + 300
    for k in range(2):
        b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), 40 + k)
        if k == 1:
            v = b.frames[:n * 64].reshape(n, 64)
            whole = drops[:1] == ("all",)
            for t in (drops[1:] if whole else drops):
                rows = np.arange(t * 1024, min(n, t * 1024 + 1024)) if whole else np.arange(t * 1024 + 17, min(n, t * 1024 + 1024), 101)
                v[rows, 36] = 0x4E                              # dst port 20000: not bound
                v[rows, 37] = 0x20
        want, got = _rx_both(gpu_ctx, b, lists, 1)
        _assert_same(want, got, f"drops={drops} call={k}")


def _drop(b, rows):
    v = b.frames[:b.n * 64].reshape(b.n, 64)
    v[rows, 36] = 0x4E                                          # dst port 20000: not bound
    v[rows, 37] = 0x20


@pytest.mark.parametrize("case", ["first", "middle", "last_but_one", "whole_tile", "many", "every_other",
                                  "cap_4096_tiles"])
def test_fused_repair(gpu_ctx, case):
    """A single-lane call whose tiles are not all full is repaired inside the same launch: the
    last arrival opens the repair and the shards' last arrivals that saw the call's short-tile flag
    join it (full tiles written as frame-index runs, short ones from their verdict words). Exact
    against the oracle for short tiles at the start, middle and end, a whole dropped tile, many
    short tiles, every other tile short, and the 4096-tile cap of the fused form; each case runs
    between clean calls on the same context, so a stale flag, work or done word would show."""
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    n = (4096 if case == "cap_4096_tiles" else 1024) * 1024 - 77
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    for k in range(3):
        b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), 60 + k)
        if k == 1:
            nt = -(-n // 1024)
            if case == "first":
                rows = [5]
            elif case == "middle":
                rows = [500 * 1024 + 3]
            elif case == "last_but_one":
                rows = [(nt - 2) * 1024 + 1023]
            elif case == "whole_tile":
                rows = np.arange(300 * 1024, 301 * 1024)
            elif case == "many":
                rows = rng.choice(n, 3000, replace=False)
            elif case == "every_other":
                rows = np.arange(0, n, 2048)
            else:
                rows = rng.choice(n, 50, replace=False)
            _drop(b, rows)
        want, got = _rx_both(gpu_ctx, b, lists, 1)
        _assert_same(want, got, f"{case} call={k}")


def test_fused_repair_lane_overflow(gpu_ctx):
    """The repair of a call whose lane overflows its capacity: entries past the capacity are not
    written, the ones below it are exact, and the call reports ENOSPC with the true total."""
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    n = 64 * 1024
    b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), 9)
    _drop(b, [100, 20000, 20001])
    hs = abi.snapshot_from_lists(lists, 1)
    gpu_ctx.upload_snapshot(hs)
    bt = O.bindtable_from_lists(lists)
    wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, 1)
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    cap = 40000
    out = abi.rx_alloc_out(gpu_ctx, n, 1, cap)
    meta, loff, pkt, cnt, rc = abi.rx_run(gpu_ctx, db, out)
    assert rc == -errno.ENOSPC
    assert loff[1] == n - 3 and np.array_equal(meta, wm)
    assert np.array_equal(pkt, wp[:cap])


def test_empty_batch(gpu_ctx):
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    hs = abi.snapshot_from_lists(lists, 3)
    gpu_ctx.upload_snapshot(hs)
    b = abi.RxDeviceBatch(gpu_ctx.alloc(256), 0, gpu_ctx.alloc(4), gpu_ctx.alloc(4), None, 0)
    out = abi.rx_alloc_out(gpu_ctx, 0, 3, 4)
    meta, loff, pkt, cnt, rc = abi.rx_run(gpu_ctx, b, out)
    assert rc == 0 and np.all(loff == 0) and len(pkt) == 0 and np.all(cnt == 0)


def test_bad_descriptors(gpu_ctx):
    """offset + length beyond frames_bytes: verdict BAD_DESC, nothing read."""
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    b = F.build_frames(np.full(100, 64, np.uint32), np.full(100, 10001, np.uint32), 3)
    b.offset[7] = b.frames_bytes - 10
    b.offset[50] = 0xFFFFFF00
    b.length[60] = 65535
    want, got = _rx_both(gpu_ctx, b, lists, 1)
    _assert_same(want, got, "bad desc")
    assert abi.meta_verdict(got[0])[[7, 50, 60]].tolist() == [abi.V_BAD_DESC] * 3


def test_lane_overflow(gpu_ctx):
    lists = {abi.raw_port(10001): [(0, 0, 0)]}
    b = F.build_frames(np.full(1000, 64, np.uint32), np.full(1000, 10001, np.uint32), 3)
    hs = abi.snapshot_from_lists(lists, 1)
    gpu_ctx.upload_snapshot(hs)
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, 1000, 1, 100)
    meta, loff, pkt, cnt, rc = abi.rx_run(gpu_ctx, db, out)
    assert rc == -errno.ENOSPC
    assert loff[1] == 1000 and np.array_equal(pkt, np.arange(100))


def test_rx_host_end_to_end(gpu_ctx):
    """udpdk_gpu_rx_host: host batch in, host results out (pinned staging + H2D + D2H)."""
    import ctypes as C
    b = F.mixed_batch(11, 2000, [10001, 10002, 10003, 10004, 10005], [9, 20000], [IP1, IP9])
    hs = abi.snapshot_from_lists(MIXED_LISTS, 8)
    gpu_ctx.upload_snapshot(hs)
    bt = O.bindtable_from_lists(MIXED_LISTS)
    wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, 8)
    meta = np.zeros(b.n, np.uint32)
    loff = np.zeros(9, np.uint32)
    pkt = np.zeros(b.n * 4, np.uint32)
    st = abi.RxStats()
    rc = abi.lib().udpdk_gpu_rx_host(gpu_ctx.handle, b.frames.ctypes.data, b.frames_bytes,
                                     b.offset.ctypes.data, b.length.ctypes.data, None, b.n,
                                     meta.ctypes.data, loff.ctypes.data, pkt.ctypes.data,
                                     len(pkt), C.byref(st))
    assert rc == 0
    assert np.array_equal(meta, wm) and np.array_equal(loff, wl)
    assert np.array_equal(pkt[:st.deliveries], wp)
    assert np.array_equal(np.array(st.counters[:], np.uint64), wc)


@pytest.mark.parametrize("cfg,depth", [(4, 2), (4, 3), (4, 4), (2, 3)])
def test_pipeline_depth(gpu_ctx, cfg, depth):
    """Several pipes: consecutive calls on independent batches overlap; every call's outputs and
    the last call's counters still equal the oracle's (config 4: scan + scatter path, config 2:
    single-lane compaction)."""
    ws = [F.config_batch(cfg, n=30000 + 1000 * i) for i in range(depth + 2)]   # same lists
    lists = ws[0].port_lists()
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists(lists, ws[0].n_sockets))
    bt = O.bindtable_from_lists(lists)
    runs = []
    for w in ws:
        db = abi.rx_upload(gpu_ctx, w.batch.frames, w.batch.offset, w.batch.length)
        db.frames_bytes = w.batch.frames_bytes
        runs.append((w, db, abi.rx_alloc_out(gpu_ctx, w.batch.n, w.n_sockets, w.batch.n)))
    gpu_ctx.pipeline(depth)
    try:
        for w, db, out in runs:
            assert abi.rx_enqueue(gpu_ctx, db, out) == 0
        rc, st = abi.rx_stats(gpu_ctx)
        assert rc == 0
        gpu_ctx.sync()
        for w, db, out in runs:
            b = w.batch
            wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, w.n_sockets)
            assert np.array_equal(gpu_ctx.download(out.meta, np.uint32, b.n), wm)
            assert np.array_equal(gpu_ctx.download(out.lane_off, np.uint32, w.n_sockets + 1), wl)
            assert np.array_equal(gpu_ctx.download(out.lane_pkt, np.uint32, len(wp)), wp)
        assert np.array_equal(np.array(st.counters[:], np.uint64), wc)   # the last call's
    finally:
        gpu_ctx.pipeline(1)


def test_rx_host_sync_and_async(gpu_ctx):
    """Host-resident batches (udpdk_gpu_rx_host and the two-pipe udpdk_gpu_rx_host_async) give
    the device path's results; the frames buffer is staged at exactly its size + tailroom."""
    import ctypes as C
    b = F.mixed_batch(21, 5000, [10001, 10002, 10004], [9, 20000], [IP1, IP9])
    lists = {k: v for k, v in MIXED_LISTS.items()}
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists(lists, 8))
    bt = O.bindtable_from_lists(lists)
    want = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, 8)
    L = abi.lib()
    fr = np.ascontiguousarray(b.frames[:b.frames_bytes])

    def call(fn, depth):
        gpu_ctx.pipeline(depth)
        res = []
        for k in range(3):
            meta = np.zeros(b.n, np.uint32)
            loff = np.zeros(9, np.uint32)
            pkt = np.zeros(4 * b.n, np.uint32)
            st = abi.RxStats()
            rc = fn(gpu_ctx.handle, fr.ctypes.data, b.frames_bytes, b.offset.ctypes.data,
                    b.length.ctypes.data, None, b.n, meta.ctypes.data, loff.ctypes.data,
                    pkt.ctypes.data, 4 * b.n, C.byref(st))
            assert rc == 0
            res.append((meta, loff, pkt, st))
        if fn is L.udpdk_gpu_rx_host_async:
            assert L.udpdk_gpu_rx_host_wait(gpu_ctx.handle) == 0
        gpu_ctx.pipeline(1)
        return res

    for fn, depth in ((L.udpdk_gpu_rx_host, 1), (L.udpdk_gpu_rx_host_async, 2),
                      (L.udpdk_gpu_rx_host_async, 3)):
        for meta, loff, pkt, st in call(fn, depth):
            assert np.array_equal(meta, want[0])
            assert np.array_equal(loff, want[1])
            d = int(st.deliveries)
            assert d == int(want[1][-1])
            assert np.array_equal(pkt[:d], want[2])
            assert np.array_equal(np.array(st.counters[:], np.uint64), want[3])


def test_single_lane_many_tiles():
    """5 M frames in one batch (5120 tiles: past COMPACT1_DIRECT_TILES the compaction takes its
    tile bases from rx_tile_base): every frame delivered except every 997th, whose destination
    port is unbound; the lane lists the others in order."""
    w = F.config_batch(2, n=5 * (1 << 20))
    b = w.batch
    n = b.n
    drop = np.arange(0, n, 997)
    v = b.frames[:n * 64].reshape(n, 64)
    v[drop, 36] = 0x4E                                  # dst port 20000: not bound
    v[drop, 37] = 0x20
    ctx = abi.GpuContext(0, max_frames=6 << 20, max_lanes=16)
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), 1))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, n, 1, n)
    meta, loff, pkt, cnt, rc = abi.rx_run(ctx, db, out)
    keep = np.ones(n, bool)
    keep[drop] = False
    assert rc == 0 and int(loff[1]) == int(keep.sum())
    assert np.array_equal(pkt, np.nonzero(keep)[0].astype(np.uint32))
    assert np.all(abi.meta_verdict(meta[drop]) == abi.V_NO_BIND)
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
        x.free()
    ctx.close()


@pytest.mark.parametrize("tail", [1, 2, 3])
def test_tailroom_exact_allocation(gpu_ctx, tail):
    """The tailroom contract at its edge: frames_bytes % 4 == tail, the device allocation is
    exactly frames_bytes + UDPDK_GPU_FRAMES_TAILROOM, and the batch's last frame ends exactly at
    frames_bytes (its UDP checksum covers the last byte). Round 1 faulted on a buffer loaded 16 B
    past an exactly-sized allocation; this pins the fixed range."""
    import ctypes as C
    lists = {abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}
    sizes = np.array([64, 1500, 97, 333, 60 + tail + 4 * 7], np.uint32)
    sizes[-1] += (tail - int(sizes.sum()) % 4) % 4          # frames_bytes % 4 == tail
    b = F.build_frames(sizes, np.full(len(sizes), F.PORT_RECV, np.uint32), 77 + tail)
    fb = int(b.length.astype(np.int64).sum())
    assert fb % 4 == tail and int(b.offset[-1]) + int(b.length[-1]) == fb
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists(lists, 1))
    exact = gpu_ctx.alloc(fb + abi.FRAMES_TAILROOM)           # exactly the contract, no slack
    abi._check(abi.lib().udpdk_gpu_h2d(gpu_ctx.handle, C.c_void_p(exact.ptr),
                                       b.frames.ctypes.data_as(C.c_void_p), fb), "h2d")
    gpu_ctx.sync()
    db = abi.RxDeviceBatch(exact, fb, gpu_ctx.upload(b.offset.astype(np.uint32)),
                           gpu_ctx.upload(b.length.astype(np.uint16)), None, b.n)
    out = abi.rx_alloc_out(gpu_ctx, b.n, 1, b.n)
    got = abi.rx_run(gpu_ctx, db, out)
    want = O.rx(O.bindtable_from_lists(lists), b.frames, fb, b.offset, b.length, None, 1)
    _assert_same(want, got, f"tail={tail}")
    assert np.all(abi.meta_udp(got[0]) == abi.UDP_OK)
    for x in (exact, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
        x.free()


def test_config4_full_size(gpu_ctx):
    """BASELINE.json configs[3] at its full size: 1 M IMIX frames over 1024 ports, exact against
    the oracle (verdict words, lanes, counters), plus lane stability."""
    w = F.config_batch(4)
    want, got = _rx_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets)
    _assert_same(want, got, w.name)
    loff, pkt = got[1].astype(np.int64), got[2].astype(np.int64)
    assert int(loff[-1]) == w.batch.n
    d = np.diff(pkt)
    inner = np.ones(len(d), bool)
    inner[loff[1:-1][loff[1:-1] > 0] - 1] = False            # lane boundaries may step down
    assert np.all(d[inner] > 0)


@pytest.mark.parametrize("shards", [2, 4])
def test_sharded_hip_merge(gpu_ctx, shards):
    """SURVEY.md §8(e) through the HIP path: config 5's Zipf-0.99 batch over 4096 ports cut into
    contiguous shards, each shard a separate udpdk_gpu_rx call (on device 0, as one rank per GPU
    would run it), merged with shard.merge_lanes; equal to the single-batch HIP result and to the
    oracle."""
    from udpdk_amd import shard as S
    w = F.config_batch(5, n=1 << 20)
    b = w.batch
    want, got = _rx_both(gpu_ctx, b, w.port_lists(), w.n_sockets)
    _assert_same(want, got, "single batch")
    parts, metas = [], []
    for r in range(shards):
        a, e = S.shard_range(b.n, shards, r)
        sb = F.Batch(b.frames, b.offset[a:e].copy(), b.length[a:e].copy(), b.frames_bytes, None)
        _, sg = _rx_both(gpu_ctx, sb, w.port_lists(), w.n_sockets)
        assert sg[4] == 0
        parts.append((sg[1], sg[2], a))
        metas.append(sg[0])
    goff, gpkt = S.merge_lanes(parts, w.n_sockets)
    assert np.array_equal(np.concatenate(metas), got[0])
    assert np.array_equal(goff, got[1]) and np.array_equal(gpkt, got[2])
    assert np.array_equal(goff, want[1]) and np.array_equal(gpkt, want[2])
