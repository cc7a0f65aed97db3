"""The single-lane RX path's kernel forms, each forced (UDPDK_RX_FUSE / UDPDK_RX_TAILG, read at
context creation) and compared with the oracle bit for bit: the fused completion (the last
workgroup writes lane_off and the total; with a tile before the last not full it rewrites the
later tiles' entries from the verdict words) against rx_classify + rx_compact1, and
rx_classify<1> (one tail chunk group in flight) against <2> (with and without the span sweep of
steps of long back-to-back frames), and a bind table of at most 8 ports
passed in the kernel arguments against the port-table loads. The automatic choice between them
(kernel hints, udpdk_gpu.hip) only picks the faster of two exact forms."""
import os

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

# (fused completion, tail chunk groups, bind table of <= 8 ports in the kernel arguments, span
# sweep of long-frame steps allowed)
FORMS = [(1, 1, 1, 1), (1, 2, 1, 1), (1, 2, 1, 0), (0, 1, 1, 1), (0, 2, 1, 1), (1, 1, 0, 1), (0, 2, 0, 1),
         (0, 2, 0, 0)]
ENV = ("UDPDK_RX_FUSE", "UDPDK_RX_TAILG", "UDPDK_RX_NO_INLINE", "UDPDK_RX_SPAN")


@pytest.fixture(scope="module", params=FORMS, ids=lambda f: f"fuse{f[0]}-g{f[1]}-inl{f[2]}-span{f[3]}")
def form_ctx(request):
    fuse, g, inl, span = request.param
    old = {k: os.environ.get(k) for k in ENV}
    os.environ["UDPDK_RX_FUSE"] = str(fuse)
    os.environ["UDPDK_RX_TAILG"] = str(g)
    os.environ["UDPDK_RX_SPAN"] = str(span)
    if not inl:
        os.environ["UDPDK_RX_NO_INLINE"] = "1"
    else:
        os.environ.pop("UDPDK_RX_NO_INLINE", None)
    try:
        ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=64)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield ctx
    ctx.close()


LISTS1 = {abi.raw_port(10001): [(0, 0, 0)]}


def _run(ctx, b, lists=LISTS1, n_lanes=1, cap=None):
    ctx.upload_snapshot(abi.snapshot_from_lists(lists, n_lanes))
    want = O.rx(O.bindtable_from_lists(lists), b.frames, b.frames_bytes, b.offset, b.length, b.ptype,
                n_lanes, 0xFFFFFFFF)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length, b.ptype)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, n_lanes, max(1, b.n if cap is None else cap))
    got = abi.rx_run(ctx, db, out)
    for x in (db.frames, db.offset, db.length, db.ptype, out.meta, out.lane_off, out.lane_pkt):
        if x is not None:
            x.free()
    return want, got


def _same(want, got, what):
    wm, wl, wp, wc = want
    gm, gl, gp, gc, rc = got
    assert np.array_equal(wm, gm), f"{what}: verdict words"
    assert np.array_equal(wl, gl), f"{what}: lane_off {wl} vs {gl}"
    assert np.array_equal(wp[:len(gp)], gp), f"{what}: lane entries"
    assert np.array_equal(wc, gc), f"{what}: counters"


def _drop(b, rows):
    v = b.frames[:b.n * 64].reshape(b.n, 64)
    v[rows, 36] = 0x4E                                      # dst port 20000: not bound
    v[rows, 37] = 0x20


@pytest.mark.parametrize("n", [1, 1000, 1024, 1025, 10 * 1024 + 300, 70001])
@pytest.mark.parametrize("drops", ["none", "first", "middle", "last_full", "last_tile", "tiles", "all", "sparse"])
def test_single_lane_forms(form_ctx, n, drops):
    """Every frame delivered, or frames dropped in the first tile, a middle one, the last full
    tile, the last (partial) tile, two whole tiles, every frame, or every 97th frame. Each case
    runs right after an all-delivered call on the same context (no stale state may show)."""
    tiles = (n + 1023) // 1024
    for k in range(2):
        b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), 70 + k + n % 7)
        if k == 1 and drops != "none":
            t = {"first": 0, "middle": tiles // 2, "last_full": max(0, tiles - 2),
                 "last_tile": tiles - 1}.get(drops)
            if t is not None:
                _drop(b, np.arange(t * 1024 + 3, min(n, t * 1024 + 1024), 113))
            elif drops == "tiles":
                for t in (tiles // 3, tiles - 1):
                    _drop(b, np.arange(t * 1024, min(n, t * 1024 + 1024)))
            elif drops == "all":
                _drop(b, np.arange(n))
            else:
                _drop(b, np.arange(5, n, 97))
        want, got = _run(form_ctx, b)
        _same(want, got, f"n={n} drops={drops} call={k}")


def test_lane_overflow_forms(form_ctx):
    """lane_cap below the deliveries, with and without a tile that was not full: the entries
    that fit, lane_off[1] = all deliveries, ENOSPC."""
    import errno
    for dropped in (False, True):
        b = F.build_frames(np.full(5000, 64, np.uint32), np.full(5000, 10001, np.uint32), 3)
        if dropped:
            _drop(b, np.arange(10, 5000, 50))
        want, got = _run(form_ctx, b, cap=1500)
        assert got[4] == -errno.ENOSPC
        assert int(got[1][1]) == int(want[1][1])
        assert np.array_equal(want[2][:1500], got[2])


@pytest.mark.parametrize("seed", [41, 42])
def test_tail_forms(form_ctx, seed):
    """Long datagrams at every offset residue with a third corrupted (the tail pass with one or
    two chunk groups in flight), and the mixed-verdict batch, on one lane and on eight."""
    rng = np.random.default_rng(seed)
    n = 5000
    sizes = rng.integers(60, 1515, n).astype(np.uint32)
    src = F.build_frames(sizes, np.full(n, 10001, np.uint32), seed)
    off = np.zeros(n, np.int64)
    pos = 3
    for i in range(n):
        off[i] = pos
        pos += int(sizes[i]) + int(rng.integers(0, 4))
    fr = np.zeros(pos + 256, np.uint8)
    for i in range(n):
        fr[off[i]:off[i] + sizes[i]] = src.frames[int(src.offset[i]):int(src.offset[i]) + int(sizes[i])]
        if rng.random() < 1 / 3:
            fr[off[i] + int(rng.integers(34, sizes[i]))] ^= 0x21
    b = F.Batch(fr, off.astype(np.uint32), sizes.astype(np.uint16), pos)
    want, got = _run(form_ctx, b)
    _same(want, got, f"tail seed={seed}")
    m = F.mixed_batch(seed, 3000, [10001, 10002], [9, 20000], ["172.31.100.1"], with_ptype=seed % 2 == 0)
    lists = {abi.raw_port(10001): [(0, 0, 0)], abi.raw_port(10002): [(0, 1, 0)]}
    want, got = _run(form_ctx, m, lists, 8)
    _same(want, got, f"mixed seed={seed}")


IP1, IP9 = "172.31.100.1", "172.31.100.9"


@pytest.mark.parametrize("nports", [5, 8, 9])
def test_bind_table_sizes(form_ctx, nports):
    """Ports with fan-out (REUSEPORT pairs), a specific address that does not match, ANY ahead of
    a specific binding, on 5, 8 (both in the arguments) and 9 (the port table) bound ports."""
    ports = [10001 + i for i in range(nports)]
    lists = {}
    for i, p in enumerate(ports):
        kind = i % 4
        if kind == 0:
            lists[abi.raw_port(p)] = [(0, i, 0)]
        elif kind == 1:
            lists[abi.raw_port(p)] = [(abi.raw_ip(IP1), i, 1), (abi.raw_ip(IP1), 20 + i, 1)]
        elif kind == 2:
            lists[abi.raw_port(p)] = [(abi.raw_ip(IP9), i, 0)]
        else:
            lists[abi.raw_port(p)] = [(0, i, 1), (abi.raw_ip(IP1), 20 + i, 1)]
    m = F.mixed_batch(50 + nports, 4000, ports, [9, 20000, 65535], [IP1, IP9])
    want, got = _run(form_ctx, m, lists, 32)
    _same(want, got, f"ports={nports}")


@pytest.mark.parametrize("cfg", [1, 2, 3])
def test_configs_forms(form_ctx, cfg):
    w = F.config_batch(cfg, n=60000)
    for _ in range(2):
        want, got = _run(form_ctx, w.batch, w.port_lists(), w.n_sockets)
        _same(want, got, w.name)


@pytest.mark.parametrize("group,hist_cap", [(1, 0), (2048, 0), (4096, 1 << 16), (8192, 1 << 16),
                                            (16384, 1 << 16), (16384, 0)])
def test_scatter_groups(group, hist_cap):
    """rx_scatterw taking G consecutive classify tiles per workgroup (UDPDK_SCATTER_GROUP_FRAMES
    frames at most; UDPDK_SCATTER_MIN_WG = 1 so small batches group too), with the 16-wave form
    past 8192 frames and the column scan writing only the groups' base rows; small histogram caps
    give many 1024-frame tiles and ragged last groups. Multi-lane batches (IMIX over 1024 ports,
    Zipf over 4096, a mixed batch with every verdict) equal the oracle bit for bit."""
    env = {"UDPDK_SCATTER_GROUP_FRAMES": str(group), "UDPDK_SCATTER_MIN_WG": "1"}
    if hist_cap:
        env["UDPDK_RX_HIST_CAP"] = str(hist_cap)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctx = abi.GpuContext(0, max_frames=1 << 20, max_lanes=4096)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for cfg, n in ((4, 50001), (5, 300000), (5, 1 << 20)):
            w = F.config_batch(cfg, n=n)
            _same(*_run(ctx, w.batch, w.port_lists(), w.n_sockets, cap=n), f"group {group} {w.name}")
        b = F.mixed_batch(7, 30000, [10001, 10002, 10003, 10004, 10005], [9, 20000, 65535],
                          ["172.31.100.1", "172.31.100.9"])
        lists = {abi.raw_port(10001): [(0, 0, 0)], abi.raw_port(10002): [(abi.raw_ip("172.31.100.1"), 1, 0)],
                 abi.raw_port(10003): [(abi.raw_ip("172.31.100.9"), 3, 0)], abi.raw_port(10004): [(0, 4, 0)]}
        _same(*_run(ctx, b, lists, 8, cap=4 * b.n), f"group {group} mixed")
    finally:
        ctx.close()
