"""Payload delivery parity (f1): udpdk_gpu_rx_gather, the batch form of udpdk_recvfrom
(udpdk_syscall.c:401-488), against the oracle's restatement on the lanes the RX pipeline
produced: payload bytes (padding trimmed, truncated to the slot), lengths, source addresses."""
import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

IP1, IP9 = "172.31.100.1", "172.31.100.9"
LISTS = {
    abi.raw_port(10001): [(0, 0, 0)],
    abi.raw_port(10002): [(abi.raw_ip(IP1), 1, 1), (abi.raw_ip(IP1), 2, 1)],
    abi.raw_port(10004): [(0, 4, 1), (abi.raw_ip(IP1), 5, 1)],
}


def _gather_both(ctx, b, lists, n_lanes, slot, ranges=None):
    ctx.upload_snapshot(abi.snapshot_from_lists(lists, n_lanes))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length, b.ptype)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, n_lanes, max(1, 4 * b.n))
    meta, loff, pkt, cnt, rc = abi.rx_run(ctx, db, out)
    assert rc == 0
    d = int(loff[-1])
    ranges = ranges or [(0, d)]
    res = []
    for first, count in ranges:
        g = abi.rx_alloc_gather(ctx, count, slot)
        got = abi.rx_gather_run(ctx, db, out.lane_pkt, first, g)
        want = O.recv_gather(b.frames, b.offset, b.length, pkt, first, count, slot)
        res.append((want, got))
        for x in (g.payload, g.length, g.src_ip, g.src_port):
            x.free()
    for x in (db.frames, db.offset, db.length, db.ptype, out.meta, out.lane_off, out.lane_pkt):
        if x is not None:
            x.free()
    return res, loff


def _assert_same(want, got, ctx=""):
    wp, wl, wi, ws = want
    gp, gl, gi, gs = got
    assert np.array_equal(wl, gl), ctx
    assert np.array_equal(wi, gi), ctx
    assert np.array_equal(ws, gs), ctx
    for k in np.nonzero(wl)[0]:
        n = int(wl[k])
        assert np.array_equal(wp[k, :n], gp[k, :n]), f"{ctx}: payload {k}"


@pytest.mark.parametrize("slot", [16, 64, 2048])
def test_gather_mixed(gpu_ctx, slot):
    b = F.mixed_batch(7, 3000, [10001, 10002, 10004], [9, 20000], [IP1, IP9])
    res, _ = _gather_both(gpu_ctx, b, LISTS, 8, slot)
    for want, got in res:
        _assert_same(want, got, f"slot={slot}")


def test_gather_per_socket_ranges(gpu_ctx):
    b = F.mixed_batch(11, 2000, [10001, 10002, 10004], [9], [IP1])
    ctx = gpu_ctx
    ctx.upload_snapshot(abi.snapshot_from_lists(LISTS, 8))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, 8, 4 * b.n)
    _, loff, pkt, _, _ = abi.rx_run(ctx, db, out)
    for s in range(8):
        first, count = int(loff[s]), int(loff[s + 1] - loff[s])
        if not count:
            continue
        g = abi.rx_alloc_gather(ctx, count, 2048)
        got = abi.rx_gather_run(ctx, db, out.lane_pkt, first, g)
        want = O.recv_gather(b.frames, b.offset, b.length, pkt, first, count, 2048)
        _assert_same(want, got, f"socket {s}")


@pytest.mark.parametrize("cfg,n", [(2, 50000), (3, 20000), (4, 30000)])
def test_gather_configs(gpu_ctx, cfg, n):
    w = F.config_batch(cfg, n=n)
    res, _ = _gather_both(gpu_ctx, w.batch, w.port_lists(), w.n_sockets, 2048)
    for want, got in res:
        _assert_same(want, got, w.name)
        assert int(want[1].sum()) == int(got[1].sum()) > 0


@pytest.mark.parametrize("caps", ["frame", "random"])
def test_gather_packed_slots(gpu_ctx, caps):
    """udpdk_gpu_rx_gather_packed (the slabs udpdk_poll_rx fills): entry k lands at slot_off[k]
    with slot_off[k + 1] - slot_off[k] bytes of room. Caps sized to each frame (data_len - 42
    rounded up to 16: nothing truncated) or random multiples of 16 (recvfrom truncation per
    entry); lengths, addresses and bytes vs the oracle's untruncated recvfrom cut to the cap."""
    w = F.config_batch(4, n=20000)
    b = w.batch
    ctx = gpu_ctx
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, w.n_sockets, b.n)
    _, loff, pkt, _, rc = abi.rx_run(ctx, db, out)
    assert rc == 0
    d = int(loff[-1])
    assert d == b.n
    rng = np.random.default_rng(3 if caps == "frame" else 4)
    if caps == "frame":
        cap = (np.maximum(b.length[pkt[:d]].astype(np.int64) - 42, 1) + 15) // 16 * 16
    else:
        cap = rng.integers(1, 100, d) * 16
    so = np.concatenate([[0], np.cumsum(cap)]).astype(np.uint32)
    gp, gl, gi, gs = abi.rx_gather_packed_run(ctx, db, out.lane_pkt, 0, so)
    wp, wl, wi, ws = O.recv_gather(b.frames, b.offset, b.length, pkt, 0, d, 2048)   # IMIX <= 1476 B
    want_len = np.minimum(wl, cap)
    assert np.array_equal(gl, want_len) and np.array_equal(gi, wi) and np.array_equal(gs, ws)
    if caps == "frame":
        assert np.array_equal(want_len, wl)                      # nothing truncated
    else:
        assert np.any(want_len < wl)
    for k in range(d):
        n = int(want_len[k])
        assert gp[so[k]:so[k] + n].tobytes() == wp[k, :n].tobytes(), k
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
        x.free()
