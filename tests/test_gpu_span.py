"""The span sweep of rx_classify<2, 0> (RxArgs::span): a step of 64 frames that lie in ascending
order, each within 128 bytes of the previous frame's end, reads its byte span once on a line grid;
header windows come from an LDS ring, UDP checksums from prefix sums over the span minus each
frame's lead bytes (below offset + 64 in its first piece) and the bytes past its end in its last
piece. These batches put frame starts, tail starts and ends at every residue of the 16-byte piece
and 1 KiB block grid, corrupt the bytes those corrections touch, mix in padded datagrams (the tail
pass takes those), gaps on both sides of the 128-byte limit, odd offsets, frames of up to 65535
bytes (prefix sums that wrap 2^32) and a last frame ending at the buffer's end. Each batch runs
on a context with the sweep and one without; both must equal the oracle bit for bit."""
import os

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

LISTS = {abi.raw_port(10001): [(0, 0, 0)], abi.raw_port(10002): [(0, 1, 0)]}


def _ctx(span):
    old = {k: os.environ.get(k) for k in ("UDPDK_RX_SPAN", "UDPDK_RX_TAILG")}
    os.environ["UDPDK_RX_SPAN"] = str(span)
    os.environ["UDPDK_RX_TAILG"] = "2"
    try:
        return abi.GpuContext(0, max_frames=1 << 18, max_lanes=1024)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=[1, 0], ids=["span", "nospan"])
def ctx(request):
    c = _ctx(request.param)
    yield c
    c.close()


def _run(ctx, b, n_lanes=2):
    ctx.upload_snapshot(abi.snapshot_from_lists(LISTS, n_lanes))
    want = O.rx(O.bindtable_from_lists(LISTS), b.frames, b.frames_bytes, b.offset, b.length, b.ptype,
                n_lanes, 0xFFFFFFFF)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length, b.ptype)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, b.n, n_lanes, max(1, b.n))
    got = abi.rx_run(ctx, db, out)
    for x in (db.frames, db.offset, db.length, db.ptype, out.meta, out.lane_off, out.lane_pkt):
        if x is not None:
            x.free()
    wm, wl, wp, wc = want
    gm, gl, gp, gc, rc = got
    assert rc == 0
    bad = np.nonzero(wm != gm)[0]
    assert len(bad) == 0, f"verdict words differ at {bad[:8]}: {wm[bad[:4]]} vs {gm[bad[:4]]}"
    assert np.array_equal(wl, gl)
    assert np.array_equal(wp[:len(gp)], gp)
    assert np.array_equal(wc, gc)
    return wm


def _relayout(src, start, gaps, tailroom=16):
    """src's frames re-placed from byte `start` with gaps[i] bytes after frame i."""
    n = src.n
    sizes = src.length.astype(np.int64)
    off = np.zeros(n, np.int64)
    pos = start
    for i in range(n):
        off[i] = pos
        pos += int(sizes[i]) + int(gaps[i])
    end = int(off[-1] + sizes[-1])
    fr = np.zeros((end + tailroom + 15) // 16 * 16, np.uint8)
    fr[:start] = 0xA5
    for i in range(n):
        o = int(src.offset[i])
        fr[off[i]:off[i] + sizes[i]] = src.frames[o:o + int(sizes[i])]
        g = int(gaps[i])
        if g and i + 1 < n:
            fr[off[i] + sizes[i]:off[i] + sizes[i] + g] = 0x5A
    return F.Batch(fr, off.astype(np.uint32), sizes.astype(np.uint16), end)


def _corrupt(rng, b, frac=0.5):
    """Flip one byte of about frac of the frames, at positions the sweep's corrections touch."""
    for i in np.nonzero(rng.random(b.n) < frac)[0]:
        L = int(b.length[i])
        if L <= 42:
            continue
        o = int(b.offset[i])
        lead = 64 - ((o + 64) & 15)                 # first byte of the piece holding byte 64
        cand = [34, 40, 41, 63, 64, 65, lead, lead + 1, L - 1, L - 2, L - 16, int(rng.integers(42, L))]
        k = min(L - 1, max(34, cand[int(rng.integers(0, len(cand)))]))
        b.frames[o + k] ^= np.uint8(1 << int(rng.integers(0, 8)))


@pytest.mark.parametrize("start", [0, 1, 2, 3, 15, 17, 64, 127, 1000])
def test_span_every_residue(ctx, start):
    rng = np.random.default_rng(100 + start)
    n = 6000
    sizes = rng.integers(64, 1515, n).astype(np.uint32)
    src = F.build_frames(sizes, np.where(rng.random(n) < 0.9, 10001, 10002).astype(np.uint32), start)
    b = _relayout(src, start, np.zeros(n, np.int64))
    _corrupt(rng, b)
    _run(ctx, b)


@pytest.mark.parametrize("seed", [1, 2])
def test_span_gaps(ctx, seed):
    """Gaps of 0-127 bytes (swept) and, in some steps, 128-300 (those steps take windows + tails),
    odd and even; a short frame (42-63 B) now and then inside swept steps."""
    rng = np.random.default_rng(seed)
    n = 8000
    sizes = rng.integers(100, 1515, n).astype(np.uint32)
    sizes[rng.random(n) < 0.05] = 50
    src = F.build_frames(sizes, np.full(n, 10001, np.uint32), seed)
    gaps = rng.integers(0, 128, n)
    steps_far = rng.random(n // 64 + 1) < 0.25
    for s in np.nonzero(steps_far)[0]:
        i = min(n - 1, 64 * s + int(rng.integers(0, 64)))
        gaps[i] = int(rng.integers(128, 300))
    b = _relayout(src, 5, gaps)
    _corrupt(rng, b, 0.3)
    _run(ctx, b)


def test_span_padded_datagrams(ctx):
    """Datagrams shorter than their frames (Ethernet padding or trailing bytes after the UDP
    length): checksummed over the datagram only, by the tail pass inside swept steps."""
    rng = np.random.default_rng(7)
    out = bytearray()
    offs, lens = [], []
    for i in range(4000):
        r = rng.random()
        if r < 0.3:
            f = F.make_frame(rng, dport=10001, payload_len=int(rng.integers(30, 1400)),
                             pad=int(rng.integers(1, 60)), udp_cksum="ok" if rng.random() < 0.7 else "bad")
        elif r < 0.4:
            f = F.make_frame(rng, dport=10002, payload_len=int(rng.integers(0, 20)), pad=int(rng.integers(1, 100)))
        else:
            f = F.make_frame(rng, dport=10001, payload_len=int(rng.integers(60, 1460)),
                             udp_cksum="ok" if rng.random() < 0.8 else "bad")
        offs.append(len(out))
        lens.append(len(f))
        out += f
        out += bytes(int(rng.integers(0, 3)))
    fr = np.zeros(len(out) + 256, np.uint8)
    fr[:len(out)] = np.frombuffer(bytes(out), np.uint8)
    b = F.Batch(fr, np.array(offs, np.uint32), np.array(lens, np.uint16), offs[-1] + lens[-1])
    _run(ctx, b)


def test_span_large_frames_and_buffer_end(ctx):
    """Frames up to 65535 bytes (one step's prefix sums pass 2^32 and wrap), 1514-byte and 9000-byte
    runs, a partial last step, and the last frame ending exactly at frames_bytes with only the ABI's
    16 bytes of tailroom after it."""
    rng = np.random.default_rng(9)
    sizes = np.concatenate([np.full(130, 1514), rng.integers(60000, 65536, 70), np.full(200, 9000),
                            rng.integers(64, 1515, 333)]).astype(np.uint32)
    src = F.build_frames(sizes, np.full(len(sizes), 10001, np.uint32), 9, chunk=64)
    b = _relayout(src, 3, np.zeros(len(sizes), np.int64), tailroom=16)
    _corrupt(rng, b, 0.4)
    _run(ctx, b)


@pytest.mark.parametrize("cfg", [1, 3, 4])
def test_span_configs(ctx, cfg):
    """BASELINE configs 1 (106 B), 3 (1500 B) and 4 (IMIX over 1024 sockets), reduced."""
    w = F.config_batch(cfg, n=70000)
    lists = w.port_lists()
    ctx.upload_snapshot(abi.snapshot_from_lists(lists, w.n_sockets))
    want = O.rx(O.bindtable_from_lists(lists), w.batch.frames, w.batch.frames_bytes, w.batch.offset,
                w.batch.length, w.batch.ptype, w.n_sockets, 0xFFFFFFFF)
    db = abi.rx_upload(ctx, w.batch.frames, w.batch.offset, w.batch.length, w.batch.ptype)
    db.frames_bytes = w.batch.frames_bytes
    out = abi.rx_alloc_out(ctx, w.batch.n, w.n_sockets, w.batch.n)
    got = abi.rx_run(ctx, db, out)
    for x in (db.frames, db.offset, db.length, db.ptype, out.meta, out.lane_off, out.lane_pkt):
        if x is not None:
            x.free()
    assert got[4] == 0
    for a, g in zip(want, got[:4]):
        assert np.array_equal(a, g)
