"""Receive-side scaling parity (f4): udpdk_gpu_rss against the oracle's restatement (hash per
frame, redirection table, per-queue lists in arrival order) on mixed batches with every verdict
class, several redirection tables, hash-type sets and queue counts, ptype given or derived; frames
built from the published verification vectors; and full-size config 5 frames over 8 queues."""
import json
import os
import socket

import numpy as np
import pytest

import oracle as O
from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rss_vectors.json")))
KEY = bytes.fromhex(G["key"])


def _both(ctx, b, cf, ptype=None):
    reta = [cf.reta[i] for i in range(cf.reta_size)]
    want = O.rss(bytes(cf.key), cf.hash_types, reta, cf.n_queues, b.frames, b.frames_bytes,
                 b.offset, b.length, ptype)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length, ptype)
    db.frames_bytes = b.frames_bytes
    got = abi.rss_run(ctx, db, cf)
    for x in (db.frames, db.offset, db.length, db.ptype):
        if x is not None:
            x.free()
    return want, got


@pytest.mark.parametrize("nq,reta_size,types", [(8, 128, 3), (1, 1, 3), (64, 512, 3), (5, 64, 1),
                                                (3, 256, 2), (16, 128, 0)])
@pytest.mark.parametrize("with_ptype", [False, True])
def test_rss_mixed(gpu_ctx, nq, reta_size, types, with_ptype):
    b = F.mixed_batch(7 + nq, 5000, [10001, 10002, 10004], [9, 20000], ["172.31.100.1", "172.31.100.9"],
                      with_ptype=with_ptype)
    rng = np.random.default_rng(nq * 7 + reta_size)
    cf = abi.rss_conf(nq, reta=rng.integers(0, nq, reta_size), hash_types=types)
    (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, b, cf, b.ptype)
    assert np.array_equal(wh, gh)
    assert np.array_equal(wo, go)
    assert np.array_equal(wp, gp)


def test_rss_verification_frames(gpu_ctx):
    """UDP frames carrying the verification suite's addresses and ports hash to its values."""
    frames = []
    for v in G["ipv4"]:
        fr = bytearray(F.make_frame(np.random.default_rng(0), dport=v["dport"], dst_ip=v["dst"],
                                    src_ip=v["src"]))
        fr[34:36] = v["sport"].to_bytes(2, "big")
        frames.append(bytes(fr))
    off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint32)
    buf = np.zeros(int(off[-1]) + len(frames[-1]) + 64, np.uint8)
    for o, f in zip(off, frames):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    b = F.Batch(buf, off, np.array([len(f) for f in frames], np.uint16), len(buf) - 64)
    cf = abi.rss_conf(4)
    _, (gh, _, _) = _both(gpu_ctx, b, cf)
    assert [int(x) for x in gh] == [int(v["ipv4_l4"], 16) for v in G["ipv4"]]
    cf = abi.rss_conf(4, hash_types=1)
    _, (gh, _, _) = _both(gpu_ctx, b, cf)
    assert [int(x) for x in gh] == [int(v["ipv4"], 16) for v in G["ipv4"]]


@pytest.mark.parametrize("nq", [8, 64])
def test_rss_full_size_config5(gpu_ctx, nq):
    """4 M x 64 B over 4096 ports (Zipf): 8 queues take the one-workgroup base scan (rss_base),
    64 queues (4096 tiles x 64 entries) the three-pass column scan."""
    w = F.config_batch(5)
    (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, w.batch, abi.rss_conf(nq))
    assert np.array_equal(wh, gh) and np.array_equal(wo, go) and np.array_equal(wp, gp)
    assert go[-1] == w.batch.n


@pytest.mark.parametrize("nq,n", [(8, None), (7, None), (3, 700001)])
def test_rss_config4(gpu_ctx, nq, n):
    """1 M IMIX frames over 1024 ports (uniform destination ports, so every queue gets frames):
    the one-workgroup base scan over 1024 tiles x 8 queues; 7 queues and a ragged 700001-frame
    batch put queue rows across its threads' 32-entry boundaries."""
    w = F.config_batch(4, n=n)
    (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, w.batch, abi.rss_conf(nq))
    assert np.array_equal(wh, gh) and np.array_equal(wo, go) and np.array_equal(wp, gp)
    assert go[-1] == w.batch.n and np.all(np.diff(go.astype(np.int64)) > 0)


@pytest.mark.parametrize("fuse", ["0", "1"])
def test_rss_base_forms(gpu_ctx, monkeypatch, fuse):
    """The queue bases from the last rss_hash workgroup (fused, the default) and from the separate
    rss_base launch (UDPDK_RSS_FUSE=0, read by udpdk_gpu_rss_config), on a ragged IMIX batch, a
    small mixed one and a single frame, alternating on one context (the fan-in words reset)."""
    monkeypatch.setenv("UDPDK_RSS_FUSE", fuse)
    w = F.config_batch(4, n=300001)
    small = F.mixed_batch(13, 2500, [10001, 10002], [9], ["172.31.100.1"])
    one = F.mixed_batch(1, 1, [10001], [9], ["172.31.100.1"])
    for b, nq in ((w.batch, 8), (small, 5), (one, 2), (w.batch, 3), (small, 64)):
        (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, b, abi.rss_conf(nq))
        assert np.array_equal(wh, gh) and np.array_equal(wo, go) and np.array_equal(wp, gp)
        assert go[-1] == b.n


def test_rss_edges(gpu_ctx):
    """Empty batch, bad configurations, a single frame; the RSS call needs a configuration."""
    import ctypes as C
    cf = abi.rss_conf(4)
    assert abi.lib().udpdk_gpu_rss_config(gpu_ctx.handle, C.byref(cf)) == 0
    qo = gpu_ctx.alloc(4 * 5)
    bt = abi.RxBatch(None, 0, None, None, None, 0)
    assert abi.lib().udpdk_gpu_rss(gpu_ctx.handle, C.byref(bt), C.byref(abi.RssOut(None, qo.ptr, None))) == 0
    gpu_ctx.sync()
    assert np.array_equal(gpu_ctx.download(qo, np.uint32, 5), np.zeros(5, np.uint32))
    qo.free()
    for bad in (dict(n_queues=0), dict(n_queues=65), dict(reta_size=3), dict(reta_size=1024),
                dict(hash_types=4)):
        c2 = abi.rss_conf(4)
        for k, v in bad.items():
            setattr(c2, k, v)
        assert abi.lib().udpdk_gpu_rss_config(gpu_ctx.handle, C.byref(c2)) == -22, bad
    c3 = abi.rss_conf(4)
    c3.reta[0] = 4                                     # queue out of range
    assert abi.lib().udpdk_gpu_rss_config(gpu_ctx.handle, C.byref(c3)) == -22
    b = F.mixed_batch(1, 1, [10001], [9], ["172.31.100.1"])
    (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, b, abi.rss_conf(3))
    assert np.array_equal(wh, gh) and np.array_equal(wo, go) and np.array_equal(wp, gp)


def test_rss_repeats_of_different_sizes(gpu_ctx):
    """Calls of different sizes and queue counts alternate on one context (per-call histogram
    and list state): 1 M frames (4096 ports, Zipf) over 8 and 16 queues and a small mixed batch."""
    w = F.config_batch(5, n=1 << 20)
    small = F.mixed_batch(11, 3000, [10001, 10002, 10004], [9, 20000], ["172.31.100.1"])
    for b, nq in ((w.batch, 8), (small, 8), (w.batch, 16), (w.batch, 8), (small, 3), (w.batch, 8)):
        (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, b, abi.rss_conf(nq))
        assert np.array_equal(wh, gh) and np.array_equal(wo, go) and np.array_equal(wp, gp)
        assert go[-1] == b.n


@pytest.mark.parametrize("seed", [41, 42])
def test_rss_fuzzed_headers_and_descriptors(gpu_ctx, seed):
    """Header bits flipped in 30 % of the frames (ether_type, flags, protocol, addresses, ports),
    5 % of the offsets moved to any byte (past the batch included), 5 % of the lengths set to edge
    values around the 34- and 38-byte hash inputs: hashes and queue lists equal the oracle's."""
    rng = np.random.default_rng(seed)
    base = F.mixed_batch(seed, 4000, [10001, 10002], [9, 20000], ["172.31.100.1", "172.31.100.9"],
                         with_ptype=seed % 2 == 0)
    fr = base.frames.copy()
    for i in rng.choice(base.n, base.n * 3 // 10, replace=False):
        o = int(base.offset[i])
        for _ in range(int(rng.integers(1, 4))):
            pos = o + 12 + int(rng.integers(0, 28))
            if pos < base.frames_bytes:
                fr[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    off = base.offset.astype(np.uint64).copy()
    ln = base.length.astype(np.uint32).copy()
    k = rng.choice(base.n, base.n // 20, replace=False)
    off[k] = rng.integers(0, base.frames_bytes + 5000, len(k))
    k = rng.choice(base.n, base.n // 20, replace=False)
    ln[k] = rng.choice([0, 13, 14, 33, 34, 35, 37, 38, 39, 65535], len(k))
    b = F.Batch(fr, off.astype(np.uint32), ln.astype(np.uint16), base.frames_bytes, base.ptype)
    cf = abi.rss_conf(8, reta=rng.integers(0, 8, 128), hash_types=3)
    (wh, wo, wp), (gh, go, gp) = _both(gpu_ctx, b, cf, b.ptype)
    assert np.array_equal(wh, gh)
    assert np.array_equal(wo, go)
    assert np.array_equal(wp, gp)
