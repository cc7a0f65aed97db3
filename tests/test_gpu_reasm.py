"""RX reassembly parity (f2): udpdk_gpu_rx_reassemble against the oracle's restatement of the
poller's rte_ipv4_frag_reassemble_packet step (oracle_reassemble), over multi-batch seeded
scenarios with shuffled, lost, duplicated, overlapping and hole-making fragments, flow expiry and
key reuse; the reassembled datagrams then go through udpdk_gpu_rx (the demux the reference runs
on them) and are compared with the oracle's RX of the oracle's datagrams. Plus a GPU-only loop:
udpdk_gpu_tx_build_mtu's fragments come back as the datagrams that were sent."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from reasm_util import batch, scenario
from udpdk_amd import abi

pytestmark = pytest.mark.gpu

PORTS = (10000, 10001, 10002, 10003)
LISTS = {abi.raw_port(p): [(0, k, 0)] for k, p in enumerate(PORTS)}


def _frames(ctx, rb):
    off = abi.download_ptr(ctx, rb.offset.ptr, np.uint32, rb.n)
    ln = abi.download_ptr(ctx, rb.length.ptr, np.uint16, rb.n)
    buf = abi.download_ptr(ctx, rb.frames.ptr, np.uint8, rb.frames_bytes)
    return buf, off, ln


def _check_scenario(gpu_ctx, frames_tms, geometry, inplace=False, pad=True):
    """Run a multi-batch scenario through the GPU and the oracle: every datagram, origin, length
    and outcome count exact (including "expired" and "stored", which depend on which flow gets
    which table entry when); then the demux of the reassembled datagrams. Returns the totals."""
    abi.frag_table_create(gpu_ctx, **geometry)
    t = O.FragTable(**geometry)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists(LISTS, 4))
    bt = O.bindtable_from_lists(LISTS)
    tot = {}
    for b, (frames, tms) in enumerate(frames_tms):
        buf, off, ln = batch(frames, pad=pad)
        n = len(off)
        db = abi.rx_upload(gpu_ctx, buf, off, ln)
        db.frames_bytes = len(buf) - 64
        out = abi.rx_alloc_out(gpu_ctx, n, 4, 4 * n)
        gm, gl, gp, gc, rc = abi.rx_run(gpu_ctx, db, out)
        wm, wl, wp, wc = O.rx(bt, buf, len(buf) - 64, off, ln, None, 4)
        assert rc == 0 and np.array_equal(gm, wm)
        rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, tms, inplace=inplace)
        wout, woo, wol, wog, wst = t.reassemble(buf, off, ln, wm, tms)
        tot["in_place"] = tot.get("in_place", 0) + int(rb.n > 0 and rb.frames.ptr == db.frames.ptr)
        serial = gst.pop("serial")
        tot["sorted"] = tot.get("sorted", 0) + gst.pop("sorted")
        assert gst == wst, f"batch {b}: stats {gst} vs {wst}"
        assert rb.n == len(woo)
        for k, v in gst.items():
            tot[k] = tot.get(k, 0) + v
        tot["serial"] = tot.get("serial", 0) + serial
        if rb.n:
            gbuf, goff, gln = _frames(gpu_ctx, rb)
            gorg = abi.download_ptr(gpu_ctx, origin.ptr, np.uint32, rb.n)
            assert np.array_equal(gorg, wog) and np.array_equal(gln, wol)
            for k in range(rb.n):
                g = gbuf[goff[k]:goff[k] + gln[k]].tobytes()
                w = wout[woo[k]:woo[k] + wol[k]].tobytes()
                assert g == w, f"batch {b} datagram {k}"
            # the demux of the reassembled datagrams (poller.c:362-412 after reassembly)
            out2 = abi.rx_alloc_out(gpu_ctx, rb.n, 4, 4 * rb.n)
            g2 = abi.rx_run(gpu_ctx, rb, out2)
            w2 = O.rx(bt, wout, len(wout), woo, wol, np.full(rb.n, 0x211, np.uint32), 4)
            assert g2[4] == 0
            for x, y in zip(w2[:3], g2[:3]):
                assert np.array_equal(x, y)
            assert np.all(abi.meta_verdict(g2[0]) == 0)          # every datagram delivered
            assert np.all(abi.meta_udp(g2[0]) == 0)             # checksum 0: "absent"
            for bb in (out2.meta, out2.lane_off, out2.lane_pkt):
                bb.free()
        for bb in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
            bb.free()
    return tot


@pytest.mark.parametrize("seed", [5, 6, 7])
def test_reassembly_matches_oracle(gpu_ctx, seed):
    tot = _check_scenario(gpu_ctx, scenario(seed), dict(bucket_num=256, bucket_entries=16, max_cycles=25))
    for k in ("errors", "holes", "expired", "done", "stored"):
        assert tot[k] > 0, (k, tot)
    assert 0 < tot["serial"] < tot["frags"], tot          # both paths ran
    assert tot["sorted"] > 0, tot                         # shuffled arrival: the sorted path


@pytest.mark.parametrize("inplace", [False, True])
def test_reassembly_unpadded_short_fragments(gpu_ctx, inplace):
    """Frames as sent, without Ethernet padding: a last fragment of 1-7 data bytes is a 34-41 B
    frame, shorter than the 42-byte Eth/IPv4/UDP header. The poller hands any fragment to
    rte_ipv4_frag_reassemble_packet on its IPv4 header alone (poller.c:338-361), so such frames get
    the FRAG verdict (shorter non-fragments stay TRUNC) and their datagrams complete: verdicts,
    datagrams and counts equal the oracle's."""
    fts = scenario(43, n_batches=4, flows_per_batch=90, dt=12, grouped=True)
    short = sum(1 for fs, _ in fts for f in fs if 34 <= len(f) < 42 and (f[20] & 0x3F or f[21]))
    assert short >= 10, short                             # the scenario has short fragments
    tot = _check_scenario(gpu_ctx, fts, dict(bucket_num=256, bucket_entries=16, max_cycles=20),
                          inplace=inplace, pad=False)
    assert tot["done"] > 0, tot


@pytest.mark.parametrize("seed,buckets,entries", [(21, 256, 16), (22, 4, 4), (23, 1, 8)])
def test_reassembly_grouped_batches_exact(gpu_ctx, seed, buckets, entries):
    """Fragments of each datagram back to back (the grouped path: no key sorts, no overlap test,
    completions by a select) with flows cut by batch boundaries, lost fragments, duplicates and
    flow expiry; tables from roomy to far too small: every outcome equals the oracle's."""
    tot = _check_scenario(gpu_ctx, scenario(seed, n_batches=5, flows_per_batch=90, dt=12, grouped=True),
                          dict(bucket_num=buckets, bucket_entries=entries, max_cycles=20))
    for k in ("done", "stored", "expired"):
        assert tot[k] > 0, (k, tot)
    assert tot["sorted"] == 0, tot                        # every batch took the grouped path


@pytest.mark.parametrize("seed,buckets,entries,grouped", [(21, 256, 16, True), (24, 256, 16, True), (22, 4, 4, True),
                                                         (11, 4, 4, False)])
def test_reassembly_inplace_scenarios_exact(gpu_ctx, seed, buckets, entries, grouped):
    """udpdk_gpu_rx_reassemble_inplace over the multi-batch scenarios: a batch whose completions
    all have their fragments back to back and in order is reassembled in place, any other falls
    back to the copy; either way every datagram, origin and count equals the oracle's."""
    tot = _check_scenario(gpu_ctx, scenario(seed, n_batches=5, flows_per_batch=90, dt=12, grouped=grouped),
                          dict(bucket_num=buckets, bucket_entries=entries, max_cycles=20), inplace=True)
    assert tot["done"] > 0, tot


def _check_frag_batch(gpu_ctx, b, n_dgrams, inplace, expect_inplace):
    """One batch of frames.frag_batch through the GPU and the oracle at the bench's table
    geometry: counts, datagrams, origins and their demux equal; in place when expected."""
    geometry = dict(bucket_num=0x1000, bucket_entries=16, max_cycles=1 << 40)
    abi.frag_table_create(gpu_ctx, geometry["bucket_num"], geometry["bucket_entries"], geometry["max_cycles"], 65515)
    t = O.FragTable(**geometry)
    from udpdk_amd import frames as FR
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(FR.PORT_RECV): [(0, 0, 0)]}, 4))
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, b.n, 4, 4 * b.n)
    gm = abi.rx_run(gpu_ctx, db, out)[0]
    rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, 0, inplace=inplace)
    wout, woo, wol, wog, wst = t.reassemble(b.frames, b.offset, b.length, gm, 0)
    gst.pop("serial"), gst.pop("sorted")
    assert gst == wst and gst["done"] == n_dgrams, (gst, wst)
    assert (rb.frames.ptr == db.frames.ptr) == expect_inplace
    gbuf, goff, gln = _frames(gpu_ctx, rb)
    gorg = abi.download_ptr(gpu_ctx, origin.ptr, np.uint32, rb.n)
    assert np.array_equal(gorg, wog) and np.array_equal(gln, wol)
    for k in range(rb.n):
        assert gbuf[goff[k]:goff[k] + gln[k]].tobytes() == wout[woo[k]:woo[k] + wol[k]].tobytes(), k
    out2 = abi.rx_alloc_out(gpu_ctx, rb.n, 4, 4 * rb.n)
    g2 = abi.rx_run(gpu_ctx, rb, out2)
    assert g2[4] == 0 and np.all(abi.meta_verdict(g2[0]) == 0) and np.all(abi.meta_udp(g2[0]) == abi.UDP_OK)
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt, out2.meta,
              out2.lane_off, out2.lane_pkt):
        x.free()


@pytest.mark.parametrize("payload", [2952, 2951, 4001, 5900])
def test_reassembly_inplace_in_order(gpu_ctx, payload):
    """Fragments of each datagram back to back and in order (frames.frag_batch, the bench's
    workload: 2, 3 and 4 fragments, odd frame sizes so later datagrams start at odd offsets): the
    call reassembles every datagram in place (the output batch is the input buffer) and the
    datagrams, origins, counts and their demux equal the oracle's."""
    from udpdk_amd import frames as FR
    _check_frag_batch(gpu_ctx, FR.frag_batch(3000, payload), 3000, True, True)


def _frames_flat(buf, off, ln):
    """The bytes of frames (off, ln) of buf, concatenated (vectorised)."""
    off = off.astype(np.int64)
    ln = ln.astype(np.int64)
    starts = np.repeat(off - np.concatenate(([0], np.cumsum(ln)[:-1])), ln)
    return buf[starts + np.arange(int(ln.sum()))]


@pytest.mark.parametrize("inplace", [False, True])
def test_reassembly_at_capacity(gpu_ctx, inplace):
    """The context's largest batch (2^22 frames: 2^21 two-fragment datagrams at MTU 68, so
    every FRAG count block and scan block of the grouped path is full): counts, origins, lengths
    and every datagram byte equal the oracle's; in place when asked."""
    from udpdk_amd import frames as FR
    n_d = 1 << 21
    b = FR.frag_batch(n_d, 60, mtu=68)
    assert b.n == 1 << 22
    geometry = dict(bucket_num=0x1000, bucket_entries=16, max_cycles=1 << 40)
    abi.frag_table_create(gpu_ctx, geometry["bucket_num"], geometry["bucket_entries"], geometry["max_cycles"], 65515)
    t = O.FragTable(**geometry)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(FR.PORT_RECV): [(0, 0, 0)]}, 4))
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, b.n, 4, 4 * b.n)
    gm = abi.rx_run(gpu_ctx, db, out)[0]
    rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, 0, inplace=inplace)
    wout, woo, wol, wog, wst = t.reassemble(b.frames, b.offset, b.length, gm, 0)
    gst.pop("serial"), gst.pop("sorted")
    assert gst == wst and gst["done"] == n_d, (gst, wst)
    assert (rb.frames.ptr == db.frames.ptr) == inplace
    gbuf, goff, gln = _frames(gpu_ctx, rb)
    gorg = abi.download_ptr(gpu_ctx, origin.ptr, np.uint32, rb.n)
    assert np.array_equal(gorg, wog) and np.array_equal(gln, wol)
    assert np.array_equal(_frames_flat(gbuf, goff, gln), _frames_flat(wout, woo, wol))
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
        x.free()


def _reorder(b, order):
    """The frames of batch b in the given order, packed again (a Batch-like namespace)."""
    import types
    buf, off, ln = batch([b.frames[int(b.offset[x]):int(b.offset[x]) + int(b.length[x])].tobytes() for x in order])
    return types.SimpleNamespace(frames=buf, offset=off, length=ln, n=len(off), frames_bytes=len(buf) - 64)


@pytest.mark.parametrize("case", ["split_last", "split_first", "shuffled", "shuffled_large", "shuffled_wide"])
def test_reassembly_run_test_at_scale(gpu_ctx, case):
    """40 000 fragments over many reasm_scan blocks with one key split into two runs far apart
    (a datagram's last or first fragment moved to the batch's end), or the whole batch shuffled
    (also at 80 000 fragments, beyond 2^16 positions; shuffled_wide in 2^16 buckets, so the
    overlap records' (bucket, position) keys take 33 bits): the run test must find the batch not
    grouped (the sorted path, "sorted" = 1) and every outcome equals the oracle's."""
    from udpdk_amd import frames as FR
    n_d = 40000 if case in ("shuffled_large", "shuffled_wide") else 20000
    b = FR.frag_batch(n_d, 2952)
    order = list(range(b.n))
    if case == "split_last":
        order.remove(2 * 12345 + 1)
        order.append(2 * 12345 + 1)
    elif case == "split_first":
        order.remove(2 * 7)
        order.append(2 * 7)
    else:
        order = list(np.random.default_rng(3).permutation(b.n))
    sb = _reorder(b, order)
    geometry = dict(bucket_num=1 << 16 if case == "shuffled_wide" else 0x1000, bucket_entries=16, max_cycles=1 << 40)
    abi.frag_table_create(gpu_ctx, geometry["bucket_num"], geometry["bucket_entries"], geometry["max_cycles"], 65515)
    t = O.FragTable(**geometry)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(FR.PORT_RECV): [(0, 0, 0)]}, 4))
    db = abi.rx_upload(gpu_ctx, sb.frames, sb.offset, sb.length)
    db.frames_bytes = sb.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, sb.n, 4, 4 * sb.n)
    gm = abi.rx_run(gpu_ctx, db, out)[0]
    rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, 0)
    wout, woo, wol, wog, wst = t.reassemble(sb.frames, sb.offset, sb.length, gm, 0)
    gst.pop("serial")
    assert gst.pop("sorted") == 1
    assert gst == wst and gst["done"] == n_d, (gst, wst)
    gbuf, goff, gln = _frames(gpu_ctx, rb)
    gorg = abi.download_ptr(gpu_ctx, origin.ptr, np.uint32, rb.n)
    assert np.array_equal(gorg, wog) and np.array_equal(gln, wol)
    assert np.array_equal(_frames_flat(gbuf, goff, gln), _frames_flat(wout, woo, wol))
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
        x.free()


@pytest.mark.parametrize("cc", [1, 0])
@pytest.mark.parametrize("buckets,entries", [(512, 16), (64, 4)])
def test_reassembly_interleaved_serial_components(gpu_ctx, monkeypatch, cc, buckets, entries):
    """Pairs of flows interleaved (A1 B1 A2 B2 over 20 000 datagrams, then a second batch with the
    pairs' order reversed): flows whose spans overlap on a shared bucket go through the table. With
    UDPDK_RS_CC (default) the serial fragments are split by bucket component, one wave per
    component; without, one wave takes them all. Both equal the oracle exactly, in roomy and
    crowded tables (entries expire, held fragments, no space)."""
    from udpdk_amd import frames as FR
    monkeypatch.setenv("UDPDK_RS_CC", str(cc))
    b = FR.frag_batch(20000, 2952)
    pairs = np.arange(b.n).reshape(-1, 2, 2)
    geometry = dict(bucket_num=buckets, bucket_entries=entries, max_cycles=20)
    abi.frag_table_create(gpu_ctx, geometry["bucket_num"], geometry["bucket_entries"], geometry["max_cycles"], 65515)
    t = O.FragTable(**geometry)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(FR.PORT_RECV): [(0, 0, 0)]}, 4))
    serial = 0
    for step, order in enumerate((pairs.transpose(0, 2, 1).reshape(-1), pairs[:, ::-1, :].transpose(0, 2, 1).reshape(-1))):
        sb = _reorder(b, list(order))
        db = abi.rx_upload(gpu_ctx, sb.frames, sb.offset, sb.length)
        db.frames_bytes = sb.frames_bytes
        out = abi.rx_alloc_out(gpu_ctx, sb.n, 4, 4 * sb.n)
        gm = abi.rx_run(gpu_ctx, db, out)[0]
        tms = 10 * step
        rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, tms)
        wout, woo, wol, wog, wst = t.reassemble(sb.frames, sb.offset, sb.length, gm, tms)
        serial += gst.pop("serial")
        gst.pop("sorted")
        assert gst == wst, (step, gst, wst)
        gbuf, goff, gln = _frames(gpu_ctx, rb)
        gorg = abi.download_ptr(gpu_ctx, origin.ptr, np.uint32, rb.n)
        assert np.array_equal(gorg, wog) and np.array_equal(gln, wol)
        assert np.array_equal(_frames_flat(gbuf, goff, gln), _frames_flat(wout, woo, wol))
        for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt):
            x.free()
    assert serial >= 64, serial                           # the component path ran


@pytest.mark.parametrize("run,inplace", [(150, True), (150, False), (700, True), (700, False)])
def test_reassembly_long_same_key_runs(gpu_ctx, run, inplace):
    """`run` consecutive datagrams share one flow key (each completes before the next one's first
    fragment, so ip_frag_find gives the next a fresh entry): one flow segment of 2 x run positions,
    walked past its wave's and its block's positions, with completions in the next completion-list
    chunk (150: the speculative tail counts them; in place) or in several (700: the host counts
    again; the batch is copied). Datagrams, origins and counts equal the oracle's."""
    b = _same_key_batch(3000, run, (200, 1500))      # positions 400.. and 3000..: across 512, 3072
    _check_frag_batch(gpu_ctx, b, 3000, inplace, inplace and run == 150)


def _same_key_batch(n, run, starts):
    """frames.frag_batch(n, 2952) with datagrams a0 .. a0 + run - 1 given datagram a0's IPv4 id
    for each a0 in starts (IPv4 header checksums redone)."""
    from udpdk_amd import frames as FR
    b = FR.frag_batch(n, 2952)
    fr = b.frames
    for a0 in starts:
        for k in range(a0, a0 + run):
            for j in range(2):
                o = int(b.offset[2 * k + j])
                fr[o + 18], fr[o + 19] = a0 & 0xFF, a0 >> 8      # datagram a0's IPv4 id
                fr[o + 24] = fr[o + 25] = 0
                h = fr[o + 14:o + 34].astype(np.uint64)
                c = int(h[0::2].sum() + 256 * h[1::2].sum())
                while c >> 16:
                    c = (c & 0xFFFF) + (c >> 16)
                c = ~c & 0xFFFF
                fr[o + 24], fr[o + 25] = c & 0xFF, c >> 8
    return b


@pytest.mark.parametrize("inplace", [False, True])
def test_reassembly_sparse_fragments_long_runs(gpu_ctx, inplace):
    """Fragments between ordinary datagrams (1-3 after each fragment), with a key reused by 300
    consecutive datagrams: the fragment list's positions of a block come from several count
    blocks of frames, and the long flow's walk finds its fragments past its block among the
    other frames. Every outcome equals the oracle's; fragments that are not back to back are
    copied, not joined in place."""
    import types
    from udpdk_amd import frames as FR
    b = _same_key_batch(1200, 300, (100,))
    other = FR.build_frames(np.full(3000, 200, np.uint32), np.full(3000, FR.PORT_RECV + 1, np.uint32), 77)
    rng = np.random.default_rng(9)
    fl, k = [], 0
    for x in range(b.n):
        o, ln = int(b.offset[x]), int(b.length[x])
        fl.append(b.frames[o:o + ln].tobytes())
        for _ in range(int(rng.integers(1, 4))):
            oo, ol = int(other.offset[k % other.n]), int(other.length[k % other.n])
            fl.append(other.frames[oo:oo + ol].tobytes())
            k += 1
    buf, off, ln = batch(fl)
    sb = types.SimpleNamespace(frames=buf, offset=off, length=ln, n=len(off), frames_bytes=len(buf) - 64)
    _check_frag_batch(gpu_ctx, sb, 1200, inplace, False)


@pytest.mark.parametrize("seed,buckets,entries", [(11, 4, 4), (12, 8, 2), (13, 16, 4), (14, 1, 8)])
def test_reassembly_contention_exact(gpu_ctx, seed, buckets, entries):
    """Tables far too small for the batch: flows compete for the last free and expired entries
    of their buckets, find no space, reclaim stale entries, and every outcome (including which
    flow reclaims which expired entry, i.e. the "expired" count) equals the oracle's arrival-order
    processing."""
    tot = _check_scenario(gpu_ctx, scenario(seed, n_batches=5, flows_per_batch=90, dt=12),
                          dict(bucket_num=buckets, bucket_entries=entries, max_cycles=20))
    for k in ("no_space", "expired", "done", "stored"):
        assert tot[k] > 0, (k, tot)


@pytest.mark.parametrize("max_entries", [0, 0xFFFF])
def test_reassembly_in_order_is_parallel(gpu_ctx, max_entries):
    """Datagrams whose fragments arrive back to back (frames.frag_batch, the bench's workload) never
    meet another flow in the table: no fragment takes the serial path, also under the reference's
    max_entries = NUM_FLOWS_MAX (the bound on the entries a grouped batch holds stays far below)."""
    from udpdk_amd import frames as FR
    b = FR.frag_batch(4096, 2952)
    abi.frag_table_create(gpu_ctx, 0x1000, 16, 1 << 40, 65515, max_entries=max_entries)
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, b.n, 1, b.n)
    assert abi.rx_run(gpu_ctx, db, out)[4] == 0
    rb, _, st = abi.rx_reassemble(gpu_ctx, db, out.meta, 0)
    assert st["done"] == 4096 and st["serial"] == 0 and st["sorted"] == 0, st


def test_no_space_and_table_reuse(gpu_ctx):
    """Two-slot table: a third live flow finds no space; expired flows free their slots."""
    from reasm_util import split, udp_datagram, raw_ip
    abi.frag_table_create(gpu_ctx, bucket_num=1, bucket_entries=2, max_cycles=100, max_dgram=256)
    t = O.FragTable(bucket_num=1, bucket_entries=2, max_cycles=100, max_dgram=256)
    src, dst = raw_ip("10.0.0.1"), raw_ip("172.31.100.1")
    d = udp_datagram(1, 2, b"c" * 24)
    fa, fb, fc = (split(src, dst, pid, d, [16, 16]) for pid in (10, 11, 12))
    big = split(src, dst, 13, udp_datagram(1, 2, b"d" * 300), [160, 148])   # past max_dgram
    steps = [([fa[0], fb[0]], 0), ([fc[0]], 50), ([fa[1]], 101), ([fc[0], fc[1]], 102), (big, 103)]
    for frames, tms in steps:
        buf, off, ln = batch(frames)
        db = abi.rx_upload(gpu_ctx, buf, off, ln)
        db.frames_bytes = len(buf) - 64
        meta = O.rx(O.BindTable(), buf, len(buf) - 64, off, ln, None, 1)[0]
        mb = gpu_ctx.upload(meta)
        rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, mb, tms)
        _, woo, _, _, wst = t.reassemble(buf, off, ln, meta, tms)
        gst.pop("serial")
        gst.pop("sorted")
        assert gst == wst and rb.n == len(woo), (tms, gst, wst)
        for bb in (db.frames, db.offset, db.length, mb):
            bb.free()


def test_tx_fragments_come_back(gpu_ctx):
    """GPU loop: tx_build_mtu (udpdk_sendto + the poller's fragmentation) -> rx -> reassembly ->
    rx on the datagrams: every datagram is delivered with the payload that was sent."""
    rng = np.random.default_rng(9)
    mtu, n = 1500, 300
    # every datagram length, including those whose last fragment carries 1-7 bytes: a 35-41 B
    # frame (unpadded, as built), which the RX verdict still sends to reassembly
    lens = [1480 * m + k - 8 for m in (1, 2, 3) for k in range(1, 8)]
    lens += rng.integers(1473, 5900, n - len(lens)).tolist()
    pays = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    port = abi.raw_port(10001)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({port: [(0, 0, 0)]}, 1,
                                                    slots=[(0, abi.raw_port(10000), 1)]))
    abi.frag_table_create(gpu_ctx, bucket_num=64, bucket_entries=16, max_cycles=1000)
    po = np.cumsum([0] + lens[:-1]).astype(np.uint32)
    pay = np.zeros(int(po[-1]) + lens[-1] + 64, np.uint8)
    for o, p in zip(po, pays):
        pay[o:o + len(p)] = np.frombuffer(p, np.uint8)
    spans = [int(abi.lib().udpdk_gpu_tx_span(L, mtu, None)) for L in lens]
    fo = np.cumsum([0] + spans[:-1]).astype(np.uint32)
    cap = int(fo[-1]) + spans[-1] + 64
    bufs = [gpu_ctx.upload(pay), gpu_ctx.upload(po), gpu_ctx.upload(np.array(lens, np.uint16)),
            gpu_ctx.upload(np.zeros(n, np.int32)),
            gpu_ctx.upload(np.full(n, abi.raw_ip("172.31.100.1"), np.uint32)),
            gpu_ctx.upload(np.full(n, port, np.uint16)), gpu_ctx.upload(fo)]
    frames = gpu_ctx.alloc(cap)
    cfg = abi.TxConfig((C.c_uint8 * 6)(*bytes.fromhex("6805ca95f8ec")),
                       (C.c_uint8 * 6)(*bytes.fromhex("6805ca95fa64")), abi.raw_ip("172.31.100.2"))
    tb = abi.TxBatch(bufs[0].ptr, len(pay), bufs[1].ptr, bufs[2].ptr, bufs[3].ptr, bufs[4].ptr,
                     bufs[5].ptr, n)
    assert abi.lib().udpdk_gpu_tx_build_mtu(gpu_ctx.handle, C.byref(cfg), C.byref(tb),
                                            C.byref(abi.TxOut(frames.ptr, cap, bufs[6].ptr)), mtu) == 0
    # the fragment frames as an RX batch, in send order (every datagram has id 0, as sent)
    off, ln = [], []
    for L, f0 in zip(lens, fo):
        nf = -(-(L + 8) // (mtu - 20))
        for k in range(nf):
            off.append(int(f0) + k * (mtu + 14))
            ln.append(mtu + 14 if k + 1 < nf else 34 + (L + 8) - (nf - 1) * (mtu - 20))
    off, ln = np.array(off, np.uint32), np.array(ln, np.uint16)
    db = abi.RxDeviceBatch(frames, cap - 64, gpu_ctx.upload(off), gpu_ctx.upload(ln), None, len(off))
    out = abi.rx_alloc_out(gpu_ctx, len(off), 1, len(off))
    m1 = abi.rx_run(gpu_ctx, db, out)[0]
    assert np.all(abi.meta_verdict(m1) == abi.V_FRAG)
    rb, origin, st = abi.rx_reassemble(gpu_ctx, db, out.meta, 0)
    assert st["done"] == n and st["errors"] == st["holes"] == st["stored"] == st["serial"] == 0
    out2 = abi.rx_alloc_out(gpu_ctx, n, 1, n)
    m2, loff, lp, cnt, rc = abi.rx_run(gpu_ctx, rb, out2)
    assert rc == 0 and np.all(abi.meta_verdict(m2) == 0) and np.array_equal(lp, np.arange(n))
    g = abi.rx_alloc_gather(gpu_ctx, n, 6016)
    gp, glen, gip, gport = abi.rx_gather_run(gpu_ctx, rb, out2.lane_pkt, 0, g)
    for k in range(n):
        assert glen[k] == lens[k] and gp[k, :lens[k]].tobytes() == pays[k], k
    assert np.all(gport == abi.raw_port(10000)) and np.all(gip == abi.raw_ip("172.31.100.2"))


def test_reassembly_edges(gpu_ctx):
    """Bad table geometry -> EINVAL; an empty batch and a batch without fragments give no
    datagrams."""
    import ctypes as C
    from reasm_util import udp_datagram, ip_frame, raw_ip
    bad = abi.FragTableCfg(0, 16, 100, 65515)
    assert abi.lib().udpdk_gpu_frag_table_create(gpu_ctx.handle, C.byref(bad)) == -22
    bad = abi.FragTableCfg(16, 3, 100, 65515)                 # bucket_entries not a power of two
    assert abi.lib().udpdk_gpu_frag_table_create(gpu_ctx.handle, C.byref(bad)) == -22
    bad = abi.FragTableCfg(16, 16, 100, 70000)                # max_dgram past IPv4
    assert abi.lib().udpdk_gpu_frag_table_create(gpu_ctx.handle, C.byref(bad)) == -22
    bad = abi.FragTableCfg(16, 16, 100, 4096, 257)            # max_entries past the 256 entries
    assert abi.lib().udpdk_gpu_frag_table_create(gpu_ctx.handle, C.byref(bad)) == -22
    bad = abi.FragTableCfg(16, 16, 100, 4096, 0, 2)           # unknown flag
    assert abi.lib().udpdk_gpu_frag_table_create(gpu_ctx.handle, C.byref(bad)) == -22
    abi.frag_table_create(gpu_ctx, 16, 16, 100, 4096)
    frames = [ip_frame(raw_ip("10.0.0.1"), raw_ip("172.31.100.1"), 1, 0, udp_datagram(1, 2, b"x" * 40), False)]
    buf, off, ln = batch(frames)
    db = abi.rx_upload(gpu_ctx, buf, off, ln)
    db.frames_bytes = len(buf) - 64
    meta = gpu_ctx.upload(O.rx(O.BindTable(), buf, len(buf) - 64, off, ln, None, 1)[0])
    rb, _, st = abi.rx_reassemble(gpu_ctx, db, meta, 0)
    assert rb.n == 0 and st["frags"] == 0
    db.n = 0
    rb, _, st = abi.rx_reassemble(gpu_ctx, db, meta, 0)
    assert rb.n == 0 and sum(st.values()) == 0


@pytest.mark.parametrize("seed,buckets,entries,max_entries,grouped",
                         [(31, 256, 16, 24, False), (32, 64, 4, 40, True), (33, 16, 4, 60, False),
                          (35, 256, 16, 8, True), (34, 256, 16, 4095, True)])
def test_reassembly_max_entries_exact(gpu_ctx, seed, buckets, entries, max_entries, grouped):
    """rte_ip_frag_table_create's max_entries (NUM_FLOWS_MAX, udpdk_poller.c:130-131): at the limit
    ip_frag_find deletes the LRU entry when it has expired and otherwise drops the fragment. Limits
    far below the table size over multi-batch scenarios with expiry: every datagram, origin and
    count equals the oracle's; a limit the batches cannot reach keeps the parallel path."""
    tot = _check_scenario(gpu_ctx, scenario(seed, n_batches=6, flows_per_batch=90, dt=12, grouped=grouped),
                          dict(bucket_num=buckets, bucket_entries=entries, max_cycles=20,
                               max_entries=max_entries))
    assert tot["done"] > 0, tot
    if max_entries < 100:
        assert tot["no_space"] > 0 and tot["expired"] > 0, tot
    else:
        assert tot["serial"] < tot["frags"], tot


def test_reassembly_lru_rule_exact(gpu_ctx):
    """The oracle's hand-derived max_entries sequence (tests/test_reasm_oracle.py) on the GPU: a
    fourth flow finds no space while the oldest entry is alive, takes a slot once it has expired
    (the LRU deletion, not a stale slot of its own buckets), and later flows see the count."""
    from reasm_util import split, udp_datagram, raw_ip
    src, dst = raw_ip("172.31.100.2"), raw_ip("172.31.100.1")

    def bk(pid):
        mask = (64 * 4 - 1) & ~3
        s1, s2 = O.frag_hash(src, dst, pid)
        return {(s1 & mask) // 4, (s2 & mask) // 4}
    used = bk(21) | bk(22) | bk(23)
    d = next(p for p in range(100, 10000) if not (bk(p) & used))
    geo = dict(bucket_num=64, bucket_entries=4, max_cycles=10, max_dgram=256, max_entries=3)
    abi.frag_table_create(gpu_ctx, **geo)
    t = O.FragTable(**geo)
    dg = udp_datagram(1, 2, b"q" * 24)
    fa, fb, fc, fd = (split(src, dst, p, dg, [16, 16]) for p in (21, 22, 23, d))
    steps = [([fa[0]], 0), ([fb[0], fc[0]], 5), ([fd[0]], 9), ([fd[0]], 11), ([fb[1], fa[1]], 12), ([fd[1]], 13)]
    want_ns = [0, 0, 1, 0, 0, 0]
    for (frames, tms), ns in zip(steps, want_ns):
        buf, off, ln = batch(frames)
        db = abi.rx_upload(gpu_ctx, buf, off, ln)
        db.frames_bytes = len(buf) - 64
        meta = O.rx(O.BindTable(), buf, len(buf) - 64, off, ln, None, 1)[0]
        mb = gpu_ctx.upload(meta)
        rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, mb, tms)
        _, woo, _, _, wst = t.reassemble(buf, off, ln, meta, tms)
        gst.pop("serial")
        gst.pop("sorted")
        assert gst == wst and rb.n == len(woo), (tms, gst, wst)
        assert gst["no_space"] == ns, (tms, gst)
        for bb in (db.frames, db.offset, db.length, mb):
            bb.free()


@pytest.mark.parametrize("inplace", [False, True])
def test_reassembly_dpdk_checksum(gpu_ctx, inplace):
    """UDPDK_FRAG_CKSUM_DPDK ([gpu] reasm_cksum = dpdk): the reassembled header's checksum is 0 as
    DPDK's ipv4_frag_reassemble leaves it (udpdk_poller.c:355-360), through the copying and the
    in-place emit; the datagrams equal the oracle's in the same mode, and their demux reports the
    IPv4 checksum bad (verdict bit 4 clear) as the reference's bytes would give."""
    from udpdk_amd import frames as FR
    b = FR.frag_batch(500, 2952)
    abi.frag_table_create(gpu_ctx, 0x1000, 16, 1 << 40, 65515, flags=abi.FRAG_CKSUM_DPDK)
    t = O.FragTable(0x1000, 16, 1 << 40, 65515, flags=1)
    gpu_ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(FR.PORT_RECV): [(0, 0, 0)]}, 4))
    db = abi.rx_upload(gpu_ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(gpu_ctx, b.n, 4, 4 * b.n)
    gm = abi.rx_run(gpu_ctx, db, out)[0]
    rb, origin, gst = abi.rx_reassemble(gpu_ctx, db, out.meta, 0, inplace=inplace)
    wout, woo, wol, wog, wst = t.reassemble(b.frames, b.offset, b.length, gm, 0)
    gst.pop("serial"), gst.pop("sorted")
    assert gst == wst and gst["done"] == 500, (gst, wst)
    assert (rb.frames.ptr == db.frames.ptr) == inplace
    gbuf, goff, gln = _frames(gpu_ctx, rb)
    for k in range(rb.n):
        g = gbuf[goff[k]:goff[k] + gln[k]].tobytes()
        assert g == wout[woo[k]:woo[k] + wol[k]].tobytes(), k
        assert g[24:26] == b"\0\0"
    out2 = abi.rx_alloc_out(gpu_ctx, rb.n, 4, 4 * rb.n)
    g2 = abi.rx_run(gpu_ctx, rb, out2)
    assert g2[4] == 0 and np.all(abi.meta_verdict(g2[0]) == 0)
    assert not np.any(g2[0] & (1 << 4))                   # IPv4 checksum not ok
    for x in (db.frames, db.offset, db.length, out.meta, out.lane_off, out.lane_pkt, out2.meta,
              out2.lane_off, out2.lane_pkt):
        x.free()
