"""The golden fixtures straight through the HIP path, no oracle in between (-m gpu): the RX
behaviour the survey recorded by running the reference's reassemble() (tests/golden/
rx_probes.json: the ptype-vs-ethertype gate, DF-only vs MF/offset fragments, NOT_UDP, ANY-first
list order, reuse fan-out sequence, NO_MATCH, NO_BIND, and the (uint8_t) slot aliasing counts at
300 / 1024 sockets) and the published checksum examples (tests/golden/checksum_vectors.json) as
frames. Bindings are made by the product's host bind table (udpdk_bind / setsockopt through
udpdk_api.h), flattened by udpdk_btable_snapshot, uploaded, and the frames run through
udpdk_gpu_rx; the assertions are the fixtures' expected values."""
import json
import os
import socket
import struct

import numpy as np
import pytest

from udpdk_amd import abi, frames as F

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(HERE, name)) as f:
        return json.load(f)


def _run(ctx, frames, ptype=None, n_lanes=16, lists=None, lane_mask=0xFFFFFFFF):
    out = bytearray()
    offs = []
    for f in frames:
        offs.append(len(out))
        out += f
    buf = np.zeros(len(out) + 256, np.uint8)
    buf[:len(out)] = np.frombuffer(bytes(out), np.uint8)
    ctx.upload_snapshot(abi.snapshot_from_lists(lists or {}, n_lanes, lane_mask))
    b = abi.rx_upload(ctx, buf, np.array(offs, np.uint32), np.array([len(f) for f in frames], np.uint16),
                      None if ptype is None else np.asarray(ptype, np.uint32))
    b.frames_bytes = len(out)
    o = abi.rx_alloc_out(ctx, len(frames), n_lanes, 8 * len(frames))
    meta, loff, pkt, cnt, rc = abi.rx_run(ctx, b, o)
    assert rc == 0
    for x in (b.frames, b.offset, b.length, o.meta, o.lane_off, o.lane_pkt) + ((b.ptype,) if b.ptype else ()):
        x.free()
    return meta, loff, pkt, cnt


def _bind_lists(api, binds, port=10001):
    """The product's bind table after the probe's binds (sockfd, ip, so_options), in order."""
    api.reset()
    top = max((s for s, _, _ in binds), default=-1)
    for _ in range(top + 1):
        assert api.socket() >= 0
    for s, ip, opts in binds:
        if opts & abi.SO_REUSEPORT == abi.SO_REUSEPORT:
            assert api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEPORT, 1) == 0
        elif opts & abi.SO_REUSEADDR:
            assert api.setsockopt(s, abi.SOL_SOCKET, abi.SO_REUSEADDR, 1) == 0
        assert api.bind(s, ip, port) == 0
    return api.port_lists()


def test_rx_probes_on_the_gpu(gpu_ctx, host_api):
    rng = np.random.default_rng(0)
    for p in _load("rx_probes.json")["frames"]:
        kw = dict(dport=10001, dst_ip=p.get("dst_ip", "172.31.100.1"), payload_len=22)
        for k in ("ethertype", "frag", "proto"):
            if k in p:
                kw[k] = p[k]
        f = F.make_frame(rng, **kw)
        lists = _bind_lists(host_api, p["binds"]) if "binds" in p else \
            _bind_lists(host_api, [(0, "0.0.0.0", 0)])
        pt = [p["ptype"]] if "ptype" in p else None
        meta, loff, pkt, cnt = _run(gpu_ctx, [f], pt, 16, lists)
        assert abi.VERDICT_NAMES[int(abi.meta_verdict(meta[0]))] == p["expect_verdict"], p["id"]
        if "expect_deliveries" in p:
            got = [lane for lane in range(16) for _ in range(loff[lane + 1] - loff[lane])]
            assert got == sorted(p["expect_deliveries"]), p["id"]
            assert int(cnt[abi.C_DELIVERIES]) == len(p["expect_deliveries"]), p["id"]
            if p["expect_deliveries"]:
                assert int(abi.meta_sockfd(meta[0])) == p["expect_deliveries"][0], p["id"]
                assert int(abi.meta_fanout(meta[0])) == len(p["expect_deliveries"]), p["id"]


@pytest.mark.parametrize("probe", _load("rx_probes.json")["alias"])
def test_uint8_slot_aliasing_on_the_gpu(gpu_ctx, probe):
    """n sockets bound ANY to 10000 + i, one frame to each: the reference's (uint8_t) slot index
    aliases every sockfd >= 256 (44 of 300, 768 of 1024 recorded); compat lanes (lane_mask 0xFF)
    hold what the reference's exch_slots[(uint8_t)sockfd] would."""
    n = probe["n_sockets"]
    rng = np.random.default_rng(1)
    frames = [F.make_frame(rng, dport=10000 + i) for i in range(n)]
    lists = {abi.raw_port(10000 + i): [(0, i, 0)] for i in range(n)}
    meta, loff, pkt, _ = _run(gpu_ctx, frames, None, 256, lists, 0xFF)
    socks = abi.meta_sockfd(meta)
    assert int(np.sum(socks >= 256)) == probe["aliased"]
    for k in range(256):
        assert pkt[loff[k]:loff[k + 1]].tolist() == [i for i in range(n) if i & 0xFF == k]


def _ip_frame(hdr20: bytes, udp: bytes) -> bytes:
    return bytes.fromhex("6805ca95fa646805ca95f8ec0800") + hdr20 + udp


def test_checksum_vectors_as_frames(gpu_ctx):
    """checksum_vectors.json on the GPU: the published IPv4 header (checksum b861) passes the RX
    IPv4 check (verdict bit 4) and fails with one bit flipped; the RFC 1071 example bytes as a
    UDP payload whose checksum field is set from the fixture's own sum (sum_be) pass the RX UDP
    check (bits 5-6 = OK) and fail with a payload byte changed."""
    vec = {v["id"]: v for v in _load("checksum_vectors.json")}
    ip = vec["ipv4-b861"]
    hdr = bytearray(bytes.fromhex(ip["bytes"]))
    hdr[10:12] = struct.pack(">H", ip["cksum_be"])
    # the header says total length 0x73 = 115: a UDP datagram of 95 bytes behind it
    bad = bytearray(hdr)
    bad[15] ^= 0x01
    pl = bytes(87)
    udp0 = struct.pack(">HHHH", 4000, 10001, 8 + len(pl), 0) + pl        # UDP checksum absent
    meta, _, _, _ = _run(gpu_ctx, [_ip_frame(bytes(hdr), udp0), _ip_frame(bytes(bad), udp0)], None, 1,
                         {abi.raw_port(10001): [(0, 0, 0)]})
    assert (int(meta[0]) >> 4) & 1 == 1 and (int(meta[1]) >> 4) & 1 == 0

    r = vec["rfc1071-s3"]
    payload = bytes.fromhex(r["bytes"])
    src, dst = socket.inet_aton("172.31.100.2"), socket.inet_aton("172.31.100.1")
    ulen = 8 + len(payload)
    h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + ulen, 1, 0, 64, 17, 0, src, dst))
    s = sum(struct.unpack(">10H", bytes(h)))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    h[10:12] = struct.pack(">H", (~s) & 0xFFFF)
    # one's-complement sum: pseudo header + UDP header (checksum 0) + the fixture's payload sum
    words = sum(struct.unpack(">4H", src + dst)) + 17 + ulen + 4000 + 10001 + ulen + r["sum_be"]
    while words >> 16:
        words = (words & 0xFFFF) + (words >> 16)
    ck = (~words) & 0xFFFF or 0xFFFF
    good = struct.pack(">HHHH", 4000, 10001, ulen, ck) + payload
    corrupt = bytearray(good)
    corrupt[8] ^= 0x40
    meta, _, _, cnt = _run(gpu_ctx, [_ip_frame(bytes(h), good), _ip_frame(bytes(h), bytes(corrupt))], None, 1,
                           {abi.raw_port(10001): [(0, 0, 0)]})
    assert abi.meta_udp(meta).tolist() == [abi.UDP_OK, abi.UDP_BAD]
    assert abi.meta_verdict(meta).tolist() == [abi.V_DELIVERED, abi.V_DELIVERED]   # flags only
