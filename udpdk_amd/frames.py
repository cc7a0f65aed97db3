"""Synthetic Eth/IPv4/UDP frame batches.

* :func:`build_frames` — the benchmark recipe of SURVEY.md §8(d): frames packed back to back,
  dst MAC 68:05:ca:95:f8:ec, src MAC 68:05:ca:95:fa:64, IPv4 172.31.100.2 -> 172.31.100.1
  (apps/pktgen/main.c:27), TTL 64, seeded id, UDP src 10000, valid non-zero UDP checksum,
  seeded payload. Vectorised numpy, sized for 1 M-4 M frames.
* :func:`config_batch` — BASELINE.json configs 2-5.
* :func:`mixed_batch` — small batches that hit every verdict and checksum class, odd offsets,
  padding and length errors, for parity tests.
"""
from __future__ import annotations

import socket
import struct
from dataclasses import dataclass, field

import numpy as np

ETH_DST = bytes.fromhex("6805ca95f8ec")   # receiver port0 (config.ini:9-10)
ETH_SRC = bytes.fromhex("6805ca95fa64")   # sender ([port0_dst], config.ini:13-14)
IP_SRC = "172.31.100.2"
IP_DST = "172.31.100.1"
UDP_SRC = 10000
PORT_RECV = 10001                          # apps/pktgen/main.c:26


@dataclass
class Batch:
    frames: np.ndarray          # uint8, padded to a multiple of 256 bytes
    offset: np.ndarray          # uint32 [n]
    length: np.ndarray          # uint16 [n]
    frames_bytes: int           # bytes covered by frames (before padding)
    ptype: np.ndarray | None = None
    meta: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(len(self.offset))


def _fold(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    for _ in range(4):
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _random_bytes(rng: np.random.Generator, nbytes: int) -> np.ndarray:
    words = (nbytes + 7) // 8
    w = rng.integers(0, np.iinfo(np.uint64).max, size=words, dtype=np.uint64, endpoint=True)
    return w.view(np.uint8)[:nbytes]


def _headers(sizes: np.ndarray, dports: np.ndarray, ident: np.ndarray) -> np.ndarray:
    n = len(sizes)
    h = np.zeros((n, 42), np.uint8)
    h[:, 0:6] = np.frombuffer(ETH_DST, np.uint8)
    h[:, 6:12] = np.frombuffer(ETH_SRC, np.uint8)
    h[:, 12] = 0x08
    tl = (sizes.astype(np.uint32) - 14)
    h[:, 14] = 0x45
    h[:, 16] = tl >> 8
    h[:, 17] = tl & 0xFF
    h[:, 18] = ident >> 8
    h[:, 19] = ident & 0xFF
    h[:, 22] = 64
    h[:, 23] = 17
    h[:, 26:30] = np.frombuffer(socket.inet_aton(IP_SRC), np.uint8)
    h[:, 30:34] = np.frombuffer(socket.inet_aton(IP_DST), np.uint8)
    h[:, 34] = UDP_SRC >> 8
    h[:, 35] = UDP_SRC & 0xFF
    dp = dports.astype(np.uint32)
    h[:, 36] = dp >> 8
    h[:, 37] = dp & 0xFF
    ul = sizes.astype(np.uint32) - 34
    h[:, 38] = ul >> 8
    h[:, 39] = ul & 0xFF
    w = h[:, 14:34:2].astype(np.uint64) + h[:, 15:34:2].astype(np.uint64) * 256
    c = (~_fold(w.sum(1))) & 0xFFFF
    h[:, 24] = c & 0xFF
    h[:, 25] = c >> 8
    return h


def _udp_cksum(h: np.ndarray, pay: np.ndarray) -> np.ndarray:
    """pay: [k, m] payload bytes at frame-relative offset 42 (even)."""
    s = pay[:, 0::2].astype(np.uint64).sum(1) + pay[:, 1::2].astype(np.uint64).sum(1) * 256
    s += (h[:, 34:42:2].astype(np.uint64) + h[:, 35:42:2].astype(np.uint64) * 256).sum(1)
    s += (h[:, 26:34:2].astype(np.uint64) + h[:, 27:34:2].astype(np.uint64) * 256).sum(1)
    s += 0x1100 + h[:, 38].astype(np.uint64) + h[:, 39].astype(np.uint64) * 256
    c = (~_fold(s)) & 0xFFFF
    c[c == 0] = 0xFFFF
    return c


def build_frames(sizes: np.ndarray, dports_host: np.ndarray, seed: int, chunk: int = 8192) -> Batch:
    """Back-to-back frames of the given sizes (>= 42) with valid IPv4 and UDP checksums."""
    sizes = np.asarray(sizes, np.uint32)
    n = len(sizes)
    off = np.zeros(n, np.uint64)
    if n > 1:
        off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    total = int(off[-1] + sizes[-1]) if n else 0
    padded = (total + 255) // 256 * 256 + 256
    rng = np.random.default_rng(seed)
    flat = np.zeros(padded, np.uint8)
    flat[:total] = _random_bytes(rng, total)
    ident = rng.integers(0, 65536, n, dtype=np.uint32)
    dports_host = np.asarray(dports_host, np.uint32)
    uniform = n > 0 and bool(np.all(sizes == sizes[0]))
    if uniform:
        L = int(sizes[0])
        view = flat[:total].reshape(n, L)
        for a in range(0, n, chunk * 8):
            b = min(n, a + chunk * 8)
            h = _headers(sizes[a:b], dports_host[a:b], ident[a:b])
            cs = _udp_cksum(h, view[a:b, 42:])
            h[:, 40] = cs & 0xFF
            h[:, 41] = cs >> 8
            view[a:b, :42] = h
    else:
        for L in np.unique(sizes):
            idx_all = np.nonzero(sizes == L)[0]
            cols = np.arange(int(L), dtype=np.uint64)
            for a in range(0, len(idx_all), chunk):
                idx = idx_all[a:a + chunk]
                pos = off[idx][:, None] + cols[None, :]
                rows = flat[pos]
                h = _headers(sizes[idx], dports_host[idx], ident[idx])
                cs = _udp_cksum(h, rows[:, 42:])
                h[:, 40] = cs & 0xFF
                h[:, 41] = cs >> 8
                flat[pos[:, :42]] = h
    return Batch(flat, off.astype(np.uint32), sizes.astype(np.uint16), total)


# ---- BASELINE.json configs ------------------------------------------------------------------------
IMIX_SIZES = np.array([64, 594, 1500], np.uint32)
IMIX_WEIGHTS = np.array([7, 4, 1], np.float64)


def zipf_ports(rng: np.random.Generator, n: int, n_ports: int, s: float = 0.99) -> np.ndarray:
    r = np.arange(1, n_ports + 1, dtype=np.float64)
    p = r ** -s
    p /= p.sum()
    return rng.choice(n_ports, size=n, p=p).astype(np.uint32)


@dataclass
class Workload:
    name: str
    batch: Batch
    n_sockets: int                 # sockets 0..n_sockets-1 bound ANY to 10000 + i (config 1: 10001)
    base_port: int

    def port_lists(self):
        from .abi import raw_port
        return {raw_port(self.base_port + i): [(0, i, 0)] for i in range(self.n_sockets)}


def _nlabel(n: int) -> str:
    return f"{n >> 20}M" if n % (1 << 20) == 0 else str(n)


def config_batch(cfg: int, n: int | None = None, shard: int = 0) -> Workload:
    """BASELINE.json configs[cfg] (1-based as in BASELINE.md: 1 = CPU pktgen case). The workload
    name carries the frame count (profiles/traffic.json is keyed by it)."""
    if cfg == 1:   # apps/pktgen -s 64: 64 B payload -> 106 B frames, one socket ANY:10001
        n = n or (1 << 20)
        b = build_frames(np.full(n, 106, np.uint32), np.full(n, PORT_RECV, np.uint32), 0x5EED ^ shard)
        return Workload("pktgen-64B-payload-1port", b, 1, PORT_RECV)
    if cfg == 2:
        n = n or (1 << 20)
        b = build_frames(np.full(n, 64, np.uint32), np.full(n, PORT_RECV, np.uint32), 0x5EED ^ shard)
        return Workload(f"{_nlabel(n)}-64B-1port", b, 1, PORT_RECV)
    if cfg == 3:
        n = n or (1 << 20)
        b = build_frames(np.full(n, 1500, np.uint32), np.full(n, PORT_RECV, np.uint32), 0x5EED ^ shard)
        return Workload(f"{_nlabel(n)}-1500B-1port", b, 1, PORT_RECV)
    if cfg == 4:
        n = n or (1 << 20)
        rng = np.random.default_rng(4 + shard)
        sizes = IMIX_SIZES[rng.choice(3, size=n, p=IMIX_WEIGHTS / IMIX_WEIGHTS.sum())]
        ports = 10000 + rng.integers(0, 1024, n, dtype=np.uint32)
        b = build_frames(sizes, ports, 0x5EED ^ shard)
        return Workload("IMIX-1024ports-uniform" + ("" if n == 1 << 20 else f"-{_nlabel(n)}"), b, 1024, 10000)
    if cfg == 5:
        n = n or (1 << 22)
        rng = np.random.default_rng(1000 + shard)
        ports = 10000 + zipf_ports(rng, n, 4096)
        b = build_frames(np.full(n, 64, np.uint32), ports, 0x5EED ^ shard)
        return Workload(f"{_nlabel(n)}-64B-4096ports-zipf0.99", b, 4096, 10000)
    raise ValueError(cfg)


# ---- mixed edge-case batches for parity tests --------------------------------------------------
def _csum16(b: bytes) -> int:
    if len(b) % 2:
        b = b + b"\0"
    s = sum(struct.unpack(f"<{len(b) // 2}H", b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def make_frame(rng: np.random.Generator, *, dport: int, dst_ip: str = IP_DST, src_ip: str = IP_SRC,
               payload_len: int = 22, ethertype: int = 0x0800, ihl: int = 5, frag: int = 0,
               proto: int = 17, udp_len: int | None = None, udp_cksum: str = "ok",
               ip_cksum: str = "ok", pad: int = 0, total_len: int | None = None) -> bytes:
    payload = rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()
    ul = 8 + payload_len if udp_len is None else udp_len
    ident = int(rng.integers(0, 65536))
    tl = 20 + 8 + payload_len if total_len is None else total_len
    ip = bytearray(struct.pack(">BBHHHBBH4s4s", (4 << 4) | ihl, 0, tl, ident, frag, 64, proto, 0,
                               socket.inet_aton(src_ip), socket.inet_aton(dst_ip)))
    c = (~_csum16(bytes(ip))) & 0xFFFF
    if ip_cksum == "bad":
        c ^= 0x0101
    ip[10:12] = struct.pack("<H", c)
    udp = bytearray(struct.pack(">HHHH", UDP_SRC, dport, ul & 0xFFFF, 0))
    if udp_cksum in ("ok", "bad"):
        seg = bytes(udp) + payload
        pseudo = ip[12:20] + struct.pack(">BBH", 0, 17, ul & 0xFFFF)
        cs = (~_csum16(bytes(pseudo) + seg[:max(0, ul)])) & 0xFFFF
        if cs == 0:
            cs = 0xFFFF
        if udp_cksum == "bad":
            cs = cs ^ 0x8001 or 0x1234
        udp[6:8] = struct.pack("<H", cs)
    eth = ETH_DST + ETH_SRC + struct.pack(">H", ethertype)
    return eth + bytes(ip) + bytes(udp) + payload + bytes(pad)


def mixed_batch(seed: int, n: int, bound_ports: list[int], unbound_ports: list[int],
                dst_ips: list[str], align_jitter: bool = True, with_ptype: bool = False) -> Batch:
    """n frames drawn over every verdict/checksum class; gaps of 0-3 bytes give odd offsets."""
    rng = np.random.default_rng(seed)
    kinds = ["ok", "ok", "ok", "ok", "nobind", "udp_zero", "udp_bad", "ip_bad", "mf", "fragoff",
             "df", "tcp", "ipv6", "arp", "trunc", "ihl6", "pad", "lenbig", "lensmall", "big",
             "tiny_ok"]
    out = bytearray()
    offs, lens, pts, kk = [], [], [], []
    for _ in range(n):
        k = kinds[int(rng.integers(0, len(kinds)))]
        port = int(rng.choice(bound_ports)) if k != "nobind" else int(rng.choice(unbound_ports))
        dip = str(rng.choice(dst_ips))
        pl = int(rng.integers(0, 200))
        kw = dict(dport=port, dst_ip=dip, payload_len=pl)
        if k == "udp_zero":
            kw["udp_cksum"] = "zero"
        elif k == "udp_bad":
            kw["udp_cksum"] = "bad"
        elif k == "ip_bad":
            kw["ip_cksum"] = "bad"
        elif k == "mf":
            kw["frag"] = 0x2000
        elif k == "fragoff":
            kw["frag"] = int(rng.integers(1, 0x1FFF))
        elif k == "df":
            kw["frag"] = 0x4000
        elif k == "tcp":
            kw["proto"] = 6
        elif k == "ipv6":
            kw["ethertype"] = 0x86DD
        elif k == "arp":
            kw["ethertype"] = 0x0806
        elif k == "ihl6":
            kw["ihl"] = 6
        elif k == "pad":
            kw["payload_len"] = int(rng.integers(0, 18))
            kw["pad"] = int(rng.integers(1, 30))
        elif k == "lenbig":
            kw["udp_len"] = 8 + pl + int(rng.integers(1, 50))
        elif k == "lensmall":
            kw["udp_len"] = int(rng.integers(0, 8))
        elif k == "big":
            kw["payload_len"] = int(rng.integers(1000, 1473))
        elif k == "tiny_ok":
            kw["payload_len"] = int(rng.integers(0, 4))
        f = make_frame(rng, **kw)
        if k == "trunc":
            f = f[:int(rng.integers(0, 42))]
        if align_jitter:
            out += bytes(int(rng.integers(0, 4)))
        offs.append(len(out))
        lens.append(len(f))
        out += f
        kk.append(k)
        # NIC-reported packet_type: mostly consistent; some deliberate mismatches (ptype rules)
        if with_ptype:
            et = struct.unpack(">H", f[12:14])[0] if len(f) >= 14 else 0
            pt = 0x211 if et == 0x0800 else 0x1
            r = rng.random()
            if r < 0.05:
                pt = 0x211 if pt == 0x1 else 0x1    # disagree with ether_type
            elif r < 0.10:
                pt = 0x91                            # L3_IPV4_EXT_UNKNOWN still has bit 0x10
            pts.append(pt)
    total = len(out)
    flat = np.zeros((total + 255) // 256 * 256 + 256, np.uint8)
    flat[:total] = np.frombuffer(bytes(out), np.uint8)
    return Batch(flat, np.array(offs, np.uint32), np.array(lens, np.uint16), total,
                 np.array(pts, np.uint32) if with_ptype else None, {"kinds": kk})


# ---- fragment workloads (f2) --------------------------------------------------------------------
def frag_batch(n_dgrams: int, payload_len: int, mtu: int = 1500, seed: int = 0x5EED) -> Batch:
    """n_dgrams UDP datagrams of payload_len bytes (valid UDP checksums), each cut the way the
    poller's rte_ipv4_fragment_packet cuts it at `mtu` (mtu - 20 data bytes per fragment), the
    fragments of a datagram back to back and in order. Datagram k has IPv4 id k & 0xffff and
    source 172.31.(100 + (k >> 16)).2, so every datagram is its own flow."""
    L = payload_len
    fpl = mtu - 20
    ipl = L + 8
    nf = -(-ipl // fpl)
    src = build_frames(np.full(n_dgrams, L + 42, np.uint32), np.full(n_dgrams, PORT_RECV, np.uint32), seed)
    whole = src.frames[:src.frames_bytes].reshape(n_dgrams, L + 42)
    k = np.arange(n_dgrams, dtype=np.uint32)
    sizes = [34 + min(fpl, ipl - j * fpl) for j in range(nf)]
    per = sum(sizes)
    total = n_dgrams * per
    flat = np.zeros((total + 255) // 256 * 256 + 256, np.uint8)
    view = flat[:total].reshape(n_dgrams, per)
    pos = 0
    for j, fs in enumerate(sizes):
        h = whole[:, :34].copy()
        tl = fs - 14
        h[:, 16] = tl >> 8
        h[:, 17] = tl & 0xFF
        h[:, 18] = k & 0xFF                                  # id raw LE = k & 0xffff
        h[:, 19] = (k >> 8) & 0xFF
        ff = (j * fpl) // 8 | (0x2000 if j + 1 < nf else 0)
        h[:, 20] = ff >> 8
        h[:, 21] = ff & 0xFF
        h[:, 28] = 100 + (k >> 16)                           # source 172.31.(100 + k >> 16).2
        h[:, 24] = 0
        h[:, 25] = 0
        w = h[:, 14:34:2].astype(np.uint64) + h[:, 15:34:2].astype(np.uint64) * 256
        c = (~_fold(w.sum(1))) & 0xFFFF
        h[:, 24] = c & 0xFF
        h[:, 25] = c >> 8
        view[:, pos:pos + 34] = h
        view[:, pos + 34:pos + fs] = whole[:, 34 + j * fpl:34 + j * fpl + fs - 34]
        pos += fs
    # the UDP checksum covers the pseudo header's source address (+ (k >> 16) in the LE word of
    # bytes 28-29): fold the change into the checksum in the first fragment (bytes 40-41)
    hi = (k >> 16).astype(np.uint64)
    if np.any(hi):
        c = view[:, 40].astype(np.uint64) | (view[:, 41].astype(np.uint64) << 8)
        c2 = (~_fold((~c & 0xFFFF) + hi)) & 0xFFFF
        c2[c2 == 0] = 0xFFFF
        view[:, 40] = (c2 & 0xFF).astype(np.uint8)
        view[:, 41] = (c2 >> 8).astype(np.uint8)
    off = (np.arange(n_dgrams, dtype=np.uint64)[:, None] * per +
           np.cumsum([0] + sizes[:-1])[None, :]).reshape(-1).astype(np.uint32)
    ln = np.tile(np.array(sizes, np.uint16), n_dgrams)
    return Batch(flat, off, ln, total)
