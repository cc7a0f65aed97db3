"""Shared helpers for the reassembly tests: fragment frames and batches."""
import numpy as np

import oracle as O
from udpdk_amd import abi

SRC_MAC = bytes.fromhex("6805ca95f8ec")
DST_MAC = bytes.fromhex("6805ca95fa64")


def ip_frame(src, dst, pid, ofs, data, mf, df=False, proto=17):
    """Eth/IPv4 frame carrying `data` as the IP payload at fragment offset `ofs` (bytes)."""
    tl = 20 + len(data)
    ff = (ofs // 8) | (0x2000 if mf else 0) | (0x4000 if df else 0)
    h = bytearray(b"\x45\x00" + tl.to_bytes(2, "big") + pid.to_bytes(2, "little") + ff.to_bytes(2, "big")
                  + bytes([64, proto, 0, 0]) + src.to_bytes(4, "little") + dst.to_bytes(4, "little"))
    s = sum(h[i] | (h[i + 1] << 8) for i in range(0, 20, 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    h[10:12] = ((~s) & 0xFFFF).to_bytes(2, "little")
    return DST_MAC + SRC_MAC + b"\x08\x00" + bytes(h) + bytes(data)


def udp_datagram(sport, dport, payload):
    """UDP header + payload (checksum 0)."""
    return sport.to_bytes(2, "little") + dport.to_bytes(2, "little") + \
        (len(payload) + 8).to_bytes(2, "big") + b"\0\0" + bytes(payload)


def split(src, dst, pid, ip_payload, sizes):
    """Fragments of ip_payload cut at the given data sizes (multiples of 8 except the last)."""
    out, pos = [], 0
    for k, sz in enumerate(sizes):
        out.append(ip_frame(src, dst, pid, pos, ip_payload[pos:pos + sz], k + 1 < len(sizes)))
        pos += sz
    assert pos == len(ip_payload)
    return out


def wire(f):
    """The frame as a NIC delivers it: Ethernet frames shorter than 60 B (no FCS) are padded
    (a 1-byte last fragment from the TX fragmentation is 35 B before the NIC)."""
    return f if len(f) >= 60 else f + bytes(60 - len(f))


def batch(frames, align=1, pad=True):
    """Pack frames back to back: (buffer u8 with tailroom, offset u32, length u16). pad=False keeps
    short frames as they are (a 1-7 byte last fragment is a 35-41 B frame)."""
    frames = [wire(f) if pad else f for f in frames]
    off, pos = [], 0
    for f in frames:
        off.append(pos)
        pos += (len(f) + align - 1) // align * align
    buf = np.zeros(pos + 64, np.uint8)
    for o, f in zip(off, frames):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return buf, np.array(off, np.uint32), np.array([len(f) for f in frames], np.uint16)


def verdicts(buf, off, ln):
    """The oracle's RX verdict words (no bindings: fragments FRAG, the rest NO_BIND etc.)."""
    bt = O.BindTable()
    meta, _, _, _ = O.rx(bt, buf, len(buf) - 64, off, ln, None, 1)
    return meta


def frames_of(out, oo, ol):
    return [out[o:o + l].tobytes() for o, l in zip(oo, ol)]


def raw_ip(s):
    return abi.raw_ip(s)


def scenario(seed, n_batches=6, flows_per_batch=120, normal_per_batch=200, ports=(10000, 10001, 10002, 10003),
             dt=10, grouped=False):
    """Seeded multi-batch fragment workload: [(frames list, tms)]. Datagrams are cut into 2..4
    fragments (some into 5: too many), fragments arrive shuffled within a window that spans
    batch boundaries; some are lost (their flows expire later), duplicated (first/last
    duplicates error a flow) or overlapping; keys are sometimes reused after completion;
    unfragmented UDP frames to the same ports are interleaved. grouped: each datagram's
    fragments arrive back to back (in order, duplicates after them) and keys are not reused, so
    every key is one run of the batch's fragments (batch boundaries still cut flows)."""
    rng = np.random.default_rng(seed)
    src_pool = [raw_ip(f"10.0.{k}.{j}") for k in range(4) for j in range(1, 5)]
    dst = raw_ip("172.31.100.1")
    events = []                                   # (time position, frame)
    pos = 0.0
    used_keys = []
    for b in range(n_batches):
        for k in range(flows_per_batch):
            src = int(rng.choice(src_pool))
            if used_keys and rng.random() < 0.05 and not grouped:
                src, pid = used_keys[int(rng.integers(len(used_keys)))]
            else:
                pid = int(rng.integers(0, 65536))
            used_keys.append((src, pid))
            port = int(rng.choice(ports))
            L = int(rng.integers(1, 4000))
            d = udp_datagram(0x1027, int.from_bytes(port.to_bytes(2, "big"), "little"),
                             rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            n = len(d)
            nf = int(rng.choice([2, 3, 4, 5], p=[0.45, 0.3, 0.2, 0.05]))
            nf = max(2, min(nf, n // 8))
            cuts = sorted(rng.choice(np.arange(1, (n - 1) // 8 + 1), nf - 1, replace=False) * 8) if n > 16 else [8]
            sizes = np.diff([0] + list(cuts) + [n]).tolist()
            frs = split(src, dst, pid, d, sizes)
            r = rng.random()
            if r > 0.96 and n >= 40:                      # hole: a middle piece sent twice,
                m = 8 * max(1, (n // 4) // 8)             # its equal-sized neighbour never
                frs = split(src, dst, pid, d, [m, m, m, n - 3 * m])
                frs = [frs[0], frs[1], frs[1], frs[3]]
            elif r < 0.06:
                frs = frs[1:]                             # lost first fragment
            elif r < 0.10:
                frs = frs + [frs[0]]                      # duplicate first
            elif r < 0.13:
                frs = frs + [frs[-1]]                     # duplicate last
            elif r < 0.16 and len(sizes) >= 2:            # overlapping rewrite of fragment 0
                frs = frs + [ip_frame(src, dst, pid, 0, d[:sizes[0] + 8], True)]
            t0 = pos + rng.random() * 0.6
            for j, f in enumerate(frs):
                events.append((pos + 1e-6 * j if grouped else t0 + rng.random() * 1.4, f))
            pos += 1.0 / flows_per_batch
        for k in range(normal_per_batch):
            port = int(rng.choice(ports))
            d = udp_datagram(0x1027, int.from_bytes(port.to_bytes(2, "big"), "little"),
                             rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes())
            tn = b + rng.random()
            if grouped:                                   # between two datagrams' fragments
                tn = int(tn * flows_per_batch) / flows_per_batch + 0.5 / flows_per_batch
            events.append((tn, ip_frame(int(rng.choice(src_pool)), dst, 0, 0, d, False)))
    events.sort(key=lambda e: e[0])
    out = []
    for b in range(n_batches + 2):
        fs = [f for t, f in events if b <= t < b + 1]
        if fs:
            out.append((fs, 1000 + b * dt))
    return out
