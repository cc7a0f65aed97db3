"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see udpdk_oracle.h). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg load this module; the product library
never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.oracle_btable_new.restype = P
        L.oracle_btable_free.argtypes = [P]
        L.oracle_btable_add.argtypes = [P, C.c_int, C.c_uint32, C.c_uint32, C.c_int]
        L.oracle_btable_del.argtypes = [P, C.c_int, C.c_uint32]
        L.oracle_btable_free_port.argtypes = [P]
        L.oracle_btable_port_len.argtypes = [P, C.c_uint32]
        L.oracle_btable_port_at.argtypes = [P, C.c_uint32, C.c_int, C.POINTER(C.c_int),
                                            C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
        L.oracle_rx.restype = C.c_int64
        L.oracle_rx.argtypes = [P, P, C.c_uint64, P, P, P, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_int, P, P, P, C.c_uint32, P]
        L.oracle_rx_parallel.restype = C.c_double
        L.oracle_rx_parallel.argtypes = [P, P, C.c_uint64, P, P, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_int, C.c_int, C.c_int]
        L.oracle_rte_ipv4_cksum.restype = C.c_uint16
        L.oracle_rte_ipv4_cksum.argtypes = [P]
        L.oracle_tx_frame.argtypes = [P, P, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                                      C.c_uint32, C.c_uint32, P, C.c_uint32, P]
        L.oracle_tx_fragment.restype = C.c_uint32
        L.oracle_tx_fragment.argtypes = [P, C.c_uint32, C.c_uint32, P]
        L.oracle_ftable_new.restype = P
        L.oracle_ftable_new.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.oracle_ftable_free.argtypes = [P]
        L.oracle_frag_hash.restype = C.c_uint32
        L.oracle_frag_hash.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
        L.oracle_reassemble.restype = C.c_int64
        L.oracle_reassemble.argtypes = [P, P, C.c_uint64, P, P, P, C.c_uint32, C.c_uint64, P,
                                        C.c_uint64, P, P, P, C.c_uint32, P]
        L.oracle_toeplitz.restype = C.c_uint32
        L.oracle_toeplitz.argtypes = [P, P, C.c_uint32]
        L.oracle_rss.restype = C.c_int
        L.oracle_rss.argtypes = [P, C.c_uint32, P, C.c_uint32, C.c_uint32, P, C.c_uint64, P, P, P,
                                 C.c_uint32, P, P, P]
        L.oracle_recv_gather.argtypes = [P, P, P, P, C.c_uint32, C.c_uint32, C.c_uint32, P, P, P, P]
        _lib = L
    return _lib


class BindTable:
    """sock_bind_table restated (udpdk_bind_table.c)."""

    def __init__(self):
        self.h = C.c_void_p(lib().oracle_btable_new())

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_btable_free(self.h)
            self.h = None

    def add(self, sockfd: int, ip_raw: int, port_raw: int, opts: int) -> int:
        return lib().oracle_btable_add(self.h, sockfd, ip_raw, port_raw, opts)

    def delete(self, sockfd: int, port_raw: int):
        lib().oracle_btable_del(self.h, sockfd, port_raw)

    def free_port(self) -> int:
        return lib().oracle_btable_free_port(self.h)

    def port_list(self, port_raw: int) -> list[tuple[int, int, int]]:
        out = []
        n = lib().oracle_btable_port_len(self.h, port_raw)
        s, ip, r = C.c_int(), C.c_uint32(), C.c_int()
        for i in range(n):
            lib().oracle_btable_port_at(self.h, port_raw, i, C.byref(s), C.byref(ip), C.byref(r))
            out.append((ip.value, s.value, r.value))
        return out


def rx(bt: BindTable, frames: np.ndarray, frames_bytes: int, offset: np.ndarray, length: np.ndarray,
       ptype: np.ndarray | None, n_lanes: int, lane_mask: int = 0xFFFFFFFF, do_csum: bool = True,
       lane_cap: int | None = None):
    """Returns (meta, lane_off, lane_pkt, counters)."""
    n = len(offset)
    offset = np.ascontiguousarray(offset, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    meta = np.zeros(max(1, n), np.uint32)
    loff = np.zeros(n_lanes + 1, np.uint32)
    cap = lane_cap if lane_cap is not None else max(1, n * 8)
    pkt = np.zeros(cap, np.uint32)
    cnt = np.zeros(16, np.uint64)
    pt = np.ascontiguousarray(ptype, np.uint32) if ptype is not None else None
    d = lib().oracle_rx(bt.h, frames.ctypes.data, frames_bytes, offset.ctypes.data,
                        length.ctypes.data, pt.ctypes.data if pt is not None else None, n,
                        lane_mask, n_lanes, int(do_csum), meta.ctypes.data, loff.ctypes.data,
                        pkt.ctypes.data, cap, cnt.ctypes.data)
    if d < 0:
        raise RuntimeError("oracle_rx failed (lane capacity or key out of range)")
    return meta[:n], loff, pkt[:d], cnt


def rx_parallel(bt: BindTable, frames: np.ndarray, frames_bytes: int, offset: np.ndarray,
                length: np.ndarray, n_lanes: int, do_csum: bool, threads: int, reps: int) -> float:
    offset = np.ascontiguousarray(offset, np.uint32)
    length = np.ascontiguousarray(length, np.uint16)
    return lib().oracle_rx_parallel(bt.h, frames.ctypes.data, frames_bytes, offset.ctypes.data,
                                     length.ctypes.data, len(offset), 0xFFFFFFFF, n_lanes,
                                     int(do_csum), threads, reps)


def ipv4_cksum(hdr20: bytes) -> int:
    b = C.create_string_buffer(hdr20, 20)
    return lib().oracle_rte_ipv4_cksum(b)


def tx_frame(src_mac: bytes, dst_mac: bytes, cfg_src_ip: int, slot_bound: int, slot_ip: int,
             slot_port: int, dst_ip: int, dst_port: int, payload: bytes) -> bytes:
    out = C.create_string_buffer(len(payload) + 42)
    pb = C.create_string_buffer(payload, max(1, len(payload)))
    lib().oracle_tx_frame(C.create_string_buffer(src_mac, 6), C.create_string_buffer(dst_mac, 6),
                          cfg_src_ip, slot_bound, slot_ip, slot_port, dst_ip, dst_port, pb,
                          len(payload), out)
    return out.raw


def tx_fragment(frame: bytes, mtu: int) -> list[bytes]:
    """The poller's fragmentation of one sendto frame (udpdk_poller.c:461-501): the frames."""
    n_max = max(1, (len(frame) + mtu) // max(1, mtu - 20) + 2) if mtu else 1
    out = C.create_string_buffer(len(frame) + 34 * n_max + 16)
    n = lib().oracle_tx_fragment(C.create_string_buffer(frame, len(frame)), len(frame), mtu, out)
    raw, frames, pos = out.raw, [], 0
    for _ in range(n):
        flen = 14 + ((raw[pos + 16] << 8) | raw[pos + 17])     # IPv4 total length + Ethernet
        frames.append(raw[pos:pos + flen])
        pos += flen
    return frames


def bindtable_from_lists(port_lists: dict[int, list[tuple[int, int, int]]]) -> BindTable:
    """Replay bindings so that each port's list ends up in the given order. ANY bindings are
    lpush'ed, specific ones rpush'ed, so replaying ANY entries in reverse list order first and the
    specific ones in list order reproduces any list whose ANY entries precede the specific ones."""
    bt = BindTable()
    for p, lst in port_lists.items():
        anys = [x for x in lst if x[0] == 0]
        specs = [x for x in lst if x[0] != 0]
        assert lst == anys + specs, "list order not reachable through bind()"
        for ip, s, reuse in reversed(anys):
            assert bt.add(s, ip, p, 15 if reuse else 0) == 0
        for ip, s, reuse in specs:
            assert bt.add(s, ip, p, 15 if reuse else 0) == 0
    return bt


def recv_gather(frames: np.ndarray, offset: np.ndarray, length: np.ndarray, lane_pkt: np.ndarray,
                first: int, count: int, slot: int):
    """recvfrom payload delivery (udpdk_syscall.c:401-488) for lane entries [first, first+count):
    (payload [count, slot] u8, len u32, src_ip u32 raw, src_port u16 raw)."""
    fr = np.ascontiguousarray(frames, np.uint8)
    off = np.ascontiguousarray(offset, np.uint32)
    ln = np.ascontiguousarray(length, np.uint16)
    lp = np.ascontiguousarray(lane_pkt, np.uint32)
    pay = np.zeros((max(1, count), slot), np.uint8)
    olen = np.zeros(max(1, count), np.uint32)
    sip = np.zeros(max(1, count), np.uint32)
    spt = np.zeros(max(1, count), np.uint16)
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    lib().oracle_recv_gather(P(fr), P(off), P(ln), P(lp), first, count, slot, P(pay), P(olen),
                             P(sip), P(spt))
    return pay[:count], olen[:count], sip[:count], spt[:count]


RS_STATS = ("frags", "drop_len", "drop_short", "no_space", "errors", "holes", "expired", "done",
            "stored")


class FragTable:
    """The poller's reassembly table (udpdk_poller.c:130 rte_ip_frag_table_create) restated:
    state persists across reassemble() calls like the reference's."""

    def __init__(self, bucket_num=0x1000, bucket_entries=16, max_cycles=1000, max_dgram=65515,
                 max_entries=0, flags=0):
        self.h = C.c_void_p(lib().oracle_ftable_new(bucket_num, bucket_entries, max_cycles, max_dgram,
                                                    max_entries, flags))
        if not self.h:
            raise ValueError("bad table geometry")
        self.fed = 0          # bytes fed so far: bounds what held fragments can add to an output

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_ftable_free(self.h)
            self.h = None

    def reassemble(self, frames: np.ndarray, offset, length, meta, tms: int):
        """FRAG frames of one batch -> (frames u8, offset u32, length u16, origin u32, stats)."""
        fr = np.ascontiguousarray(frames, np.uint8)
        off = np.ascontiguousarray(offset, np.uint32)
        ln = np.ascontiguousarray(length, np.uint16)
        mt = np.ascontiguousarray(meta, np.uint32)
        n = len(off)
        self.fed += int(ln.astype(np.int64).sum())
        cap = self.fed + 64 * n + 64
        out = np.zeros(cap, np.uint8)
        oo = np.zeros(max(1, n), np.uint32)
        ol = np.zeros(max(1, n), np.uint16)
        og = np.zeros(max(1, n), np.uint32)
        st = np.zeros(len(RS_STATS), np.uint64)
        P = lambda a: a.ctypes.data_as(C.c_void_p)
        k = lib().oracle_reassemble(self.h, P(fr), len(fr), P(off), P(ln), P(mt), n, tms, P(out),
                                    cap, P(oo), P(ol), P(og), max(1, n), P(st))
        if k < 0:
            raise RuntimeError("oracle_reassemble: output capacity")
        return out, oo[:k], ol[:k], og[:k], dict(zip(RS_STATS, st.tolist()))


def frag_hash(src: int, dst: int, pid: int):
    s2 = C.c_uint32()
    s1 = lib().oracle_frag_hash(src, dst, pid, C.byref(s2))
    return s1, s2.value


def toeplitz(key: bytes, data: bytes) -> int:
    return lib().oracle_toeplitz(C.create_string_buffer(key, 40), C.create_string_buffer(data, len(data)),
                                 len(data))


def rss(key: bytes, hash_types: int, reta, n_queues: int, frames: np.ndarray, frames_bytes: int,
        offset, length, ptype=None):
    """-> (hash u32[n], queue_off u32[Q+1], queue_pkt u32[n])."""
    off = np.ascontiguousarray(offset, np.uint32)
    ln = np.ascontiguousarray(length, np.uint16)
    rt = np.ascontiguousarray(reta, np.uint16)
    n = len(off)
    h = np.zeros(max(1, n), np.uint32)
    qo = np.zeros(n_queues + 1, np.uint32)
    qp = np.zeros(max(1, n), np.uint32)
    pt = np.ascontiguousarray(ptype, np.uint32) if ptype is not None else None
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = lib().oracle_rss(C.create_string_buffer(key, 40), hash_types, P(rt), len(rt), n_queues,
                          P(np.ascontiguousarray(frames, np.uint8)), frames_bytes, P(off), P(ln),
                          P(pt) if pt is not None else None, n, P(h), P(qo), P(qp))
    if rc:
        raise ValueError("oracle_rss")
    return h[:n], qo, qp[:n]
