"""ctypes bindings to libudpdk_amd.so (the C ABI of include/udpdk_gpu.h and include/udpdk_api.h).

Used by tests/ and bench.py. Everything that computes goes through the shared library; numpy
arrays are only host staging for the C-ABI calls.
"""
from __future__ import annotations

import ctypes as C
import errno
import os
import socket
import struct
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UDPDK_LIB_OVERRIDE") or os.path.join(_HERE, "libudpdk_amd.so")

# ---- constants mirrored from include/udpdk_gpu.h -------------------------------------------
V_DELIVERED, V_NOT_IPV4, V_FRAG, V_NOT_UDP, V_NO_BIND, V_NO_MATCH, V_TRUNC, V_BAD_DESC = range(8)
VERDICT_NAMES = ["DELIVERED", "NOT_IPV4", "FRAG", "NOT_UDP", "NO_BIND", "NO_MATCH", "TRUNC",
                 "BAD_DESC"]
UDP_NONE, UDP_OK, UDP_BAD = 0, 1, 2
N_COUNTERS = 16
N_KERNEL_IDS = 5          # udpdk_gpu_kernel_id: classify, scan, scatter, tx_build, rx_gather
C_DELIVERIES, C_IP_BAD, C_UDP_OK, C_UDP_BAD, C_UDP_NONE, C_LEN_BAD, C_IHL_NE5, C_BYTES = range(8, 16)
K_RX_CLASSIFY, K_RX_SCAN, K_RX_SCATTER, K_TX_BUILD = range(4)
MAX_LANES = 16384


def meta_verdict(m):
    return np.asarray(m) & 0xF


def meta_sockfd(m):
    return np.asarray(m) >> 16


def meta_fanout(m):
    return (np.asarray(m) >> 9) & 0x7F


def meta_udp(m):
    return (np.asarray(m) >> 5) & 3


class Binding(C.Structure):
    _fields_ = [("ip", C.c_uint32), ("sockfd", C.c_int32), ("reuse", C.c_uint32)]


class Slot(C.Structure):
    _fields_ = [("ip", C.c_uint32), ("udp_port", C.c_uint32), ("bound", C.c_uint32)]


class BindSnapshot(C.Structure):
    _fields_ = [("port_first", C.POINTER(C.c_uint32)), ("port_count", C.POINTER(C.c_uint16)),
                ("binds", C.POINTER(Binding)), ("n_binds", C.c_uint32),
                ("n_lanes", C.c_uint32), ("lane_mask", C.c_uint32),
                ("slots", C.POINTER(Slot)), ("n_slots", C.c_uint32),
                ("version", C.c_uint64)]


class RxBatch(C.Structure):
    _fields_ = [("frames_dev", C.c_void_p), ("frames_bytes", C.c_uint64),
                ("offset_dev", C.c_void_p), ("length_dev", C.c_void_p),
                ("ptype_dev", C.c_void_p), ("n", C.c_uint32)]


class RxOut(C.Structure):
    _fields_ = [("meta_dev", C.c_void_p), ("lane_off_dev", C.c_void_p),
                ("lane_pkt_dev", C.c_void_p), ("lane_cap", C.c_uint32)]


class RxStats(C.Structure):
    _fields_ = [("counters", C.c_uint64 * N_COUNTERS), ("deliveries", C.c_uint32),
                ("overflow", C.c_uint32)]


class RxGather(C.Structure):
    _fields_ = [("payload_dev", C.c_void_p), ("slot_bytes", C.c_uint32), ("len_dev", C.c_void_p),
                ("src_ip_dev", C.c_void_p), ("src_port_dev", C.c_void_p)]


RS_N = 11                 # udpdk_rs_stat
RS_STATS = ("frags", "drop_len", "drop_short", "no_space", "errors", "holes", "expired", "done",
            "stored", "serial", "sorted")


class FragTableCfg(C.Structure):
    _fields_ = [("bucket_num", C.c_uint32), ("bucket_entries", C.c_uint32),
                ("max_cycles", C.c_uint64), ("max_dgram", C.c_uint32), ("max_entries", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32)]


FRAG_CKSUM_DPDK = 1       # UDPDK_FRAG_CKSUM_DPDK


class ReasmOut(C.Structure):
    _fields_ = [("batch", RxBatch), ("origin_dev", C.c_void_p), ("stats", C.c_uint64 * RS_N)]


class RssConf(C.Structure):
    _fields_ = [("key", C.c_uint8 * 40), ("hash_types", C.c_uint32), ("n_queues", C.c_uint32),
                ("reta_size", C.c_uint32), ("reta", C.c_uint16 * 512)]


class RssOut(C.Structure):
    _fields_ = [("hash_dev", C.c_void_p), ("queue_off_dev", C.c_void_p), ("queue_pkt_dev", C.c_void_p)]


class TxConfig(C.Structure):
    _fields_ = [("src_mac", C.c_uint8 * 6), ("dst_mac", C.c_uint8 * 6), ("src_ip", C.c_uint32)]


class TxBatch(C.Structure):
    _fields_ = [("payload_dev", C.c_void_p), ("payload_bytes", C.c_uint64),
                ("payload_off_dev", C.c_void_p), ("payload_len_dev", C.c_void_p),
                ("sockfd_dev", C.c_void_p), ("dst_ip_dev", C.c_void_p),
                ("dst_port_dev", C.c_void_p), ("n", C.c_uint32)]


RX_BURST_FN = C.CFUNCTYPE(C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                          C.c_uint32)
TX_BURST_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32)


class PortOps(C.Structure):
    """udpdk_port_ops_t (udpdk_api.h): a port for the poller thread."""
    _fields_ = [("rx_burst", RX_BURST_FN), ("tx_burst", TX_BURST_FN), ("user", C.c_void_p),
                ("batch_frames", C.c_uint32)]


class TxOut(C.Structure):
    _fields_ = [("frames_dev", C.c_void_p), ("frames_bytes", C.c_uint64),
                ("frame_off_dev", C.c_void_p)]


# name -> (restype, argtypes); every symbol the headers declare
_P = C.c_void_p
_PROTOS = {
    # udpdk_gpu.h
    "udpdk_gpu_abi_version": (C.c_int, []),
    "udpdk_gpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "udpdk_gpu_ctx_create": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.POINTER(_P)]),
    "udpdk_gpu_ctx_destroy": (C.c_int, [_P]),
    "udpdk_gpu_sync": (C.c_int, [_P]),
    "udpdk_gpu_last_hip_error": (C.c_int, [_P]),
    "udpdk_gpu_stream": (_P, [_P]),
    "udpdk_gpu_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "udpdk_gpu_free": (C.c_int, [_P, _P]),
    "udpdk_gpu_host_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "udpdk_gpu_host_free": (C.c_int, [_P, _P]),
    "udpdk_gpu_memset": (C.c_int, [_P, _P, C.c_int, C.c_size_t]),
    "udpdk_gpu_h2d": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "udpdk_gpu_d2h": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "udpdk_gpu_bind_snapshot_upload": (C.c_int, [_P, C.POINTER(BindSnapshot)]),
    "udpdk_gpu_rx": (C.c_int, [_P, C.POINTER(RxBatch), C.POINTER(RxOut)]),
    "udpdk_gpu_rx_stats": (C.c_int, [_P, C.POINTER(RxStats)]),
    "udpdk_gpu_pipeline_depth": (C.c_int, [_P, C.c_int]),
    "udpdk_gpu_join": (C.c_int, [_P]),
    "udpdk_gpu_rx_host": (C.c_int, [_P, _P, C.c_uint64, _P, _P, _P, C.c_uint32, _P, _P, _P,
                                    C.c_uint32, C.POINTER(RxStats)]),
    "udpdk_gpu_rx_host_async": (C.c_int, [_P, _P, C.c_uint64, _P, _P, _P, C.c_uint32, _P, _P, _P,
                                          C.c_uint32, C.POINTER(RxStats)]),
    "udpdk_gpu_rx_host_wait": (C.c_int, [_P]),
    "udpdk_gpu_rx_host_batch": (C.c_int, [_P, C.POINTER(RxBatch), C.POINTER(_P)]),
    # poller internals (udpdk_poll_rx's pipelined form)
    "udpdk_gpu_pipe_rx_host": (C.c_int, [_P, C.c_int, _P, C.c_uint64, _P, C.c_uint32, _P, _P, C.c_uint32,
                                         _P, _P, _P, C.c_uint32, C.POINTER(RxStats)]),
    "udpdk_gpu_pipe_wait": (C.c_int, [_P, C.c_int]),
    "udpdk_gpu_pipe_batch": (C.c_int, [_P, C.c_int, C.POINTER(RxBatch), C.POINTER(_P)]),
    "udpdk_gpu_pipe_h2d": (C.c_int, [_P, C.c_int, _P, _P, C.c_size_t]),
    "udpdk_gpu_pipe_d2h": (C.c_int, [_P, C.c_int, _P, _P, C.c_size_t]),
    "udpdk_gpu_pipe_gather_packed": (C.c_int, [_P, C.c_int, C.POINTER(RxBatch), _P, C.c_uint32, C.c_uint32,
                                               _P, C.POINTER(RxGather)]),
    "udpdk_gpu_rx_gather": (C.c_int, [_P, C.POINTER(RxBatch), _P, C.c_uint32, C.c_uint32,
                                      C.POINTER(RxGather)]),
    "udpdk_gpu_rx_gather_packed": (C.c_int, [_P, C.POINTER(RxBatch), _P, C.c_uint32, C.c_uint32, _P,
                                             C.POINTER(RxGather)]),
    "udpdk_gpu_frag_table_create": (C.c_int, [_P, C.POINTER(FragTableCfg)]),
    "udpdk_gpu_rx_reassemble": (C.c_int, [_P, C.POINTER(RxBatch), _P, C.c_uint64, C.POINTER(ReasmOut)]),
    "udpdk_gpu_rx_reassemble_inplace": (C.c_int, [_P, C.POINTER(RxBatch), _P, C.c_uint64, C.POINTER(ReasmOut)]),
    "udpdk_gpu_rss_default_conf": (C.c_int, [C.POINTER(RssConf), C.c_uint32]),
    "udpdk_gpu_rss_config": (C.c_int, [_P, C.POINTER(RssConf)]),
    "udpdk_gpu_rss": (C.c_int, [_P, C.POINTER(RxBatch), C.POINTER(RssOut)]),
    "udpdk_gpu_tx_build": (C.c_int, [_P, C.POINTER(TxConfig), C.POINTER(TxBatch), C.POINTER(TxOut)]),
    "udpdk_gpu_tx_build_mtu": (C.c_int, [_P, C.POINTER(TxConfig), C.POINTER(TxBatch),
                                         C.POINTER(TxOut), C.c_uint32]),
    "udpdk_gpu_tx_span": (C.c_uint64, [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "udpdk_gpu_timing_enable": (C.c_int, [_P, C.c_int]),
    "udpdk_gpu_timing_read": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
    "udpdk_gpu_rx_geometry": (C.c_int, [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]),
    # udpdk_api.h
    "udpdk_init": (C.c_int, [C.c_int, C.POINTER(C.c_char_p)]),
    "udpdk_interrupt": (None, [C.c_int]),
    "udpdk_cleanup": (None, []),
    "udpdk_socket": (C.c_int, [C.c_int, C.c_int, C.c_int]),
    "udpdk_getsockopt": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.POINTER(C.c_uint32)]),
    "udpdk_setsockopt": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, C.c_uint32]),
    "udpdk_bind": (C.c_int, [C.c_int, _P, C.c_uint32]),
    "udpdk_sendto": (C.c_ssize_t, [C.c_int, _P, C.c_size_t, C.c_int, _P, C.c_uint32]),
    "udpdk_recvfrom": (C.c_ssize_t, [C.c_int, _P, C.c_size_t, C.c_int, _P, C.POINTER(C.c_uint32)]),
    "udpdk_close": (C.c_int, [C.c_int]),
    "udpdk_dump_payload": (None, [C.c_char_p, C.c_int]),
    "udpdk_poll_rx": (C.c_int, [_P, C.c_uint64, _P, _P, _P, C.c_uint32, C.POINTER(RxStats)]),
    "udpdk_tx_drain": (C.c_int, [_P, C.c_uint64, _P, _P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "udpdk_btable_snapshot": (C.c_int, [C.POINTER(BindSnapshot), C.c_int]),
    "udpdk_gpu_context": (_P, []),
    "udpdk_shard_devices": (C.c_int, [_P, C.c_int]),
    "udpdk_shard_plan": (C.c_int, [C.c_char_p, _P, C.c_int]),
    "udpdk_shard_frames": (C.c_int, [_P, C.c_int]),
    "udpdk_config_set": (C.c_int, [_P, _P, C.c_uint32]),
    "udpdk_config_get": (C.c_int, [_P, _P, C.POINTER(C.c_uint32)]),
    "udpdk_config_mtu": (C.c_int, [C.c_uint32]),
    "udpdk_tx_pending": (C.c_uint64, []),
    "udpdk_tx_dropped": (C.c_uint64, []),
    "udpdk_rx_nobufs": (C.c_uint64, []),
    "udpdk_port_attach": (C.c_int, [C.POINTER(PortOps)]),
    "udpdk_port_detach": (C.c_int, []),
    "udpdk_port_loopback": (C.c_int, [C.POINTER(PortOps)]),
    "udpdk_slot_table": (C.c_int, [C.POINTER(Slot), C.c_uint32]),
    "udpdk_host_reset": (None, []),
}

_lib = None


def lib() -> C.CDLL:
    """Load libudpdk_amd.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _PROTOS.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                # an A/B build of an older tree (tools/ab.py) may predate a newer entry point
                if os.environ.get("UDPDK_LIB_OVERRIDE"):
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def declared_symbols() -> list[str]:
    return sorted(_PROTOS)


class UdpdkError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc != 0:
        raise UdpdkError(f"{what} failed: rc={rc} ({errno.errorcode.get(-rc, '?')})")


def device_count() -> int:
    n = C.c_int(0)
    lib().udpdk_gpu_device_count(C.byref(n))
    return n.value


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---- snapshot construction from Python binding lists -------------------------------------------
@dataclass
class HostSnapshot:
    """Arrays behind a BindSnapshot (kept alive with the struct)."""
    port_first: np.ndarray
    port_count: np.ndarray
    binds: C.Array
    slots: C.Array | None
    snap: BindSnapshot


def snapshot_from_lists(port_lists: dict[int, list[tuple[int, int, int]]], n_lanes: int,
                        lane_mask: int = 0xFFFFFFFF, slots: list[tuple[int, int, int]] | None = None
                        ) -> HostSnapshot:
    """port_lists: raw port -> [(ip_raw, sockfd, reuse)] in list (head -> tail) order."""
    first = np.zeros(65536, np.uint32)
    count = np.zeros(65536, np.uint16)
    flat = []
    for p in sorted(port_lists):
        lst = port_lists[p]
        if not lst:
            continue
        first[p] = len(flat)
        count[p] = len(lst)
        flat.extend(lst)
    arr = (Binding * max(1, len(flat)))()
    for i, (ip, sock, reuse) in enumerate(flat):
        arr[i].ip, arr[i].sockfd, arr[i].reuse = ip, sock, reuse
    sl = None
    if slots:
        sl = (Slot * len(slots))()
        for i, (ip, port, bound) in enumerate(slots):
            sl[i].ip, sl[i].udp_port, sl[i].bound = ip, port, bound
    snap = BindSnapshot(first.ctypes.data_as(C.POINTER(C.c_uint32)),
                        count.ctypes.data_as(C.POINTER(C.c_uint16)),
                        C.cast(arr, C.POINTER(Binding)), len(flat), n_lanes, lane_mask,
                        C.cast(sl, C.POINTER(Slot)) if sl is not None else None,
                        len(slots) if slots else 0, 1)
    return HostSnapshot(first, count, arr, sl, snap)


# ---- device context ------------------------------------------------------------------------------
class DeviceBuffer:
    def __init__(self, ctx: "GpuContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _check(lib().udpdk_gpu_alloc(ctx.handle, max(1, self.nbytes), C.byref(p)), "udpdk_gpu_alloc")
        self.ptr = p.value

    def free(self):
        if self.ptr:
            lib().udpdk_gpu_free(self.ctx.handle, C.c_void_p(self.ptr))
            self.ptr = None


class GpuContext:
    """A udpdk_gpu_ctx on one device."""

    def __init__(self, device: int = 0, max_frames: int = 1 << 20, max_lanes: int = 4096):
        h = C.c_void_p()
        _check(lib().udpdk_gpu_ctx_create(device, max_frames, max_lanes, C.byref(h)),
               "udpdk_gpu_ctx_create")
        self.handle = h
        self.device = device
        self._bufs: list[DeviceBuffer] = []

    def close(self):
        for b in self._bufs:
            b.free()
        self._bufs.clear()
        if self.handle:
            lib().udpdk_gpu_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def alloc(self, nbytes: int) -> DeviceBuffer:
        b = DeviceBuffer(self, nbytes)
        self._bufs.append(b)
        return b

    def upload(self, a: np.ndarray) -> DeviceBuffer:
        a = np.ascontiguousarray(a)
        b = self.alloc(a.nbytes)
        if a.nbytes:
            _check(lib().udpdk_gpu_h2d(self.handle, C.c_void_p(b.ptr), C.c_void_p(_ptr(a)), a.nbytes), "h2d")
            self.sync()
        return b

    def download(self, b: DeviceBuffer, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype)
        if out.nbytes:
            _check(lib().udpdk_gpu_d2h(self.handle, C.c_void_p(_ptr(out)), C.c_void_p(b.ptr), out.nbytes), "d2h")
            self.sync()
        return out

    def sync(self):
        _check(lib().udpdk_gpu_sync(self.handle), "udpdk_gpu_sync")

    def pipeline(self, depth: int):
        """1: every udpdk_gpu_rx in order on one stream; 2: consecutive calls alternate between
        two streams (independent batches with distinct outputs overlap)."""
        _check(lib().udpdk_gpu_pipeline_depth(self.handle, int(depth)), "udpdk_gpu_pipeline_depth")

    def join(self):
        _check(lib().udpdk_gpu_join(self.handle), "udpdk_gpu_join")

    def upload_snapshot(self, hs: HostSnapshot):
        _check(lib().udpdk_gpu_bind_snapshot_upload(self.handle, C.byref(hs.snap)),
               "udpdk_gpu_bind_snapshot_upload")

    def timing(self, every: int):
        """0 = off, N = record kernel events on every Nth udpdk_gpu_rx call."""
        _check(lib().udpdk_gpu_timing_enable(self.handle, int(every)), "timing_enable")

    def timing_read(self):
        ms = (C.c_double * N_KERNEL_IDS)()
        n = (C.c_uint32 * N_KERNEL_IDS)()
        _check(lib().udpdk_gpu_timing_read(self.handle, ms, n), "timing_read")
        return list(ms), list(n)


@dataclass
class RxDeviceBatch:
    frames: DeviceBuffer
    frames_bytes: int
    offset: DeviceBuffer
    length: DeviceBuffer
    ptype: DeviceBuffer | None
    n: int


@dataclass
class RxDeviceOut:
    meta: DeviceBuffer
    lane_off: DeviceBuffer
    lane_pkt: DeviceBuffer
    lane_cap: int
    n: int
    n_lanes: int


FRAMES_TAILROOM = 16    # UDPDK_GPU_FRAMES_TAILROOM


def rx_upload(ctx: GpuContext, frames: np.ndarray, offset: np.ndarray, length: np.ndarray,
              ptype: np.ndarray | None = None) -> RxDeviceBatch:
    """Device copies of a batch; the frames buffer gets UDPDK_GPU_FRAMES_TAILROOM readable bytes
    past the frame data."""
    fb = ctx.alloc(int(frames.nbytes) + FRAMES_TAILROOM)
    _check(lib().udpdk_gpu_h2d(ctx.handle, C.c_void_p(fb.ptr), frames.ctypes.data_as(C.c_void_p),
                               int(frames.nbytes)), "udpdk_gpu_h2d")
    ctx.sync()
    return RxDeviceBatch(fb, int(frames.nbytes), ctx.upload(offset.astype(np.uint32)),
                         ctx.upload(length.astype(np.uint16)),
                         ctx.upload(ptype.astype(np.uint32)) if ptype is not None else None,
                         int(len(offset)))


def rx_alloc_out(ctx: GpuContext, n: int, n_lanes: int, lane_cap: int) -> RxDeviceOut:
    return RxDeviceOut(ctx.alloc(4 * max(1, n)), ctx.alloc(4 * (n_lanes + 1)),
                       ctx.alloc(4 * max(1, lane_cap)), lane_cap, n, n_lanes)


def rx_enqueue(ctx: GpuContext, b: RxDeviceBatch, o: RxDeviceOut) -> int:
    bt = RxBatch(b.frames.ptr, b.frames_bytes, b.offset.ptr, b.length.ptr,
                 b.ptype.ptr if b.ptype is not None else None, b.n)
    ot = RxOut(o.meta.ptr, o.lane_off.ptr, o.lane_pkt.ptr, o.lane_cap)
    return lib().udpdk_gpu_rx(ctx.handle, C.byref(bt), C.byref(ot))


def rx_stats(ctx: GpuContext) -> tuple[int, RxStats]:
    st = RxStats()
    rc = lib().udpdk_gpu_rx_stats(ctx.handle, C.byref(st))
    return rc, st


def rx_run(ctx: GpuContext, b: RxDeviceBatch, o: RxDeviceOut):
    """Run the RX pipeline and download (meta, lane_off, lane_pkt[:D], counters)."""
    _check(rx_enqueue(ctx, b, o), "udpdk_gpu_rx")
    rc, st = rx_stats(ctx)
    if rc not in (0, -errno.ENOSPC):
        _check(rc, "udpdk_gpu_rx_stats")
    meta = ctx.download(o.meta, np.uint32, o.n)
    loff = ctx.download(o.lane_off, np.uint32, o.n_lanes + 1)
    d = min(int(st.deliveries), o.lane_cap)
    pkt = ctx.download(o.lane_pkt, np.uint32, d)
    return meta, loff, pkt, np.array(st.counters[:], np.uint64), rc


@dataclass
class RxDeviceGather:
    payload: DeviceBuffer
    slot_bytes: int
    length: DeviceBuffer
    src_ip: DeviceBuffer
    src_port: DeviceBuffer
    count: int


def rx_alloc_gather(ctx: GpuContext, count: int, slot_bytes: int) -> RxDeviceGather:
    c = max(1, count)
    return RxDeviceGather(ctx.alloc(c * slot_bytes), slot_bytes, ctx.alloc(4 * c), ctx.alloc(4 * c),
                          ctx.alloc(2 * c), count)


def rx_gather_enqueue(ctx: GpuContext, b: RxDeviceBatch, lane_pkt: DeviceBuffer, first: int,
                      g: RxDeviceGather) -> int:
    bt = RxBatch(b.frames.ptr, b.frames_bytes, b.offset.ptr, b.length.ptr,
                 b.ptype.ptr if b.ptype is not None else None, b.n)
    gt = RxGather(g.payload.ptr, g.slot_bytes, g.length.ptr, g.src_ip.ptr, g.src_port.ptr)
    return lib().udpdk_gpu_rx_gather(ctx.handle, C.byref(bt), C.c_void_p(lane_pkt.ptr), first,
                                     g.count, C.byref(gt))


def rx_gather_run(ctx: GpuContext, b: RxDeviceBatch, lane_pkt: DeviceBuffer, first: int,
                  g: RxDeviceGather):
    """Gather lane entries [first, first + count) and download (payload slots as a
    [count, slot_bytes] u8 array, len, src_ip, src_port)."""
    _check(rx_gather_enqueue(ctx, b, lane_pkt, first, g), "udpdk_gpu_rx_gather")
    ctx.sync()
    pay = ctx.download(g.payload, np.uint8, g.count * g.slot_bytes).reshape(g.count, g.slot_bytes)
    return (pay, ctx.download(g.length, np.uint32, g.count), ctx.download(g.src_ip, np.uint32, g.count),
            ctx.download(g.src_port, np.uint16, g.count))


def rx_gather_packed_run(ctx: GpuContext, b: RxDeviceBatch, lane_pkt: DeviceBuffer, first: int,
                         slot_off: np.ndarray):
    """udpdk_gpu_rx_gather_packed over lane entries [first, first + len(slot_off) - 1): entry k's
    buffer is bytes [slot_off[k], slot_off[k + 1]) of one payload area. Returns (payload area
    u8, len, src_ip, src_port)."""
    count = len(slot_off) - 1
    so = ctx.upload(np.asarray(slot_off, np.uint32))
    total = int(slot_off[-1])
    pay = ctx.alloc(max(16, total))
    ln, ip, pt = ctx.alloc(4 * max(1, count)), ctx.alloc(4 * max(1, count)), ctx.alloc(2 * max(1, count))
    bt = RxBatch(b.frames.ptr, b.frames_bytes, b.offset.ptr, b.length.ptr,
                 b.ptype.ptr if b.ptype is not None else None, b.n)
    gt = RxGather(pay.ptr, 16, ln.ptr, ip.ptr, pt.ptr)
    _check(lib().udpdk_gpu_rx_gather_packed(ctx.handle, C.byref(bt), C.c_void_p(lane_pkt.ptr), first, count,
                                            C.c_void_p(so.ptr), C.byref(gt)), "udpdk_gpu_rx_gather_packed")
    ctx.sync()
    out = (ctx.download(pay, np.uint8, total), ctx.download(ln, np.uint32, count),
           ctx.download(ip, np.uint32, count), ctx.download(pt, np.uint16, count))
    for x in (so, pay, ln, ip, pt):
        x.free()
    return out


@dataclass
class DevRef:
    """A device pointer the context owns (no free)."""
    ptr: int


def frag_table_create(ctx: GpuContext, bucket_num: int = 0x1000, bucket_entries: int = 16,
                      max_cycles: int = 1000, max_dgram: int = 65515, max_entries: int = 0, flags: int = 0):
    cfg = FragTableCfg(bucket_num, bucket_entries, max_cycles, max_dgram, max_entries, flags, 0)
    _check(lib().udpdk_gpu_frag_table_create(ctx.handle, C.byref(cfg)), "udpdk_gpu_frag_table_create")


def rx_reassemble(ctx: GpuContext, b: RxDeviceBatch, meta: DeviceBuffer, tms: int, inplace: bool = False):
    """Reassembly step for a batch whose verdicts are in meta. Returns (RxDeviceBatch of the
    reassembled frames (context-owned, or b's own frame buffer when inplace reassembled every
    datagram in place), origin DevRef, stats dict)."""
    bt = RxBatch(b.frames.ptr, b.frames_bytes, b.offset.ptr, b.length.ptr,
                 b.ptype.ptr if b.ptype is not None else None, b.n)
    o = ReasmOut()
    fn = "udpdk_gpu_rx_reassemble_inplace" if inplace else "udpdk_gpu_rx_reassemble"
    _check(getattr(lib(), fn)(ctx.handle, C.byref(bt), C.c_void_p(meta.ptr), tms, C.byref(o)), fn)
    ob = o.batch
    rb = RxDeviceBatch(DevRef(ob.frames_dev or 0), int(ob.frames_bytes), DevRef(ob.offset_dev or 0),
                       DevRef(ob.length_dev or 0), DevRef(ob.ptype_dev or 0), int(ob.n))
    return rb, DevRef(o.origin_dev or 0), dict(zip(RS_STATS, list(o.stats)))


def rss_conf(n_queues: int, reta=None, key: bytes | None = None, hash_types: int = 3) -> RssConf:
    """udpdk_gpu_rss_default_conf, optionally with another redirection table / key / types."""
    cf = RssConf()
    _check(lib().udpdk_gpu_rss_default_conf(C.byref(cf), n_queues), "udpdk_gpu_rss_default_conf")
    if reta is not None:
        cf.reta_size = len(reta)
        for i, q in enumerate(reta):
            cf.reta[i] = int(q)
    if key is not None:
        for i in range(40):
            cf.key[i] = key[i]
    cf.hash_types = hash_types
    return cf


def rss_run(ctx: GpuContext, b: RxDeviceBatch, cf: RssConf):
    """Configure RSS, run it over a device batch and download (hash, queue_off, queue_pkt)."""
    _check(lib().udpdk_gpu_rss_config(ctx.handle, C.byref(cf)), "udpdk_gpu_rss_config")
    n = b.n
    h, qo, qp = ctx.alloc(4 * max(1, n)), ctx.alloc(4 * (cf.n_queues + 1)), ctx.alloc(4 * max(1, n))
    bt = RxBatch(b.frames.ptr, b.frames_bytes, b.offset.ptr, b.length.ptr,
                 b.ptype.ptr if b.ptype is not None else None, n)
    _check(lib().udpdk_gpu_rss(ctx.handle, C.byref(bt), C.byref(RssOut(h.ptr, qo.ptr, qp.ptr))),
           "udpdk_gpu_rss")
    ctx.sync()
    out = (ctx.download(h, np.uint32, n), ctx.download(qo, np.uint32, cf.n_queues + 1),
           ctx.download(qp, np.uint32, n))
    for x in (h, qo, qp):
        x.free()
    return out


def download_ptr(ctx: GpuContext, ptr: int, dtype, count: int) -> np.ndarray:
    out = np.zeros(max(1, count), dtype)
    if count:
        _check(lib().udpdk_gpu_d2h(ctx.handle, out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
                                   count * np.dtype(dtype).itemsize), "udpdk_gpu_d2h")
        ctx.sync()
    return out[:count]


def geometry(n: int, n_lanes: int) -> tuple[int, int]:
    t = C.c_uint32()
    k = C.c_uint32()
    _check(lib().udpdk_gpu_rx_geometry(n, n_lanes, C.byref(t), C.byref(k)), "rx_geometry")
    return t.value, k.value


# ---- host API helpers -----------------------------------------------------------------------------
SOL_SOCKET = socket.SOL_SOCKET
SO_REUSEADDR = socket.SO_REUSEADDR
SO_REUSEPORT = getattr(socket, "SO_REUSEPORT", 15)


def sockaddr_in(ip: str | int, port_host: int) -> bytes:
    """struct sockaddr_in with sin_port = htons(port_host)."""
    ipb = socket.inet_aton(ip) if isinstance(ip, str) else struct.pack("<I", ip)
    return struct.pack("<H", socket.AF_INET) + struct.pack(">H", port_host) + ipb + b"\0" * 8


def raw_ip(ip: str) -> int:
    """Raw network-order IPv4 as the reference holds it (s_addr read as a LE integer)."""
    return struct.unpack("<I", socket.inet_aton(ip))[0]


def raw_port(port_host: int) -> int:
    return struct.unpack("<H", struct.pack(">H", port_host))[0]


class HostApi:
    """Thin wrappers around the udpdk_api.h calls (errno via ctypes.get_errno not used: the
    library sets the C errno; we read it through the libc symbol)."""

    def __init__(self):
        self.L = lib()
        self._errno = getattr(C.CDLL(None), "__errno_location")
        self._errno.restype = C.POINTER(C.c_int)

    def errno(self) -> int:
        return self._errno().contents.value

    def reset(self):
        self.L.udpdk_host_reset()

    def socket(self, domain=socket.AF_INET, typ=socket.SOCK_DGRAM, proto=0) -> int:
        return self.L.udpdk_socket(domain, typ, proto)

    def setsockopt(self, s, level, opt, val: int) -> int:
        v = C.c_int(val)
        return self.L.udpdk_setsockopt(s, level, opt, C.byref(v), 4)

    def getsockopt(self, s, level, opt) -> tuple[int, int]:
        v = C.c_int(-1)
        ln = C.c_uint32(4)
        rc = self.L.udpdk_getsockopt(s, level, opt, C.byref(v), C.byref(ln))
        return rc, v.value

    def bind(self, s, ip: str | int, port_host: int, addrlen: int = 16) -> int:
        a = C.create_string_buffer(sockaddr_in(ip, port_host), 16)
        return self.L.udpdk_bind(s, a, addrlen)

    def close(self, s) -> int:
        return self.L.udpdk_close(s)

    def sendto(self, s, payload: bytes, ip: str, port_host: int, flags: int = 0) -> int:
        a = C.create_string_buffer(sockaddr_in(ip, port_host), 16)
        buf = C.create_string_buffer(payload, max(1, len(payload)))
        return self.L.udpdk_sendto(s, buf, len(payload), flags, a, 16)

    def recvfrom(self, s, maxlen: int = 2048):
        buf = C.create_string_buffer(maxlen)
        a = C.create_string_buffer(16)
        al = C.c_uint32(16)
        n = self.L.udpdk_recvfrom(s, buf, maxlen, 0, a, C.byref(al))
        if n < 0:
            return n, None, None
        port = struct.unpack(">H", a.raw[2:4])[0]
        ip = socket.inet_ntoa(a.raw[4:8])
        return n, buf.raw[:n], (ip, port)

    def tx_drain(self, max_frames=4096, cap=1 << 22):
        """Frames built on the GPU from the queued sends (needs udpdk_init)."""
        out = np.zeros(cap, np.uint8)
        off = np.zeros(max_frames, np.uint32)
        ln = np.zeros(max_frames, np.uint16)
        n = C.c_uint32()
        rc = self.L.udpdk_tx_drain(_ptr(out), cap, _ptr(off), _ptr(ln), max_frames, C.byref(n))
        if rc != 0:
            raise UdpdkError(f"udpdk_tx_drain errno={self.errno()}")
        return [bytes(out[off[i]:off[i] + ln[i]]) for i in range(n.value)]

    def tx_pending(self) -> int:
        return int(self.L.udpdk_tx_pending())

    def tx_dropped(self) -> int:
        return int(self.L.udpdk_tx_dropped())

    def rx_nobufs(self) -> int:
        return int(self.L.udpdk_rx_nobufs())

    def slots(self, n: int = 8):
        t = (Slot * n)()
        _check(self.L.udpdk_slot_table(t, n), "udpdk_slot_table")
        return [(t[i].ip, t[i].udp_port, t[i].bound) for i in range(n)]

    def config_set(self, src_mac: bytes, dst_mac: bytes, src_ip: str):
        s = C.create_string_buffer(src_mac, 6)
        d = C.create_string_buffer(dst_mac, 6)
        return self.L.udpdk_config_set(s, d, raw_ip(src_ip))

    def snapshot(self, compat: bool = False) -> BindSnapshot:
        snap = BindSnapshot()
        _check(self.L.udpdk_btable_snapshot(C.byref(snap), int(compat)), "udpdk_btable_snapshot")
        return snap

    def port_lists(self, compat: bool = False) -> dict[int, list[tuple[int, int, int]]]:
        s = self.snapshot(compat)
        out = {}
        for p in range(65536):
            c = s.port_count[p]
            if c:
                f = s.port_first[p]
                out[p] = [(s.binds[f + i].ip, s.binds[f + i].sockfd, s.binds[f + i].reuse) for i in range(c)]
        return out
