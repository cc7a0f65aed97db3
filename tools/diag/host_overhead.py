"""Host enqueue cost of udpdk_gpu_rx: wall time per call for a tiny batch (GPU work ~ a few us),
with and without per-kernel timing events, for the fused (1 lane) and general (1024 lanes) paths."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from udpdk_amd import abi, frames as F

ctx = abi.GpuContext(0, max_frames=1 << 20, max_lanes=4096)
L = abi.lib()
t = time.perf_counter()
for _ in range(100000):
    L.udpdk_gpu_abi_version()
print(f"ctypes call: {(time.perf_counter() - t) * 10:.2f} us")
for lanes in (1, 1024):
    n = 4096
    b = F.build_frames(np.full(n, 64, np.uint32), 10000 + np.arange(n) % lanes, 1)
    lists = {abi.raw_port(10000 + i): [(0, i, 0)] for i in range(lanes)}
    ctx.upload_snapshot(abi.snapshot_from_lists(lists, lanes))
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, n, lanes, n)
    bt = abi.RxBatch(db.frames.ptr, db.frames_bytes, db.offset.ptr, db.length.ptr, None, n)
    ot = abi.RxOut(out.meta.ptr, out.lane_off.ptr, out.lane_pkt.ptr, n)
    import ctypes as C
    pb, po = C.byref(bt), C.byref(ot)
    for timing in (0, 1, 8):
        ctx.timing(timing)
        for _ in range(50):
            L.udpdk_gpu_rx(ctx.handle, pb, po)
        ctx.sync()
        K = 2000
        t = time.perf_counter()
        for _ in range(K):
            L.udpdk_gpu_rx(ctx.handle, pb, po)
        t_enq = time.perf_counter() - t
        ctx.sync()
        t_all = time.perf_counter() - t
        ms, cnt = ctx.timing_read() if timing else ([0] * 4, [0] * 4)
        print(f"lanes={lanes} timing={timing}: enqueue {1e6 * t_enq / K:.2f} us/call, "
              f"wall {1e6 * t_all / K:.2f} us/call, gpu classify {1e3 * ms[0] / max(1, cnt[0]):.2f} us")
    ctx.timing(0)
ctx.close()
