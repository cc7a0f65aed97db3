"""Per-phase cycle stamps of rx_scan_cols (diagnostic build, make stamps): per workgroup the
column loads + chunk sums, the lane-block look-back, the base-row stores (issue), and the
dispatch timeline, for configs 5 and 4."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["UDPDK_LIB_OVERRIDE"] = os.path.join(ROOT, "tools", "diag", "libudpdk_amd.so")
sys.path.insert(0, ROOT)
import numpy as np
from udpdk_amd import abi, frames as F

PH = ["loads + chunk sums", "look-back + lane offsets", "base-row stores (issue)"]
L = abi.lib()
L.udpdk_gpu_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
NB = 4 * 8192 * 16 * 8
for cfg in (5, 4):
    dbg = ctx.upload(np.zeros(NB // 8, np.uint64))
    L.udpdk_gpu_debug_buffer(ctx.handle, C.c_void_p(dbg.ptr))
    w = F.config_batch(cfg)
    ctx.upload_snapshot(abi.snapshot_from_lists(w.port_lists(), w.n_sockets))
    db = abi.rx_upload(ctx, w.batch.frames, w.batch.offset, w.batch.length)
    db.frames_bytes = w.batch.frames_bytes
    out = abi.rx_alloc_out(ctx, w.batch.n, w.n_sockets, w.batch.n)
    for i in range(8):
        abi._check(abi.rx_enqueue(ctx, db, out), "udpdk_gpu_rx")
    abi.rx_stats(ctx)
    raw = ctx.download(dbg, np.uint64, 4 * 8192 * 16)[3 * 8192 * 16:].reshape(8192, 16)
    raw = raw[raw[:, 4] != 0]
    d = raw.astype(np.float64)
    print(f"{w.name} scan workgroups={len(raw)}")
    for k, name in enumerate(PH):
        print(f"   {name:28s} mean {d[:, k].mean():8.0f} cyc  max {d[:, k].max():8.0f}")
    st0 = raw[:, 3].astype(np.int64) - int(raw[:, 3].min())
    en0 = raw[:, 4].astype(np.int64) - int(raw[:, 3].min())
    dur = en0 - st0
    pct = lambda x: " ".join(f"{np.percentile(x, q) / 100:.2f}" for q in (0, 10, 50, 90, 100))
    print(f"   span {en0.max() / 100:.2f} us; start us p0/10/50/90/100: {pct(st0)}; duration us: {pct(dur)}")
    order = np.argsort(raw[:, 5])
    print("   end us by ticket (every 16th):", " ".join(f"{en0[order][i] / 100:.2f}" for i in range(0, len(order), 16)))
ctx.close()
