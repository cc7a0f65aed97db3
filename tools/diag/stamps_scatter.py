"""Per-phase cycle stamps of rx_scatterw (diagnostic build, make stamps): mean cycles per
workgroup (wave 0) in each phase and the dispatch timeline, for configs 5 and 4."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["UDPDK_LIB_OVERRIDE"] = os.path.join(ROOT, "tools", "diag", "libudpdk_amd.so")
sys.path.insert(0, ROOT)
import numpy as np
from udpdk_amd import abi, frames as F

PH = ["lane_cursors", "woff zero", "pass0 count", "slice offsets", "pass1 place (ranks)", "staged: global stores",
      "staged: key starts into LDS", "staged: key-order index + position", "staged: pairs into LDS"]
L = abi.lib()
L.udpdk_gpu_debug_buffer.argtypes = [C.c_void_p, C.c_void_p]
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
NB = (2 * 8192 + 8192) * 16 * 8
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
    _, tiles = abi.geometry(w.batch.n, w.n_sockets)
    raw = ctx.download(dbg, np.uint64, (2 * 8192 + tiles) * 16)[2 * 8192 * 16:].reshape(tiles, 16)
    # a scatter workgroup may take several classify tiles: keep the rows its workgroups wrote
    # (row = scatter tile; the rows past the scatter grid stay zero in the fresh buffer)
    raw = raw[raw[:, 13] != 0]
    tiles = len(raw)
    d = raw.astype(np.float64)
    print(f"{w.name} tiles={tiles}")
    for k, name in enumerate(PH):
        print(f"   {name:16s} mean {d[:, k].mean():10.0f} cyc  max {d[:, k].max():10.0f}")
    st0 = raw[:, 12].astype(np.int64) - int(raw[:, 12].min())
    en0 = raw[:, 13].astype(np.int64) - int(raw[:, 12].min())
    dur = en0 - st0
    pct = lambda x: " ".join(f"{np.percentile(x, q) / 100:.2f}" for q in (0, 10, 50, 90, 100))
    print(f"   span {en0.max() / 100:.2f} us; start us p0/10/50/90/100: {pct(st0)}; duration us: {pct(dur)}")
ctx.close()
