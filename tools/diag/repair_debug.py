"""Fused-repair diagnostics on the GPU (one-off): the failing speculation case with the first
differing lane entries printed, then a sporadic-drop loop with per-call progress."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "oracle"))
import numpy as np
import oracle as O
from udpdk_amd import abi, frames as F

ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
lists = {abi.raw_port(10001): [(0, 0, 0)]}
hs = abi.snapshot_from_lists(lists, 1)
ctx.upload_snapshot(hs)
bt = O.bindtable_from_lists(lists)
n = 10 * 1024 + 300
for k in range(3):
    b = F.build_frames(np.full(n, 64, np.uint32), np.full(n, 10001, np.uint32), 40 + k)
    if k == 1:
        v = b.frames[:n * 64].reshape(n, 64)
        rows = np.arange(17, 1024, 101)
        v[rows, 36] = 0x4E
        v[rows, 37] = 0x20
    wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, 1)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, n, 1, 4 * n)
    meta, loff, pkt, cnt, rc = abi.rx_run(ctx, db, out)
    bad = np.nonzero(wp != pkt[:len(wp)])[0] if len(pkt) >= len(wp) else np.arange(len(wp))
    print(f"call {k}: rc {rc} total {loff[1]} want {wl[1]} bad {len(bad)} first {bad[:8]}", flush=True)
    if len(bad):
        i = bad[0]
        print("  want", wp[max(0, i - 3):i + 5], "\n  got ", pkt[max(0, i - 3):i + 5], flush=True)
        tiles = np.unique(bad // 1024)
        print("  bad by position/1024:", tiles[:20], flush=True)
for k in range(20):
    t0 = time.time()
    b = F.build_frames(np.full(1 << 20, 64, np.uint32), np.full(1 << 20, 10001, np.uint32), 70 + k)
    if k % 3 == 1:
        v = b.frames[:(1 << 20) * 64].reshape(1 << 20, 64)
        v[[1000 + k * 7919], 36] = 0x4E
        v[[1000 + k * 7919], 37] = 0x20
    wm, wl, wp, wc = O.rx(bt, b.frames, b.frames_bytes, b.offset, b.length, None, 1)
    db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
    db.frames_bytes = b.frames_bytes
    out = abi.rx_alloc_out(ctx, 1 << 20, 1, 1 << 20)
    meta, loff, pkt, cnt, rc = abi.rx_run(ctx, db, out)
    print(f"loop {k}: rc {rc} same {np.array_equal(wp, pkt)} {time.time() - t0:.2f}s", flush=True)
