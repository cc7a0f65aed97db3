"""Diagnostic: reassembly of the bench's batch (256 K x 2952 B datagrams, 2 fragments each) with the
fragment frames back to back (byte-aligned sources, as the NIC would pack them) and repacked at
64-byte-aligned offsets; same table geometry. Prints per-call wall time for both."""
import json, sys, time
import numpy as np
sys.path.insert(0, '.')
from udpdk_amd import abi, frames as F

ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=16)
b = F.frag_batch(1 << 18, 2952)
ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
layouts = {"packed": (b.frames, b.offset, b.frames_bytes)}
al = ((b.length.astype(np.uint64) + 63) // 64 * 64)
off2 = np.concatenate([[0], np.cumsum(al)[:-1]]).astype(np.uint32)
fr2 = np.zeros(int(al.sum()) + 256, np.uint8)
for k in range(len(off2)):
    pass
src = b.frames
# vectorised repack: copy each frame's bytes
idx = np.repeat(np.arange(b.n), b.length.astype(np.int64))
pos_in = np.arange(int(b.length.astype(np.int64).sum())) - np.repeat(np.cumsum(b.length.astype(np.int64)) - b.length.astype(np.int64), b.length.astype(np.int64))
fr2[off2[idx].astype(np.int64) + pos_in] = src[b.offset[idx].astype(np.int64) + pos_in]
layouts["aligned64"] = (fr2, off2, int(al.sum()))
res = {}
for name, (frames, off, fb) in layouts.items():
    abi.frag_table_create(ctx, 0x1000, 16, 1 << 40, 65515)
    db = abi.rx_upload(ctx, frames, off, b.length)
    db.frames_bytes = fb
    out = abi.rx_alloc_out(ctx, b.n, 1, b.n)
    abi.rx_run(ctx, db, out)
    ts = []
    for r in range(8):
        ctx.sync()
        t0 = time.perf_counter()
        rb, _, st = abi.rx_reassemble(ctx, db, out.meta, r)
        ts.append(time.perf_counter() - t0)
        assert st["done"] == 1 << 18, st
    ts.sort()
    res[name] = round(ts[len(ts) // 2] * 1e6, 1)
print(json.dumps({"us_per_call": res}))
