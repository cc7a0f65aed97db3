"""Timing-only reassembly loop for kernel-stat diagnostics of library variants (no result checks:
diagnostic variants skip work): the bench's 2^18 x 2952 B batch, copying calls."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from udpdk_amd import abi, frames as F  # noqa: E402

ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
b = F.frag_batch(1 << 18, 2952)
ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
abi.frag_table_create(ctx, 0x1000, 16, 1 << 40, 65515)
db = abi.rx_upload(ctx, b.frames, b.offset, b.length)
db.frames_bytes = b.frames_bytes
out = abi.rx_alloc_out(ctx, b.n, 1, b.n)
abi.rx_run(ctx, db, out)
for r in range(11):
    abi.rx_reassemble(ctx, db, out.meta, r)
print("ok")
