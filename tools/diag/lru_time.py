"""Time of reassembly calls that meet the max_entries limit (the LRU head lookup).
A table of 0x1000 x 16 entries with max_entries M is filled with M pending flows (first fragments
only) in call 1; call 2, after they expired, brings N2 new flows' first fragments: a new flow
whose two buckets hold no (expired) entry finds the table at its limit and deletes the LRU head
(ip_frag_find's lru deletion) before taking an empty entry (about 1 in 7 at M = 4000), on the
serial path; the others reuse an expired entry of their buckets. Prints per-call wall time and the stats. Usage (GPU box):
  UDPDK_LIB_OVERRIDE=tools/var/prev.so python tools/diag/lru_time.py [M] [N2]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from udpdk_amd import abi, frames as F  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
N2 = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
ctx = abi.GpuContext(0, max_frames=1 << 17, max_lanes=16)
b = F.frag_batch(M + N2, 2952)                  # 2 fragments per datagram: 1514 + 1514 B frames
per = 2 * 1514
ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
abi.frag_table_create(ctx, 0x1000, 16, 1000, 65515, max_entries=M)
out = []
for k0, k1, tms in ((0, M, 0), (M, M + N2, 5000)):
    off = (np.arange(k0, k1, dtype=np.uint64) * per).astype(np.uint32)
    ln = np.full(k1 - k0, 1514, np.uint16)
    db = abi.rx_upload(ctx, b.frames, off, ln)
    db.frames_bytes = b.frames_bytes
    o = abi.rx_alloc_out(ctx, k1 - k0, 1, k1 - k0)
    abi.rx_run(ctx, db, o)
    ctx.sync()
    t0 = time.perf_counter()
    rb, _, st = abi.rx_reassemble(ctx, db, o.meta, tms)
    ms = 1e3 * (time.perf_counter() - t0)
    out.append({"call": len(out) + 1, "frags": k1 - k0, "ms": round(ms, 3),
                "stats": {k: int(v) for k, v in st.items()}})
    for x in (db.frames, db.offset, db.length, o.meta, o.lane_off, o.lane_pkt):
        x.free()
print(json.dumps({"lib": os.environ.get("UDPDK_LIB_OVERRIDE", "base"), "max_entries": M, "calls": out}))
