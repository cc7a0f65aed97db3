"""Reassembly of interleaved flows (diagnostic line for tools/ab.py --line reasmx): the bench's
2^18 x 2952 B datagrams with the fragments of consecutive datagram pairs interleaved (A1 B1 A2
B2: every flow in order, but no key forms one run), so the batch takes the key sorts."""
import time

import numpy as np

from udpdk_amd import abi, frames as F


def run(ctx, out):
    b = F.frag_batch(1 << 18, 2952)
    n = b.n
    order = np.arange(n).reshape(-1, 2, 2).transpose(0, 2, 1).reshape(-1)   # A1 B1 A2 B2
    off = b.offset[order].copy()
    ln = b.length[order].copy()
    ctx.upload_snapshot(abi.snapshot_from_lists({abi.raw_port(F.PORT_RECV): [(0, 0, 0)]}, 1))
    abi.frag_table_create(ctx, 0x1000, 16, 1 << 40, 65515)
    db = abi.rx_upload(ctx, b.frames, off, ln)
    db.frames_bytes = b.frames_bytes
    o = abi.rx_alloc_out(ctx, n, 1, n)
    abi.rx_run(ctx, db, o)
    rb, _, st = abi.rx_reassemble(ctx, db, o.meta, 0)
    assert st["done"] == 1 << 18 and st["sorted"] == 1, st
    t0 = time.perf_counter()
    for r in range(10):
        rb, _, st = abi.rx_reassemble(ctx, db, o.meta, r + 1)
    us = 1e6 * (time.perf_counter() - t0) / 10
    out({"workload": "reassembly 2^18 x 2952 B, pairs of flows interleaved (sorted path)",
         "us_per_call": round(us, 1), "serial": st["serial"], "sorted": st["sorted"]})
