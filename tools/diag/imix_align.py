"""Diagnostic: rx_classify on the config-4 IMIX batch with frames packed back to back (as built)
and the same frames repacked at 64-byte-aligned offsets (and 1500 B frames likewise, config 3):
does the alignment of the tail pass's byte-aligned chunk loads matter? Kernel durations from the
library's timing mode, depth 1."""
import json, sys
import numpy as np
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi, frames as F


def repack(b, align):
    ln = b.length.astype(np.int64)
    al = (ln + align - 1) // align * align
    off2 = np.concatenate([[0], np.cumsum(al)[:-1]]).astype(np.uint32)
    fr2 = np.zeros(int(al.sum()) + 256, np.uint8)
    idx = np.repeat(np.arange(b.n), ln)
    pos = np.arange(int(ln.sum())) - np.repeat(np.cumsum(ln) - ln, ln)
    fr2[off2[idx].astype(np.int64) + pos] = b.frames[b.offset[idx].astype(np.int64) + pos]
    return F.Batch(fr2, off2, b.length, int(al.sum()))


ctx = abi.GpuContext(0, max_frames=1 << 20, max_lanes=1024)
out = {}
for cfg in (4, 3):
    w = F.config_batch(cfg)
    for name, bb in (("packed", w.batch), ("aligned64", repack(w.batch, 64))):
        w2 = F.Workload(w.name, bb, w.n_sockets, w.base_port)
        rx = bench.Rx(ctx, w2, 640 << 20)
        ctx.pipeline(1)
        wall, gstep, kt, st = bench.time_loop(rx, 50, 5, lambda: None, 1)
        out[f"config {cfg} {name}"] = {"classify_us": round(kt.get("rx_classify", 0), 2), "step_us": round(gstep * 1e3, 2)}
        del rx
print(json.dumps(out))
