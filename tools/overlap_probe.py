"""Does pipelining consecutive batches over two contexts (two streams, own workspaces) raise
device-resident throughput? Config 2 batch, rotated device copies, K calls alternating between
the contexts vs all on one; host wall time between syncs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from udpdk_amd import abi, frames as F  # noqa: E402

w = F.config_batch(int(os.environ.get("CFG", "2")))
ctxs = [abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096) for _ in range(2)]
rxs = [bench.Rx(c, w, 640 << 20) for c in ctxs]
K = 200
for depth in (1, 2):
    for i in range(20):
        rxs[i % depth].step(i)
    for c in ctxs:
        c.sync()
    t0 = time.perf_counter()
    for i in range(K):
        rxs[i % depth].step(i)
    for c in ctxs:
        c.sync()
    dt = (time.perf_counter() - t0) / K
    print(f"{w.name} depth {depth}: {1e6 * dt:.2f} us/step, {w.batch.n / dt / 1e6:.0f} Mpkt/s")
for r in rxs:
    r.check()
