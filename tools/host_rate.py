"""Host enqueue rate of the bench's timed loop vs the GPU's rate: time to issue K udpdk_gpu_rx
calls without waiting, then until the GPU finishes them (config 2, pipelined as the bench)."""
import sys, time, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi, frames as F

ctx = abi.GpuContext(0, max_frames=1 << 20, max_lanes=16)
w = F.config_batch(2)
rx = bench.Rx(ctx, w, 640 << 20)
ctx.pipeline(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
for i in range(20):
    rx.step(i)
ctx.sync()
for K in (20, 200, 1000):
    best = None
    for rep in range(3):
        ctx.sync()
        t0 = time.perf_counter()
        for i in range(K):
            rx.step(i)
        t1 = time.perf_counter()
        ctx.join()
        ctx.sync()
        t2 = time.perf_counter()
        r = ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6)
        best = r if best is None or r[1] < best[1] else best
    print(json.dumps({"K": K, "host_issue_us_per_step": round(best[0], 2), "wall_us_per_step": round(best[1], 2)}))
