"""Where the bench's 20-step timed region goes (config 2, pipelined): host enqueue time of the K
calls alone (no sync inside), the whole region (device sync on both sides), and an empty region
(the two syncs alone), for K = 1, 20 and 200. Prints one JSON line per K."""
import json
import sys
import time

sys.path.insert(0, '.')
import bench
from udpdk_amd import abi, frames as F

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
rx = bench.Rx(ctx, F.config_batch(cfg), 640 << 20)
ctx.pipeline(depth)
for i in range(20):
    rx.step(i)
rx.check()
for K in (1, 20, 200):
    best = {}
    for rep in range(5):
        bench.device_sync()
        t0 = time.perf_counter()
        for i in range(K):
            rx.step(i)
        t1 = time.perf_counter()
        bench.device_sync()
        t2 = time.perf_counter()
        bench.device_sync()
        t3 = time.perf_counter()
        bench.device_sync()
        t4 = time.perf_counter()
        r = {"enqueue_us_per_step": 1e6 * (t1 - t0) / K, "region_us_per_step": 1e6 * (t2 - t0) / K,
             "region_us": 1e6 * (t2 - t0), "empty_sync_us": 1e6 * (t4 - t3)}
        for k, v in r.items():
            best.setdefault(k, []).append(round(v, 2))
    print(json.dumps({"config": cfg, "depth": depth, "K": K, **best}), flush=True)
rx.check()
