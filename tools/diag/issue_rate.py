"""Host issue time of bench.py's config-2 step (udpdk_gpu_rx through ctypes) against the GPU's
pace: K calls timed on the host without a sync (the issue rate), then to the closing sync (the
region bench.py times), at pipeline depth 3. Usage (GPU box): python tools/diag/issue_rate.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from udpdk_amd import abi, frames as F  # noqa: E402

if os.environ.get("SPIN"):
    import ctypes
    print("hipSetDeviceFlags", ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(int(os.environ["SPIN"])))
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
rx_depth = int(os.environ.get("DEPTH", "3"))
rx = bench.Rx(ctx, F.config_batch(2), 640 << 20)
ctx.pipeline(rx_depth)
for i in range(50):
    rx.step(i)
bench.device_sync()
for K in (1, 2, 5, 20, 200, 20, 200):
    bench.device_sync()
    t0 = time.perf_counter()
    for i in range(K):
        rx.step(i)
    t1 = time.perf_counter()
    bench.device_sync()
    t2 = time.perf_counter()
    print(f"K={K:4d} issue {1e6 * (t1 - t0) / K:7.2f} us/call  region {1e6 * (t2 - t0) / K:7.2f} us/call  "
          f"(total {1e6 * (t2 - t0):8.1f} us, after last issue {1e6 * (t2 - t1):7.1f} us)", flush=True)
