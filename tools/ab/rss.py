import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
for cfg in (2, 5):
    print(json.dumps(bench.rss_line(ctx, cfg, 8, 50)))
