import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=4096)
for cfg in (2, 3):
    print(json.dumps(bench.gather_line(ctx, cfg, 50)))
print(json.dumps(bench.gather_line(ctx, 2, 50, slot=0)))
