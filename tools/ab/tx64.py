import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=4096)
print(json.dumps(bench.tx_line(ctx, 22, 1 << 20, 20)))
print(json.dumps(bench.gather_line(ctx, 2, 20)))
