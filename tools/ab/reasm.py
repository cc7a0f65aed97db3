import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
print(json.dumps(bench.reasm_line(ctx, 1 << 18, 2952, 10)))
