import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=4096)
for plen in (22, 38, 1458):
    print(json.dumps(bench.tx_line(ctx, plen, 1 << 20, 50)))
