import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=4096)
for plen, n, mtu in ((22, 1 << 20, 0), (1458, 1 << 20, 0), (2952, 1 << 18, 1500), (1458, 1 << 14, 0), (8000, 1 << 16, 1500)):
    print(json.dumps(bench.tx_line(ctx, plen, n, 20, mtu=mtu) if mtu else bench.tx_line(ctx, plen, n, 20)))
