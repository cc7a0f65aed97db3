import sys, json
sys.path.insert(0, '.')
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 21, max_lanes=4096)
which = sys.argv[1] if len(sys.argv) > 1 else "both"
if which in ("both", "1500"):
    print(json.dumps(bench.tx_line(ctx, 1458, 1 << 20, 20)))
if which in ("both", "frag"):
    print(json.dumps(bench.tx_line(ctx, 2952, 1 << 18, 20, mtu=1500)))
