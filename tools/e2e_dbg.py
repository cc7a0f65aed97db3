import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
L = abi.lib()
for cfg in (3, 2, 3):
    try:
        print(cfg, bench.end_to_end(ctx, cfg, 2), flush=True)
    except Exception as e:
        print(cfg, "ERR", e, "hip", L.udpdk_gpu_last_hip_error(ctx.handle), flush=True)
        break
