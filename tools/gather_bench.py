"""Diagnostic: bench.py's gather side lines alone."""
import os
import sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench
from udpdk_amd import abi
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
for cfg in (2, 3, 4):
    print(bench.gather_line(ctx, cfg, 30), flush=True)
