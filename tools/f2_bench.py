"""Runs bench.py's f2/f4 lines alone (fragmented TX, reassembly, RSS) and prints them as JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from udpdk_amd import abi  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "all"
ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
if what in ("all", "tx"):
    print(json.dumps(bench.tx_line(ctx, 22, 1 << 20, 50)), flush=True)
    print(json.dumps(bench.tx_line(ctx, 1458, 1 << 20, 50)), flush=True)
    print(json.dumps(bench.tx_line(ctx, 2952, 1 << 18, 50, mtu=1500)), flush=True)
if what in ("all", "rss"):
    print(json.dumps(bench.rss_line(ctx, 2, 8, 50)), flush=True)
    print(json.dumps(bench.rss_line(ctx, 5, 8, 50)), flush=True)
if what in ("all", "reasm"):
    print(json.dumps(bench.reasm_line(ctx, 1 << 18, 2952, 10)), flush=True)
ctx.close()
