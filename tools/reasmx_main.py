"""One process running tools/reasm_probe_x.py's interleaved-flow reassembly line on the in-tree
library (for rocprofv3 --kernel-trace --stats, which must see the program itself after --)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from udpdk_amd import abi  # noqa: E402
import reasm_probe_x  # noqa: E402

if __name__ == "__main__":
    ctx = abi.GpuContext(0, max_frames=1 << 22, max_lanes=4096)
    reasm_probe_x.run(ctx, lambda d: print(json.dumps(d), flush=True))
