"""Socket-path sweep of [gpu] host_copy_min (payloads copied from the host frames when a poll's
mean admitted payload is at least this many bytes, else gathered on the GPU): bench.py's
socket_path lines for IMIX and 1500 B frames at each threshold. Usage (GPU box):
python tools/sock_tune.py [thresholds...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for t in [int(x) for x in sys.argv[1:]] or [64, 256, 512, 1 << 30]:
    for line in bench.socket_path_lines(((1 << 20, 0, 1024, 3), (1 << 20, 1500, 1024, 3), (1 << 20, 64, 1024, 3)),
                                        gpu_extra=f"host_copy_min = {t}\n"):
        print(json.dumps({"host_copy_min": t, "frame_bytes": line.get("frame_bytes"),
                          "poll_ms": line.get("poll_ms"), "recv_ms": line.get("recv_ms"),
                          "end_to_end_mdgram_s": line.get("end_to_end_mdgram_s"), "error": line.get("error")}),
              flush=True)
