"""Socket-path sweep of one [gpu] ini key: bench.py's socket_path lines (IMIX, 1500 B and 64 B
frames, 1 M per poll over 1024 sockets) at each value. Keys swept so far: host_copy_min (payloads
copied from the host frames from this mean payload size on), poll_chunk_mb (the pipelined poll's
chunk size, 0 = one piece). Usage (GPU box): python tools/sock_tune.py KEY VALUE..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "host_copy_min"
vals = sys.argv[2:] or ["64", "256", "512", str(1 << 30)]
sizes = [int(x) for x in os.environ.get("SOCK_SIZES", "0,1500,64").split(",")]
for v in vals:
    for line in bench.socket_path_lines(tuple((1 << 20, fb, 1024, 3) for fb in sizes),
                                        gpu_extra=f"{key} = {v}\n"):
        print(json.dumps({key: v, "frame_bytes": line.get("frame_bytes"),
                          "poll_ms": line.get("poll_ms"), "recv_ms": line.get("recv_ms"),
                          "end_to_end_mdgram_s": line.get("end_to_end_mdgram_s"),
                          "overlap_mdgram_s": line.get("overlap_mdgram_s"), "error": line.get("error")}),
              flush=True)
