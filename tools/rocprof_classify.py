"""Record the rocprofv3 mean duration of rx_classify for a workload in profiles/rocprof_classify.json.

    python tools/rocprof_classify.py profiles/r05a_config2_kernel_stats.csv 1M-64B-1port

bench.py reads the file and puts the rocprof-derived classify fraction beside the event-derived
one in its `roofline` object (same algorithmic bytes, the profiler's mean kernel duration). The
mean is taken over every rx_classify template instance in the CSV, weighted by calls.
"""
from __future__ import annotations

import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "rocprof_classify.json")


def classify_mean(stats_csv: str) -> tuple[float, int]:
    calls, total_ns = 0, 0.0
    with open(stats_csv) as f:
        for row in csv.DictReader(f):
            if "rx_classify" in row["Name"]:
                calls += int(row["Calls"])
                total_ns += float(row["TotalDurationNs"])
    if not calls:
        raise SystemExit(f"no rx_classify row in {stats_csv}")
    return total_ns / calls / 1e3, calls


def main():
    if len(sys.argv) != 3:
        raise SystemExit(__doc__)
    src, workload = sys.argv[1], sys.argv[2]
    mean_us, calls = classify_mean(src)
    d = json.load(open(OUT)) if os.path.exists(OUT) else {"workloads": {}}
    d["method"] = ("rocprofv3 --kernel-trace --stats of bench.py at pipeline depth 1 (one call at a "
                   "time); mean rx_classify duration over every template instance, weighted by calls")
    d["workloads"][workload] = {"mean_us": round(mean_us, 3), "calls": calls,
                                "source": os.path.relpath(os.path.abspath(src), ROOT)}
    with open(OUT, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")
    print(workload, round(mean_us, 3), "us over", calls, "calls")


if __name__ == "__main__":
    main()
