"""Print the mean per-dispatch value of every PMC counter in rocprofv3 counter_collection CSVs,
per kernel (diagnostic; usage: python tools/pmc_kernel.py gpurun_out/pmcp/*/p_counter_collection.csv)."""
import collections
import csv
import sys

agg = collections.defaultdict(list)
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
