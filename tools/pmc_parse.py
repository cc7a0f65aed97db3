"""Fold the rocprofv3 PMC passes of tools/pmc_traffic.sh into profiles/traffic.json.

Per workload and kernel: mean FETCH_SIZE and WRITE_SIZE per dispatch (KiB, as rocprofv3
reports them) and the HBM-side bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: on
gfx950 FETCH_SIZE tallies 128-B requests of wide (16 B/lane) reads at 64 B, so it reads half the
bytes (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16 B/lane stores."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from udpdk_amd import frames as F  # noqa: E402

src = os.path.join(ROOT, "gpurun_out", "pmc")
out = {}
for cfg in (1, 2, 3, 4, 5):
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = os.path.join(src, f"{ctr}_c{cfg}", "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            # "void udpdk::rx_classify<1>(udpdk::RxArgs)" -> "udpdk::rx_classify" (both forms)
            kn = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            agg[kn].append(float(r["Counter_Value"]))
        vals[ctr] = {k: sum(v) / len(v) for k, v in agg.items()}
    if len(vals) < 2:
        continue
    name = F.config_batch(cfg).name     # the bench workload (its default frame count)
    kern = {}
    for k in vals["FETCH_SIZE"]:
        if not k.startswith("udpdk::"):
            continue
        fk, wk = vals["FETCH_SIZE"][k], vals["WRITE_SIZE"].get(k, 0.0)
        kern[k.split("::")[1]] = {"fetch_kib": round(fk, 1), "write_kib": round(wk, 1),
                                  "hbm_bytes_per_launch": int((2 * fk + wk) * 1024)}
    out[name] = {"kernels": kern,
                 "rx_classify_hbm_bytes_per_launch": kern.get("rx_classify", {}).get("hbm_bytes_per_launch")}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
path = os.path.join(ROOT, "profiles", "traffic.json")
# workloads not measured in this pass keep their earlier entries
prev = json.load(open(path))["workloads"] if os.path.exists(path) else {}
for k, v in out.items():
    v["measured_with"] = os.environ.get("PMC_TAG", "")
prev.update(out)
with open(path, "w") as f:
    json.dump({"method": __doc__.strip().split("\n\n")[1].replace("\n", " "), "workloads": prev}, f, indent=1)
print(json.dumps(out, indent=1))
