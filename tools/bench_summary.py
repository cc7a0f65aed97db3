"""One-screen summary of a bench.py JSON line (gpurun_out/bench.json by default)."""
import json
import sys

d = json.loads(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json").read().strip().splitlines()[-1])
print(f"{d['config']['workload']}: {d['value']} Mpkt/s, gpu {d['gpu_us_per_step']} us/step, depth1 "
      f"{d['depth1']['gpu_us_per_step']} us, kernels {d['kernel_us']}, frac {d['roofline']['frac']}")
for o in d.get("other_configs", []):
    if "error" in o:
        print("  ", o)
        continue
    print(f"  {o['workload']}: {o['mpkt_s']} Mpkt/s, gpu {o['gpu_us_per_step']} us, kernels {o['kernel_us']}, "
          f"cls {o['frac_hbm_classify']}, pipe {o['frac_hbm_pipeline']}, parity {o['parity']['match']}")
for k in ("tx", "gather", "rss", "reassembly", "end_to_end"):
    for o in d.get(k, []):
        print(f"  {k}: " + ", ".join(f"{a}={b}" for a, b in o.items() if a not in ("path",)))
