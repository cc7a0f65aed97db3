#!/bin/bash
# FETCH_SIZE per dispatch of the span-sweep shapes (tools/probe/sweep_probe.hip), 1500 B and IMIX.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/sweep
for m in 1500 imix; do
  timeout -k 10 60 ./tools/bin/sweep_probe $m > gpurun_out/sweep/t_$m.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $PWD/gpurun_out/sweep/f_$m -o p -- $PWD/tools/bin/sweep_probe $m > gpurun_out/sweep/f_$m.log 2>&1 || exit 1
  echo "== $m"; cat gpurun_out/sweep/t_$m.log
  python3 - gpurun_out/sweep/f_$m <<'PY'
import csv, glob, collections, sys
for f in glob.glob(sys.argv[1] + "/**/p_counter_collection.csv", recursive=True):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0][-24:]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{k:26s} FETCH_SIZE {sum(v)/len(v):.0f} KiB  ({2*1024*sum(v)/len(v)/1e6:.1f} MB)")
PY
done
