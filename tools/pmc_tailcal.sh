#!/bin/bash
# Read-request size mix at the L2's memory side (TCC_EA0_RDREQ by size) for the tail-shape probe
# (tools/probe/tail_probe.hip: 1500 B and IMIX frames) and for rx_classify at configs 2-4: bytes =
# 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B against FETCH_SIZE x 2 (the streaming
# calibration). One rocprofv3 pass per counter group (4 TCC counters max per pass).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/tcal
CTRS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
summ() {
python3 - "$1" <<'PY'
import csv, glob, collections, sys
for f in glob.glob(sys.argv[1] + "/**/p_counter_collection.csv", recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0][-28:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        b = 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)
        print(f"{k:30s} " + " ".join(f"{c.replace('TCC_EA0_','')}={v:.0f}" for c, v in m.items()) + f"  sized_bytes={b/1e6:.1f}MB")
PY
}
for m in 1500 imix; do
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d $PWD/gpurun_out/tcal/sz_$m -o p -- $PWD/tools/bin/tail_probe $m > gpurun_out/tcal/sz_$m.log 2>&1 || exit 1
  echo "== probe $m"; tail -2 gpurun_out/tcal/sz_$m.log; summ gpurun_out/tcal/sz_$m
done
for cfg in ${CFGS:-2 3 4}; do
  timeout -s KILL 200 rocprofv3 --pmc $CTRS --output-format csv -d $PWD/gpurun_out/tcal/szc$cfg -o p -- python3 $PWD/bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra --no-scale --no-strong > gpurun_out/tcal/szc$cfg.log 2>&1 || exit 1
  echo "== classify config $cfg"; summ gpurun_out/tcal/szc$cfg | grep -E "classify|scan|scatter"
done
