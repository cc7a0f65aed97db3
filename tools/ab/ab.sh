#!/bin/bash
# A/B: alternate two library builds on the same box (bench config $CFG, single-launch kernel times).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in old new; do
    UDPDK_LIB_OVERRIDE=tools/ab/$v.so timeout -k 10 120 python bench.py --config ${CFG:-2} --steps 200 --warmup 20 --no-cpu-baseline --no-extra --pipeline 1 > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
    echo "$v $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_us"], d["roofline"]["frac"])')"
  done
done
