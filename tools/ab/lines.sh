#!/bin/bash
# A/B of one kernel family: parity tests ($TESTS) on the new build, then the lines printed by
# tools/ab/$1.py ("us_per_launch" / "us_per_call") for the old and new builds, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -20 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for i in 1 2; do
  for v in old new; do
    UDPDK_LIB_OVERRIDE=tools/ab/$v.so timeout -k 10 120 python tools/ab/$1.py > gpurun_out/ab_$1_$v.log 2>&1 || { tail -5 gpurun_out/ab_$1_$v.log; exit 1; }
    echo "$v $(python -c 'import json,sys; print([(lambda d: d.get("us_per_launch", d.get("us_per_call")))(json.loads(l)) for l in open(sys.argv[1]) if l.startswith("{")])' gpurun_out/ab_$1_$v.log)"
  done
done
