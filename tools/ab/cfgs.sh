#!/bin/bash
# A/B of two library builds (tools/ab/old.so, new.so) on the same box: RX parity tests on the
# new build, then the bench's headline line (pipelined and depth 1) for configs $CFGS, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
UDPDK_LIB_OVERRIDE=tools/ab/new.so timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_rx.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -20 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for c in ${CFGS:-2}; do for i in 1 2; do for v in old new; do
  UDPDK_LIB_OVERRIDE=tools/ab/$v.so timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "c$c $v $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["gpu_us_per_step"], "d1", d["depth1"]["gpu_us_per_step"], d["kernel_us"])')"
done; done; done
