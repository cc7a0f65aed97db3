#!/bin/bash
# Diagnostic: bench.py kernel durations for experiment builds (tools/mkvar.sh -> tools/diag/lib_<v>.so).
# usage: VARS="a b" CFG=2 bash tools/var_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS}; do
  lib=$PWD/tools/diag/lib_$v.so; [ "$v" = base ] && lib=$PWD/udpdk_amd/libudpdk_amd.so
  if [ -n "$TEST" ]; then
    UDPDK_LIB_OVERRIDE=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/var_test_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/var_test_$v.log; exit 1; }
  fi
  UDPDK_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --config ${CFG:-2} --steps 100 --warmup 10 \
    --no-cpu-baseline --no-extra --pipeline 1 > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/var_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/var_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_us"], d["roofline"]["frac"])')"
done
