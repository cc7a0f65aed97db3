#!/bin/bash
# Quick GPU iteration: parity tests, then kernel durations for the given configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-2 3}; do
  timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-extra --pipeline 1 > gpurun_out/q_$cfg.log 2>&1 || { tail -5 gpurun_out/q_$cfg.log; exit 1; }
  echo "cfg$cfg $(tail -1 gpurun_out/q_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_us"], d["roofline"]["frac"])')"
done
