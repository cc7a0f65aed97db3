#!/bin/bash
# A/B of two library builds (tools/ab/old.so, new.so) on the reassembly path: the GPU reassembly
# and host-path parity tests on the new build, then the bench's reassembly line alternately, 3x.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
UDPDK_LIB_OVERRIDE=tools/ab/new.so timeout -k 10 400 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py tests/test_gpu_tx.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -20 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for i in 1 2 3; do for v in old new; do
  UDPDK_LIB_OVERRIDE=tools/ab/$v.so timeout -k 10 200 python tools/ab/reasm.py > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_$v.log)"
done; done
