#!/bin/bash
# rx_classify<1, 2> (second window in flight, depth-1 calls): RX GPU tests, then same-box A/B
# (base vs UDPDK_RX_DEEP=0) at depth 1 (rocprof kernel means) and pipelined
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rl && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx_forms.py tests/test_gpu_rx.py tests/test_gpu_span.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rl/t.log 2>&1; rc=$?; tail -2 gpurun_out/rl/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python tools/ab.py --libs base,base@UDPDK_RX_DEEP=0 --bench "--config 2" --reps 3 || exit $?
for n in deep nodeep; do
  if [ $n = nodeep ]; then export UDPDK_RX_DEEP=0; else unset UDPDK_RX_DEEP; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/rl/$n" -o rx -- python3 "$PWD/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1 > gpurun_out/rl/$n.log 2>&1 || exit 1
  echo "$n $(grep -h rx_classify gpurun_out/rl/$n/rx_kernel_stats.csv | cut -d, -f1-4)"
done
