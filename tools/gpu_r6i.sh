cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6i
UDPDK_RX_ALL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_forms.py tests/test_gpu_rx.py > gpurun_out/r6i/t.log 2>&1 || { tail -30 gpurun_out/r6i/t.log; exit 1; }
tail -1 gpurun_out/r6i/t.log
LIBS="base,base@UDPDK_RX_ALL=1,all5@UDPDK_RX_ALL=1" SHAPES="--steps 20 --warmup 5 --no-scale;--steps 200 --warmup 20 --no-scale" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6i/ab.log 2>&1; cat gpurun_out/r6i/ab.log
