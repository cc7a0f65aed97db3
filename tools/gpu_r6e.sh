cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx.py tests/test_gpu_rx_forms.py > gpurun_out/r6e/t.log 2>&1 || { tail -30 gpurun_out/r6e/t.log; exit 1; }
tail -1 gpurun_out/r6e/t.log
UDPDK_RX_MR=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx.py > gpurun_out/r6e/t2.log 2>&1 || { tail -30 gpurun_out/r6e/t2.log; exit 1; }
tail -1 gpurun_out/r6e/t2.log
LIBS="base,base@UDPDK_RX_MR=1" SHAPES="--config 5 --steps 20 --warmup 5 --no-scale;--config 5 --steps 200 --warmup 20 --no-scale" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6e/ab.log 2>&1; cat gpurun_out/r6e/ab.log
UDPDK_LIB_OVERRIDE=$PWD/tools/var/t512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_forms.py -k "single_lane or configs" > gpurun_out/r6e/t512.log 2>&1 || { tail -30 gpurun_out/r6e/t512.log; exit 1; }
tail -1 gpurun_out/r6e/t512.log
LIBS="base,t512" SHAPES="--steps 20 --warmup 5 --no-scale;--steps 200 --warmup 20 --no-scale" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6e/ab512.log 2>&1; cat gpurun_out/r6e/ab512.log
