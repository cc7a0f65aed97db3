cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6h
UDPDK_LIB_OVERRIDE=$PWD/tools/var/b512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_span.py tests/test_gpu_rx_forms.py tests/test_gpu_rx.py > gpurun_out/r6h/t.log 2>&1 || { tail -30 gpurun_out/r6h/t.log; exit 1; }
tail -1 gpurun_out/r6h/t.log
LIBS="base,b512" SHAPES="--config 3 --steps 30 --warmup 5 --no-scale;--config 4 --steps 50 --warmup 5 --no-scale;--config 1 --steps 50 --warmup 5 --no-scale;--steps 20 --warmup 5" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6h/ab.log 2>&1; cat gpurun_out/r6h/ab.log
