cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tx.py tests/test_gpu_sock_path.py tests/test_gpu_span.py > gpurun_out/r6b/t.log 2>&1 || { tail -30 gpurun_out/r6b/t.log; exit 1; }
tail -2 gpurun_out/r6b/t.log
LIBS="r6head,base" LINE=tx REPS=3 bash tools/gpu_ab.sh > gpurun_out/r6b/ab_tx.log 2>&1; cat gpurun_out/r6b/ab_tx.log
LIBS="base,noprio" SHAPES="--steps 20 --warmup 5;--config 4 --steps 50 --warmup 5 --no-scale;--config 1 --steps 50 --warmup 5 --no-scale" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6b/ab_prio.log 2>&1; cat gpurun_out/r6b/ab_prio.log
