cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tx.py > gpurun_out/r6c/t.log 2>&1 || { tail -30 gpurun_out/r6c/t.log; exit 1; }
tail -1 gpurun_out/r6c/t.log
for L in tx txfrag; do LIBS="tx1,base,tx2w4,tx4w4" LINE=$L REPS=2 bash tools/gpu_ab.sh > gpurun_out/r6c/ab_$L.log 2>&1; cat gpurun_out/r6c/ab_$L.log; done
