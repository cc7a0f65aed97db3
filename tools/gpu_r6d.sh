cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d/t.log 2>&1 || { tail -30 gpurun_out/r6d/t.log; exit 1; }
tail -2 gpurun_out/r6d/t.log
LIBS="base,base@UDPDK_RX_HIST_CAP=4194304,base@UDPDK_RX_HIST_CAP=8388608" SHAPES="--config 5 --steps 20 --warmup 5 --no-scale" REPS=3 bash tools/gpu_ab_multi.sh > gpurun_out/r6d/ab_cap.log 2>&1; cat gpurun_out/r6d/ab_cap.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6d/bench.json 2> gpurun_out/r6d/bench.err || { tail -5 gpurun_out/r6d/bench.err; exit 1; }
tail -c 600 gpurun_out/r6d/bench.json
