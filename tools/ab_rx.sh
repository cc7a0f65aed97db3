# RX parity tests on the in-tree library, then a same-box A/B of bench.py (config from BENCH)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_rx.py tests/test_gpu_golden.py tests/test_gpu_host_path.py tests/test_gpu_multi_device.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rx.log 2>&1; rc=$?; tail -3 gpurun_out/t_rx.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab.py --libs ${LIBS:-old,base} --bench "${BENCH:-}" --reps ${REPS:-3}
