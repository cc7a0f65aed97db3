# reassembly parity tests on the in-tree library, then a same-box A/B of the reassembly line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_reasm.log 2>&1; rc=$?; tail -3 gpurun_out/t_reasm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab.py --libs ${LIBS:-old,base} --line ${LINE:-reasm} --reps ${REPS:-3}
