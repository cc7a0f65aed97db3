cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py tests/test_gpu_sock_path.py tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > gpurun_out/reasm.log 2>&1; rc=$?; tail -3 gpurun_out/reasm.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/reasm.log | head -40; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f2 -o f2 -- python3 tools/f2_bench.py reasm > gpurun_out/f2prof.log 2>&1 || exit 2
grep mdgram gpurun_out/f2prof.log
TESTS=tests/test_gpu_tx.py bash tools/ab/lines.sh tx
TESTS=tests/test_gpu_gather.py bash tools/ab/lines.sh gl
