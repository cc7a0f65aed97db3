# quick GPU check: RX/gather/host-path parity tests, then the bench (no CPU leg) with side lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2>gpurun_out/bench.err || exit 3
