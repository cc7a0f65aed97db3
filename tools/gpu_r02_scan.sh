# round 2: general-path (scan + scatter) check: RX GPU tests, configs 5/4 bench lines, PMC passes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_host_path.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/pytest.log; [ $rc -le 1 ] || exit $rc
for c in 5 4; do timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/b_c$c.json 2>gpurun_out/b_c$c.err || exit 3; done
if [ -n "$PMC" ]; then
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmc/WRITE_SIZE_c5" -o p -- python3 "$PWD/bench.py" --config 5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/pmc_w5.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmc/FETCH_SIZE_c5" -o p -- python3 "$PWD/bench.py" --config 5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/pmc_f5.log 2>&1 || exit 5
fi
