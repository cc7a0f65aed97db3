export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 ./tools/bin/stream_probe > gpurun_out/stream_probe.log 2>&1; cat gpurun_out/stream_probe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || { tail -5 gpurun_out/bench_quick.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1])
print('value', d['value'], 'd1', d['depth1'], 'k', d['kernel_us'], 'frac', d['roofline']['frac'])
print('scale', d['scale']['value'], 'strong', {k: d['strong'][k] for k in ('value','ms_per_step','frames_total','rank0_gpu_us_per_step')})
"
