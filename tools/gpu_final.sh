# Round-end evidence on one box: smoke, every GPU test, the driver-shaped (20 steps) and default bench lines, rocprofv3 kernel
# stats (configs 2, 3 and 5, one call at a time), PMC traffic passes (configs 1-5). Each step has its
# own time limit; the first failure ends the script.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step smoke; timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
step pytest; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step bench20; timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20.json 2> gpurun_out/bench_20.err || { tail gpurun_out/bench_20.err; exit 1; }
step bench; timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail gpurun_out/bench_full.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'd1', d['depth1']['gpu_us_per_step'], 'k', d['kernel_us'], 'frac', d['roofline']['frac'])
print('scale', d['scale']['value'], 'strong', d['strong']['value'], 'cpu', d['cpu_baseline']['value'])"
step prof2; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o rx -- python3 "$PWD/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1 > gpurun_out/prof.log 2>&1 || { tail gpurun_out/prof.log; exit 1; }
step prof3; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof3" -o rx -- python3 "$PWD/bench.py" --config 3 --steps 30 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1 > gpurun_out/prof3.log 2>&1 || { tail gpurun_out/prof3.log; exit 1; }
step prof5; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof5" -o rx -- python3 "$PWD/bench.py" --config 5 --steps 50 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1 > gpurun_out/prof5.log 2>&1 || { tail gpurun_out/prof5.log; exit 1; }
step profreasm; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/profr" -o rx -- python3 "$PWD/tools/ab.py" --_line reasmip > gpurun_out/profr.log 2>&1 || { tail gpurun_out/profr.log; exit 1; }
step pmc; PMC_CONFIGS="1 2 3 4 5" bash tools/pmc_traffic.sh || exit 1
step done
