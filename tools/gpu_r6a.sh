set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_span.py > gpurun_out/r6a/t_span.log 2>&1 || { tail -30 gpurun_out/r6a/t_span.log; exit 1; }
tail -3 gpurun_out/r6a/t_span.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_forms.py tests/test_gpu_rx.py > gpurun_out/r6a/t_rx.log 2>&1 || { tail -30 gpurun_out/r6a/t_rx.log; exit 1; }
tail -3 gpurun_out/r6a/t_rx.log
for c in 3 4 1; do timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong > gpurun_out/r6a/b$c.log 2>&1 || exit 1; done
PMC_CONFIGS="3 4 1" bash tools/pmc_traffic.sh && python tools/pmc_parse.py > gpurun_out/r6a/pmc.txt
