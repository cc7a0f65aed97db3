export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py tests/test_gpu_sock_path.py tests/test_gpu_rss.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1; rc=$?; tail -2 gpurun_out/t_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py --libs old,base --line reasmip --reps 3 --timeout 200 || exit 1
timeout -k 10 300 python tools/ab.py --libs old,base --line rss --reps 1 --timeout 200 || exit 1
for d in 4 3 2; do timeout -k 10 200 python bench.py --config 5 --steps 40 --warmup 10 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline $d > gpurun_out/c5_d$d.json 2>&1 || exit 1; python -c "
import json; d=json.loads(open('gpurun_out/c5_d$d.json').read().strip().splitlines()[-1]); print('c5 depth $d', d['value'], d['gpu_us_per_step'], d['kernel_us'])"; done
