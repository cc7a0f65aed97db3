export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 0 1; do
timeout -k 10 300 python tools/ab.py --libs old,base --bench "--steps 20" --reps 1 || exit 1
UDPDK_RX_NO_INLINE=1 timeout -k 10 300 python tools/ab.py --libs base --bench "--steps 20" --reps 1 || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || { tail -5 gpurun_out/bench_quick.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1])
print('value', d['value'], 'd1', d['depth1'], 'k', d['kernel_us'], 'frac', d['roofline']['frac'])
print('scale', d['scale']['value'], 'strong', {k: d['strong'][k] for k in ('value','ms_per_step','frames_total','rank0_gpu_us_per_step')})
"
