# A/B of the classify variants: RX parity tests under each forced variant, then configs 1/3/4
# bench lines (no side lines) per variant
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in long short; do
  UDPDK_CLS_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_gather.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { tail -20 gpurun_out/pytest_$v.log; exit 2; }
  tail -1 gpurun_out/pytest_$v.log
done
for c in ${CFGS:-1 3 4}; do for v in short long; do
  UDPDK_CLS_VARIANT=$v timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/ab_c${c}_$v.json 2>/dev/null || exit 3
  python tools/bench_summary.py gpurun_out/ab_c${c}_$v.json | sed "s/^/$v /"
done; done
