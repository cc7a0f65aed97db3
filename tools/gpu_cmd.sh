export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UDPDK_LIB_OVERRIDE=$PWD/tools/var/vlu2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_rx_forms.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_vlu2.log 2>&1; rc=$?; tail -2 gpurun_out/t_vlu2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py --libs base,vlu,vlu2 --bench "--steps 20" --reps 3 || exit 1
CFGS="1 3 4 5" timeout -k 10 300 python tools/ab.py --libs base,vlu2 --line cfg --reps 1 --timeout 200 || exit 1
for e in "UDPDK_RX_NO_INLINE=1" "UDPDK_RX_FUSE=0"; do
  echo "== $e"; env $e timeout -k 10 300 python tools/ab.py --libs base --bench "--steps 20" --reps 2 || exit 1
done
