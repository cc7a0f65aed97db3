export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rss.py tests/test_gpu_rx_forms.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rss.log 2>&1; rc=$?; tail -2 gpurun_out/t_rss.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py --libs old,base --line rss --reps 2 --timeout 200 || exit 1
UDPDK_LIB_OVERRIDE=$PWD/tools/var/b1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rx.py -x -q --timeout 120 --timeout-method thread -k "configs_full or mixed or single_lane_spec or edge" > gpurun_out/t_b1024.log 2>&1; tail -2 gpurun_out/t_b1024.log
timeout -k 10 300 python tools/ab.py --libs base,b512,b1024 --bench "--steps 20" --reps 2 || exit 1
timeout -k 10 300 python tools/ab.py --libs base,b512,b1024 --reps 1 || exit 1
CFGS="3 5" timeout -k 10 300 python tools/ab.py --libs base,b512,b1024 --line cfg --reps 1 --timeout 200 || exit 1
printf "[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n[gpu]\ndevice = 0\nmax_frames = 1048576\nmax_lanes = 1024\n" > gpurun_out/sock.ini
for fb in 1500 64; do timeout -k 10 200 ./tools/bin/bench_sock gpurun_out/sock.ini 1048576 $fb 1024 3 || exit 1; done
