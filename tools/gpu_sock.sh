# socket-path GPU check: all -m gpu tests, then the reference-API path end to end (bench_sock)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
printf '[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n[gpu]\ndevice = 0\nmax_frames = 1048576\nmax_lanes = 1024\n' > gpurun_out/sock.ini
for spec in "1048576 64 1024 5" "1048576 0 1024 3" "1048576 1500 1024 3"; do
  timeout -k 10 300 ./tools/bin/bench_sock gpurun_out/sock.ini $spec >> gpurun_out/bench_sock.jsonl || exit 4
done
cat gpurun_out/bench_sock.jsonl
