#!/bin/bash
# reference-API path phase profile: tools/bin/bench_sock against the -DUDPDK_POLL_PROFILE build
# (tools/diag/pollprof/libudpdk_amd.so via LD_LIBRARY_PATH, which the binary's RUNPATH yields to)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
printf '[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n[gpu]\ndevice = 0\nmax_frames = 1048576\nmax_lanes = 1024\n' > gpurun_out/sock.ini
for spec in "1048576 64 1024 5" "1048576 0 1024 3" "1048576 1500 1024 3"; do
  LD_LIBRARY_PATH=$PWD/tools/diag/pollprof timeout -k 10 300 ./tools/bin/bench_sock gpurun_out/sock.ini $spec 2>&1 || exit 4
done
