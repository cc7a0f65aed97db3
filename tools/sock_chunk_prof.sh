#!/bin/bash
# udpdk_poll_rx phase profile (the -DUDPDK_POLL_PROFILE build, tools/diag/pollprof, `make pollprof`)
# of tools/bin/bench_sock at each [gpu] poll_chunk_mb given (0 = one piece), 1 M frames of the
# sizes in SOCK_SIZES (default 1500 and IMIX) over 1024 sockets, the sequential poll + recvfrom
# reps only (BENCH_SOCK_OVERLAP=1: the poller-thread arrangement too). GPU box:
#   bash tools/sock_chunk_prof.sh 0 64 32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in "$@"; do
  printf '[port0]\nmac_addr = 68:05:ca:95:f8:ec\nip_addr = 172.31.100.1\n[port0_dst]\nmac_addr = 68:05:ca:95:fa:64\n[gpu]\ndevice = 0\nmax_frames = 1048576\nmax_lanes = 1024\npoll_chunk_mb = %s\n' "$mb" > gpurun_out/sockc.ini
  for fb in ${SOCK_SIZES:-1500 0}; do
    echo "== poll_chunk_mb $mb frame_bytes $fb"
    BENCH_SOCK_OVERLAP=${BENCH_SOCK_OVERLAP:-0} LD_LIBRARY_PATH=$PWD/tools/diag/pollprof timeout -k 10 300 ./tools/bin/bench_sock gpurun_out/sockc.ini 1048576 $fb 1024 3 2>&1 || exit 4
  done
done
