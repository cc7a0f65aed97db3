#!/bin/bash
# reasm_scan: reassembly parity, then a same-box A/B of both reassembly lines and kernel stats
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rd gpurun_out/rk && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py tests/test_gpu_golden.py tests/test_gpu_multi_device.py tests/test_gpu_sock_path.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rd/t.log 2>&1; rc=$?; tail -3 gpurun_out/rd/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py --libs old,base --line reasmip --reps 3 || exit $?
timeout -k 10 400 python tools/ab.py --libs old,base --line reasm --reps 2 || exit $?
LIBS="${KLIBS:-old base}" bash tools/gpu_r6k.sh
