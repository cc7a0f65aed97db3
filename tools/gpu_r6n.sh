#!/bin/bash
# Overlap records sorted as u32 keys when they fit: reassembly parity, same-box A/B of the
# interleaved line (prev = u64 keys), kernel stats
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rn && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_reasm.py tests/test_gpu_host_path.py tests/test_gpu_sock_path.py tests/test_gpu_golden.py tests/test_gpu_multi_device.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rn/t.log 2>&1; rc=$?; tail -3 gpurun_out/rn/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py --libs prev,base --line reasmx --reps 2 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/rn/x" -o rx -- python3 "$PWD/tools/reasmx_main.py" > gpurun_out/rn/x.log 2>&1 || exit 1
tail -1 gpurun_out/rn/x.log
