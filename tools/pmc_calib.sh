#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on kernels with known byte counts (tools/probe/stream_probe:
# lane1 / coal1 / unal1 read exactly 64 MiB of frames (+ 4 or 6 MiB descriptors) and write 4 MiB),
# one counter per pass, no tracing domains with --pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PROBE_REPS=5
mkdir -p gpurun_out/calib
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/calib/$ctr" -o p \
    -- "$PWD/tools/probe/stream_probe" > "gpurun_out/calib/$ctr.log" 2>&1 || exit 1
done
python3 tools/pmc_kernel.py gpurun_out/calib/*/p_counter_collection.csv
