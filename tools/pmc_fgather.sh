#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of rx_gather and tx_build (bench lines of tools/ab/gl.py and
# tools/ab/tx.py), one counter per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcg
for w in gl tx; do for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmcg/${w}_${ctr}" -o p \
    -- python3 "$PWD/tools/ab/$w.py" > "gpurun_out/pmcg/${w}_${ctr}.log" 2>&1 || exit 1
done; done
