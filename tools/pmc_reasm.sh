#!/bin/bash
# HBM-side traffic of the reassembly kernels (tools/reasm_probe.py, copying calls), one PMC
# counter per pass: gpurun_out/pmc_reasm/<counter>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_reasm
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmc_reasm/$ctr" -o p \
    -- python3 "$PWD/tools/reasm_probe.py" > "gpurun_out/pmc_reasm/$ctr.log" 2>&1 || exit 1
done
