#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the reassembly bench line
# (tools/ab/reasm.py): FETCH_SIZE, WRITE_SIZE, TA busy. Output: gpurun_out/pmcr/<pass>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcr
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/gpurun_out/pmcr/p$i" -o p \
    -- python3 "$PWD/tools/ab/reasm.py" > "gpurun_out/pmcr/p$i.log" 2>&1 || exit 1
done
