#!/bin/bash
# PMC passes over the TX 1500 B and fragmentation lines (tools/ab/txf.py): FETCH_SIZE,
# WRITE_SIZE, TA busy. Output: gpurun_out/pmctxf/<line>_p<pass>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmctxf
for line in 1500 frag; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/gpurun_out/pmctxf/${line}_p$i" -o p \
      -- python3 "$PWD/tools/ab/txf.py" $line > "gpurun_out/pmctxf/${line}_p$i.log" 2>&1 || exit 1
  done
done
