#!/bin/bash
# Pipeline-utilisation counters for the bench workload (one rocprofv3 pass per counter group,
# no tracing domains with --pmc). Usage: PMC_CFG=2 PMC_GROUPS="A B;C" bash tools/pmc_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=${PMC_CFG:-2}
mkdir -p gpurun_out/pmcp
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM}"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$PWD/gpurun_out/pmcp/c${cfg}_g$i" -o p \
    -- python3 "$PWD/bench.py" --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-extra \
    > "gpurun_out/pmcp/c${cfg}_g$i.log" 2>&1 || exit 1
done
