#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains with --pmc) over a command.
# Usage: PMC_TAG=c5 PMC_GROUPS="A B;C D" bash tools/pmc_groups.sh <program> [args...]
# Output: gpurun_out/pmcg/<tag>_g<i>/ ; tools/pmc_kernel.py prints per-kernel means.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcg
IFS=';' read -ra GROUPS_ <<< "$PMC_GROUPS"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/gpurun_out/pmcg/${PMC_TAG}_g$i" -o p \
    -- "$@" > "gpurun_out/pmcg/${PMC_TAG}_g$i.log" 2>&1 || exit 1
done
