#!/bin/bash
# HBM-side traffic per rx_classify launch from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no tracing domains combined with
# --pmc). Output: gpurun_out/pmc/<counter>_c<config>/ ; tools/pmc_parse.py folds them into
# profiles/traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for cfg in ${PMC_CONFIGS:-2 3}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/gpurun_out/pmc/${ctr}_c$cfg" -o p \
      -- python3 "$PWD/bench.py" --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong \
      > "gpurun_out/pmc/${ctr}_c$cfg.log" 2>&1 || exit 1
  done
done
