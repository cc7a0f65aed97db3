#!/bin/bash
# FETCH_SIZE per kernel launch for the two A/B builds (tools/ab/old.so, new.so), configs $CFGS;
# one counter per rocprofv3 pass. Output: gpurun_out/abpmc/<build>_c<config>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abpmc
for cfg in ${CFGS:-4}; do for v in old new; do
  export UDPDK_LIB_OVERRIDE=$PWD/tools/ab/$v.so
  timeout -k 10 -s KILL 120 rocprofv3 --pmc ${CTR:-FETCH_SIZE} --output-format csv -d "$PWD/gpurun_out/abpmc/${v}_c$cfg" -o p \
    -- python3 "$PWD/bench.py" --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-extra \
    > "gpurun_out/abpmc/${v}_c$cfg.log" 2>&1 || exit 1
  echo "c$cfg $v"; python3 tools/pmc_kernel.py gpurun_out/abpmc/${v}_c$cfg/*/p_counter_collection.csv 2>/dev/null | grep rx_classify || find gpurun_out/abpmc/${v}_c$cfg -name "*.csv"
done; done
