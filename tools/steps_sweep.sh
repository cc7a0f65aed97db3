#!/bin/bash
# bench value vs --steps (the timed region's fixed cost: pipeline fill/drain + closing sync), for
# the in-tree library or, with LIBS="old new", tools/ab/{old,new}.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in ${STEPS_LIST:-5 10 20 40 200}; do for v in ${LIBS:-tree}; do
  [ "$v" = tree ] && unset UDPDK_LIB_OVERRIDE || export UDPDK_LIB_OVERRIDE=tools/ab/$v.so
  timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline --no-extra $BENCH_ARGS > gpurun_out/sw_$s.log 2>&1 || { tail -5 gpurun_out/sw_$s.log; exit 1; }
  echo "steps $s $v $(tail -1 gpurun_out/sw_$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["gpu_us_per_step"])')"
done; done
