# Before/after PMC passes of rx_classify at config 2 (and config 5): an earlier revision's library
# against the current one, one counter group per rocprofv3 run. Build the earlier one first:
#   tools/build_rev.sh <rev> old          # -> tools/var/old.so
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
G2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE TA_BUSY_avr"
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1"
for lib in old new; do
  if [ $lib = old ]; then export UDPDK_LIB_OVERRIDE=$PWD/tools/var/old.so; else unset UDPDK_LIB_OVERRIDE; fi
  for cfg in 2 5; do
    PMC_TAG=${lib}_c$cfg PMC_GROUPS="$G1;$G2" bash tools/pmc_groups.sh python3 $PWD/bench.py --config $cfg $B || exit 1
    echo "== $lib c$cfg"; python tools/pmc_kernel.py gpurun_out/pmcg/${lib}_c${cfg}_g*/p_counter_collection.csv | grep classify
  done
done
