cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmctx
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d "$PWD/gpurun_out/pmctx/a" -o p -- python3 "$PWD/tools/ab/tx64.py" > gpurun_out/pmctx/a.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$PWD/gpurun_out/pmctx/b" -o p -- python3 "$PWD/tools/ab/tx64.py" > gpurun_out/pmctx/b.log 2>&1
echo rc=$?
