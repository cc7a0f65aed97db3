#!/bin/bash
# Round-6 closing pass on the final tree: full GPU suite, smoke, the driver's bench commands
# (--steps 20 and the default) and kernel stats of the interleaved-flow reassembly line
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/rm && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rm/t.log 2>&1; rc=$?; tail -3 gpurun_out/rm/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rm/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/rm/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/rm/b20.json 2> gpurun_out/rm/b20.err || exit $?
tail -c 400 gpurun_out/rm/b20.json; echo
timeout -k 10 500 python bench.py > gpurun_out/rm/bfull.json 2> gpurun_out/rm/bfull.err || exit $?
tail -c 400 gpurun_out/rm/bfull.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/rm/x" -o rx -- python3 "$PWD/tools/reasmx_main.py" > gpurun_out/rm/x.log 2>&1 || exit 1
tail -1 gpurun_out/rm/x.log
