cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pr -o r -- python3 tools/f2_bench.py reasm > gpurun_out/pr.log 2>&1

