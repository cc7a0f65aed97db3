#!/bin/bash
# Final-tree evidence for the headline kernel: rocprofv3 kernel stats of bench.py config 2 at
# pipeline depth 1 (the bench line's own HIP-event figure beside it), then the PMC traffic passes
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ro && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/ro/c2" -o rx -- python3 "$PWD/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1 > gpurun_out/ro/c2.log 2>&1 || exit 1
grep -h rx_classify gpurun_out/ro/c2/rx_kernel_stats.csv | cut -d, -f1-4
PMC_CONFIGS="2" timeout -k 10 400 bash tools/pmc_traffic.sh || exit 1
ls gpurun_out/pmc
