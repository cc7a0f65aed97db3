#!/bin/bash
# A/B of rx_classify builds in the classify_probe harness (1 M x 64 B, one port): each binary in
# tools/bin/classify_probe_* at 1 and 3 streams, classify alone and with the compaction, 3 runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for b in tools/bin/classify_probe_*; do
    for s in 1 3; do
      timeout -k 5 60 env STREAMS=$s "$b" || exit $?
      timeout -k 5 60 env STREAMS=$s COMPACT=1 "$b" || exit $?
    done
    echo "   ^ $b"
  done
done
