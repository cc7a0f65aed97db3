#!/bin/bash
# A/B of rx_classify builds in the classify_probe harness (1 M x 64 B, one port): each binary in
# tools/bin/classify_probe_* at 1 and 3 streams, classify alone and with the compaction, 3 runs.
# A binary whose name contains "512" runs 512-frame tiles (TILE=512).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for b in tools/bin/classify_probe_*; do
    case "$b" in *512*) T=512;; *) T=1024;; esac
    for s in 1 3; do
      timeout -k 5 60 env TILE=$T STREAMS=$s "$b" || exit $?
      timeout -k 5 60 env TILE=$T STREAMS=$s COMPACT=1 "$b" || exit $?
    done
    echo "   ^ $b"
  done
done
