#!/bin/bash
# rx_compact1 vs rx_compact1w (TPB consecutive tiles per workgroup) after rx_classify in the
# classify_probe harness (1 M x 64 B, one port), 1 and 3 streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for s in 1 3; do
    timeout -k 5 60 env STREAMS=$s tools/bin/classify_probe || exit $?
    for t in 0 2 4 8 16; do
      if [ $t = 0 ]; then timeout -k 5 60 env STREAMS=$s COMPACT=1 tools/bin/classify_probe || exit $?
      else timeout -k 5 60 env STREAMS=$s COMPACT=1 TPB=$t tools/bin/classify_probe | sed "s/\$/ TPB=$t/" || exit $?; fi
    done
  done
done
