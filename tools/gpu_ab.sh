#!/bin/bash
# Same-box A/B of library variants (tools/ab.py) on one bench shape: LIBS, BENCH, REPS, LINE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
if [ -n "$LINE" ]; then
  timeout -k 10 1000 python tools/ab.py --libs "$LIBS" --line "$LINE" --reps ${REPS:-3}
else
  timeout -k 10 1000 python tools/ab.py --libs "$LIBS" --bench "${BENCH:-}" --reps ${REPS:-3}
fi
