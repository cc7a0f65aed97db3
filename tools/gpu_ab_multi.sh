#!/bin/bash
# Same-box A/B (tools/ab.py) of LIBS over several bench shapes, then optional GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
IFS=';' read -ra SHAPES <<< "${SHAPES:---steps 20 --warmup 5}"
for sh in "${SHAPES[@]}"; do
  echo "== $sh"
  timeout -k 10 900 python tools/ab.py --libs "$LIBS" --bench "$sh" --reps ${REPS:-3} || exit 1
done
