#!/bin/bash
# Build the product library of another git revision into tools/var/<name>.so for same-box A/Bs
# (tools/ab.py --libs base,<name>; tools/gpu_pmc.sh OLD=<name>), without touching this tree:
#   tools/build_rev.sh e20aceb r04      # round 4's final library -> tools/var/r04.so
# tools/var/ is git-ignored; delete its libraries after the A/B (every gpurun call ships them).
set -euo pipefail
REV=$1 NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
trap 'git -C "$ROOT" worktree remove --force "$TMP" >/dev/null 2>&1 || true; rm -rf "$TMP"' EXIT
git -C "$ROOT" worktree add --detach "$TMP" "$REV" >/dev/null
make -C "$TMP" -j8 udpdk_amd/libudpdk_amd.so >/dev/null
mkdir -p "$ROOT/tools/var"
cp "$TMP/udpdk_amd/libudpdk_amd.so" "$ROOT/tools/var/$NAME.so"
echo "tools/var/$NAME.so <- $(git -C "$ROOT" rev-parse --short "$REV")"
