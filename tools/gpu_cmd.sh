export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 0 1; do
for e in "X=1" "UDPDK_RX_NO_INLINE=1" "UDPDK_RX_FUSE=0" "UDPDK_RX_TAILG=2" "UDPDK_RX_FUSE=0 UDPDK_RX_TAILG=2"; do
  echo "== $e"; env $e timeout -k 10 300 python tools/ab.py --libs base,vlu --bench "--steps 20" --reps 1 || exit 1
done; done
