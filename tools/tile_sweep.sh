# single-lane tile size sweep (diagnostic override UDPDK_ONE_LANE_TILE)
for T in 1024 2048 4096; do
  for cfg in 2 3; do
    UDPDK_ONE_LANE_TILE=$T timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --config $cfg --steps 100 > gpurun_out/tile_${T}_c$cfg.log 2>&1 || exit 1
  done
done
