for T in 1024 2048 4096 8192; do
  UDPDK_FUSED_TILE=$T timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 200 > gpurun_out/tile_$T.log 2>&1 || exit 1
done
