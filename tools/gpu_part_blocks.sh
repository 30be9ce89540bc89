set -u
mkdir -p gpurun_out
for b in 2048 512 256 2048 512 256; do
  PUPIL_PART_BLOCKS=$b timeout -k 10 200 python tools/shard_probe.py --frames 8 --worlds 1 8 > gpurun_out/pb$b.log 2>&1 || exit 1
  echo "blocks $b: $(grep -o '"world": [0-9]*, "ms_max": [0-9.]*' gpurun_out/pb$b.log | tr '\n' ' ')"
done
