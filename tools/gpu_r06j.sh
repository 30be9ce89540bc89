set -u
O=gpurun_out/r06j; mkdir -p $O
for v in default build/lib_fw3/libpupil_pt.so build/lib_fw5/libpupil_pt.so; do
  if [ $v = default ]; then E=""; else E="PUPIL_LIB=$v"; fi
  env $E timeout -k 10 300 python tools/shard_probe.py --moving 1 --worlds 8 --warmup 8 --frames 16 > $O/moving8.txt 2>&1 || { tail -5 $O/moving8.txt; exit 1; }
  echo "$v $(grep world $O/moving8.txt | cut -c1-160)"
done
PUPIL_FRAME_PATHS=3e6 timeout -k 10 300 python tools/shard_probe.py --moving 1 --worlds 1 --warmup 8 --frames 16 > $O/moving1_frame.txt 2>&1 || { tail -5 $O/moving1_frame.txt; exit 1; }
echo "N=1 moving, one-launch frame: $(grep world $O/moving1_frame.txt | cut -c1-160)"
bash tools/gpu_r06i.sh
