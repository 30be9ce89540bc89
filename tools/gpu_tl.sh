# config 4 (flat) and config 5 (flat vs two-level) bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/b4.log 2>&1 || exit 1
tail -n1 gpurun_out/b4.log | cut -c1-250
for a in ${ACCELS:-flat two_level}; do
  PUPIL_ACCEL=$a timeout -k 10 300 python bench.py --config 5 --cpu-baseline 0 --steps 3 --warmup 1 > gpurun_out/b5_$a.log 2>&1 || exit 1
  echo "config5 $a"; tail -n1 gpurun_out/b5_$a.log | cut -c1-250
done
