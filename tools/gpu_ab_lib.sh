# A/B of two builds of libpupil_pt.so on one box: A = pupiloptixlab_amd/lib (default),
# B = $B_LIB (default build/ab/libpupil_pt.so); alternating config-4 bench runs.
set -u
mkdir -p gpurun_out
B=${B_LIB:-build/ab/libpupil_pt.so}
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 10 > gpurun_out/abA$i.log 2>&1 || exit 1
  echo "A $(tail -n1 gpurun_out/abA$i.log | grep -o '"ms_per_step": [0-9.]*')"
  PUPIL_LIB=$B timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 10 > gpurun_out/abB$i.log 2>&1 || exit 1
  echo "B $(tail -n1 gpurun_out/abB$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
