# A/B/C/... of several builds of libpupil_pt.so on one box: $LIBS = space-separated
# name=path pairs; config-4 bench runs alternate over the builds, $ROUNDS rounds.
set -u
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for nv in $LIBS; do
    n=${nv%%=*}; lib=${nv#*=}
    PUPIL_LIB=$lib timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 10 > gpurun_out/ab_$n$r.log 2>&1 || exit 1
    echo "$n $(tail -n1 gpurun_out/ab_$n$r.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
