set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w8
for W in 4 8; do
PUPIL_TRACE_DIAG=1 PUPIL_BVH_WIDTH=$W timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --dropin 0 > gpurun_out/w8/diag_$W.log 2>&1 || exit 1
echo "W=$W"; grep "\[pupil\]" gpurun_out/w8/diag_$W.log | sort | uniq | head -8
done
