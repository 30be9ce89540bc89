set -u
O=gpurun_out/r06ai; mkdir -p $O
LIBS="default default,PUPIL_SAH_NODE_COST=0.6 default,PUPIL_SAH_NODE_COST=1.5 default,PUPIL_SAH_NODE_COST=2.5 default,PUPIL_SAH_NODE_COST=1.5,PUPIL_SAH_LEAF=4" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-140 $O/ab4.txt; exit $rc
