set -u
O=gpurun_out/r06ac; mkdir -p $O
LIBS="default build/lib_sd6/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-110 $O/ab4.txt; exit $rc
