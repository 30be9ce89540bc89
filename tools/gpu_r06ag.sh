set -u
O=gpurun_out/r06ag; mkdir -p $O
LIBS="default build/lib_tb64/libpupil_pt.so build/lib_tb256/libpupil_pt.so build/lib_sb128/libpupil_pt.so build/lib_sb512/libpupil_pt.so" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-120 $O/ab4.txt; exit $rc
