set -u
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 60 ./build/ubench_overlap 200000 64 > $O/overlap.txt 2>&1 || { cat $O/overlap.txt; exit 1; }
timeout -k 10 60 ./build/ubench_overlap 200000 8 >> $O/overlap.txt 2>&1 || { cat $O/overlap.txt; exit 1; }
cat $O/overlap.txt
