set -u
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 60 ./build/ubench_td 2.4 256 > $O/ubench_td.txt 2>&1 || { cat $O/ubench_td.txt; exit 1; }
cat $O/ubench_td.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/$O/td_pmc -o td --output-format csv -- $GRAFT_REPO_ROOT/build/ubench_td 2.4 256 > $GRAFT_REPO_ROOT/$O/td_pmc.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/td_pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT
STEPS="suite smoke bench4" OUT=$O bash tools/gpu_session.sh || exit 1
LIBS="default default,PUPIL_SHADE_LIST=list" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh > $O/ab5_list.txt 2>&1; rc=$?; cut -c1-130 $O/ab5_list.txt; exit $rc
