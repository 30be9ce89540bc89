#!/bin/bash
# r04 PMC evidence: config 4 on the production build and on the fused (if-if) traversal build
# (build/ab_fused, PUPIL_TRAVERSAL=fused), then config 5 on the production build.  Each
# gpu_pmc.sh call runs its counter groups as separate rocprofv3 passes (kernel trace only).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
mkdir -p $O
run() {  # <tag> <config> [env...]
  local tag=$1 cfg=$2; shift 2
  env "$@" CONFIG=$cfg PUPIL_ROUND=r04 bash $R/tools/gpu_pmc.sh > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -20 $O/$tag.log; exit 1; }
  cd $R
  mv gpurun_out/pmc_summary.txt $O/${tag}_summary.txt
  mv gpurun_out/pmc_config$cfg.json $O/${tag}_pmc_config$cfg.json
  rm -rf gpurun_out/pmc
  echo "$tag ok"
}
run c4 4 PUPIL_NOP=1
run c4_fused 4 PUPIL_LIB=$R/build/ab_fused/libpupil_pt.so PUPIL_TRAVERSAL=fused \
  "PMC_KERNELS=k_trace4f<0, false, false>|k_trace4f<3, false, false>|k_trace4f<4, false, false>"
run c5 5 PUPIL_NOP=1
