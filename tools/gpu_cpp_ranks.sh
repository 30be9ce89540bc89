#!/bin/bash
# Rehearsal of the C++ drop-in's RCCL tile gather with N ranks sharing this box's
# one GPU (both processes on device 0): if RCCL accepts the shared device, rank 0's
# gathered image must equal the single-GPU image bit for bit.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cpp_ranks
N=${N:-2}
python3 -c "
import sys; sys.path.insert(0, '.')
from pupiloptixlab_amd import scenes
scenes.cornell_xml('gpurun_out/cpp_ranks/cb.xml', 96, 72, 4)"
timeout -k 10 120 build/pupil_path_tracer gpurun_out/cpp_ranks/cb.xml 3 gpurun_out/cpp_ranks/one.pfm > gpurun_out/cpp_ranks/one.log 2>&1 || exit 1
PORT=$((20000 + RANDOM % 20000))
pids=""
for r in $(seq 0 $((N-1))); do
  RANK=$r WORLD_SIZE=$N LOCAL_RANK=0 MASTER_PORT=$PORT NCCL_DEBUG=WARN timeout -k 10 120 build/pupil_path_tracer gpurun_out/cpp_ranks/cb.xml 3 gpurun_out/cpp_ranks/multi.pfm > gpurun_out/cpp_ranks/rank$r.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
echo "ranks rc=$rc"; tail -n 3 gpurun_out/cpp_ranks/rank*.log
if [ "$rc" -ne 0 ]; then
  # RCCL refuses two ranks on one device; reaching that check means every rank found rank 0's
  # id file (same default path and nonce) and entered ncclCommInitRank together
  if grep -q "Duplicate GPU detected" gpurun_out/cpp_ranks/rank*.log; then
    echo "N=$N: id exchange completed on every rank; RCCL refuses ranks sharing this box's one GPU"
    exit 0
  fi
  exit $rc
fi
cmp gpurun_out/cpp_ranks/one.pfm gpurun_out/cpp_ranks/multi.pfm && echo "N=$N gathered image identical to 1 GPU"
