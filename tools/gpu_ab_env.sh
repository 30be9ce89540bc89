#!/bin/bash
# GPU parity tests, then the bench once per environment setting (A/B).
# VARIANTS: space-separated "NAME=VALUE[,NAME2=VALUE2]" (use NONE for the defaults); BENCH_ARGS extra bench flags.
set -u
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
  [ "$rc" -eq 0 ] || exit $rc
fi
for v in ${VARIANTS:-NONE}; do
  tag=${v//=/_}
  if [ "$v" = "NONE" ]; then envs=""; else envs="${v//,/ }"; fi
  env $envs timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/ab_$tag.log 2>&1
  rc=$?; [ "$rc" -eq 0 ] || { echo "bench $v rc=$rc"; tail -n 5 gpurun_out/ab_$tag.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); c=d['config']; print('$v', d['value'], d['ms_per_step'], c['stage_ms_per_frame'], d['roofline']['frac'], d['roofline']['ms_per_launch'])"
done
if [ "${SHARD:-0}" = "1" ]; then
  timeout -k 10 300 python tools/shard_probe.py > gpurun_out/shard.log 2>&1 || exit 1
  cut -c1-120 gpurun_out/shard.log | grep world
fi
