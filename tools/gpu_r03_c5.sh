#!/bin/bash
# r03: config 5 bench (two-level BVH, 4K 16 spp D6) with its CPU cross-checks
set -u
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
timeout -k 10 1000 python bench.py --config 5 --steps 3 --warmup 6 > gpurun_out/ev/bench5.log 2>&1
rc=$?; echo "bench5 rc=$rc"; grep '^{' gpurun_out/ev/bench5.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['cpu_baseline'], d['timed_frame_bit_exact'], d['config']['accel'], d['config']['pipeline'], d['instance_update_ms'], d['roofline']['bound'], d['roofline']['frac'])"
