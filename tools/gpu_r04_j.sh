#!/bin/bash
# r04: SIMD-efficiency diagnostics of the persistent traversal on config 4 (PUPIL_TRACE_DIAG:
# node / leaf loop wave iterations and active lanes, refills per counter frame)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04j
PUPIL_TRACE_DIAG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 2 --cpu-baseline 0 --dropin 0 > gpurun_out/r04j/diag4.log 2>&1 || { tail -5 gpurun_out/r04j/diag4.log; exit 1; }
grep "pupil\]" gpurun_out/r04j/diag4.log | head -20
