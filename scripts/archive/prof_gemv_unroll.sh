#!/bin/bash
set -u
mkdir -p gpurun_out/unroll
export TMPDIR=/tmp
for u in 8 4; do
  rm -rf /tmp/prof_u$u
  DLI_GEMV_UNROLL=$u timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_u$u -o run -- python3 bench.py --fp8 --batch-per-mb 1 --steps 8 --warmup 2 --json-out gpurun_out/unroll/prof_u$u.json > gpurun_out/unroll/prof_u$u.log 2>&1 || exit $?
  f=$(find /tmp/prof_u$u -name "*kernel_trace.csv" | head -1)
  python3 scripts/analyze_trace.py "$f" --steps 6 > gpurun_out/unroll/prof_u${u}_breakdown.txt || exit $?
  head -12 gpurun_out/unroll/prof_u${u}_breakdown.txt
done
