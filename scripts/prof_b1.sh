#!/bin/bash
# Whole-step rocprofv3 breakdown of batch-1 decode (Llama-3-70B, one GPU) for bf16, fp8 and LLM.int8,
# plus the default 512-sequence bench on the same box. Writes gpurun_out/b1/*.
set -u
mkdir -p gpurun_out/b1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --json-out gpurun_out/b1/default_bench.json > gpurun_out/b1/default_bench.log 2>&1 || exit $?
tail -1 gpurun_out/b1/default_bench.log
for mode in bf16 fp8 int8; do
  flag=""
  [ "$mode" = fp8 ] && flag="--fp8"
  [ "$mode" = int8 ] && flag="--int8"
  rm -rf /tmp/prof_b1_$mode
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_b1_$mode -o run -- python3 bench.py $flag --batch-per-mb 1 --steps 8 --warmup 2 --json-out gpurun_out/b1/${mode}_b1.json > gpurun_out/b1/${mode}_b1.log 2>&1 || exit $?
  f=$(find /tmp/prof_b1_$mode -name "*kernel_trace.csv" | head -1)
  s=$(find /tmp/prof_b1_$mode -name "*kernel_stats.csv" | head -1)
  cp "$s" gpurun_out/b1/${mode}_b1_kernel_stats.csv
  python3 scripts/analyze_trace.py "$f" --steps 6 > gpurun_out/b1/${mode}_b1_breakdown.txt || exit $?
  head -14 gpurun_out/b1/${mode}_b1_breakdown.txt
done
