#!/bin/bash
# rocprofv3 kernel trace of the default bench (bf16, 512 sequences): per-kernel decode-step breakdown
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/prof_bf16
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bf16 -o run -- python3 bench.py --steps 5 --warmup 2 --json-out gpurun_out/prof_bf16_bench.json > gpurun_out/prof_bf16.log 2>&1 || exit $?
f=$(find /tmp/prof_bf16 -name "*kernel_trace.csv" | head -1)
s=$(find /tmp/prof_bf16 -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/prof_bf16_kernel_stats.csv
python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_bf16_breakdown.txt || exit $?
head -16 gpurun_out/prof_bf16_breakdown.txt
