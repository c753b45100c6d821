#!/bin/bash
# rocprofv3 whole-step breakdown of the fp8 batch-1 decode (Llama-3-70B, one GPU)
set -u
mkdir -p gpurun_out/b1p
export TMPDIR=/tmp
rm -rf /tmp/prof_b1p
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_b1p -o run -- python3 bench.py --fp8 --batch-per-mb 1 --steps 8 --warmup 2 --json-out gpurun_out/b1p/fp8_b1.json > gpurun_out/b1p/fp8_b1.log 2>&1 || exit $?
f=$(find /tmp/prof_b1p -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py "$f" --steps 6 > gpurun_out/b1p/fp8_b1_breakdown.txt || exit $?
head -12 gpurun_out/b1p/fp8_b1_breakdown.txt
