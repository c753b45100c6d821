#!/bin/bash
# LLM.int8 fused-epilogue round: int8 GPU tests, then bench.py --int8 with the fused path
# (DLI_INT8_FUSED=1) vs the previous one (0) back to back on one box, then a rocprofv3 breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "int8" --timeout 120 --timeout-method thread > gpurun_out/int8_tests.log 2>&1
rc=$?; echo "int8 tests rc=$rc"; tail -2 gpurun_out/int8_tests.log
[ $rc -ne 0 ] && exit $rc
for mode in 1 0 1; do
  DLI_INT8_FUSED=$mode timeout -k 10 600 python bench.py --int8 --steps 10 --warmup 3 --json-out gpurun_out/int8_f$mode.json > gpurun_out/int8_bench_f$mode.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/int8_f$mode.json')); print('fused=$mode', d['value'], d['ms_per_step'])"
done
rm -rf /tmp/prof_int8
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_int8 -o run -- python3 bench.py --int8 --steps 5 --warmup 2 > gpurun_out/prof_int8.log 2>&1 || exit $?
f=$(find /tmp/prof_int8 -name "*kernel_trace.csv" | head -1)
s=$(find /tmp/prof_int8 -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/prof_int8_kernel_stats.csv
python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_int8_breakdown.txt || exit $?
head -16 gpurun_out/prof_int8_breakdown.txt
