#!/bin/bash
# fp8 check: quant / fp8 GPU tests, bench.py --fp8 twice, rocprofv3 decode breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "fp8 or quant or int8" --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fp8_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 600 python bench.py --fp8 --steps 10 --warmup 3 --json-out gpurun_out/fp8_run$i.json > gpurun_out/fp8_run$i.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/fp8_run$i.json')); print('fp8 run $i', d['value'], d['ms_per_step'])"
done
rm -rf /tmp/prof_fp8
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fp8 -o run -- python3 bench.py --fp8 --steps 5 --warmup 2 > gpurun_out/prof_fp8.log 2>&1 || exit $?
f=$(find /tmp/prof_fp8 -name "*kernel_trace.csv" | head -1)
s=$(find /tmp/prof_fp8 -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/prof_fp8_kernel_stats.csv
python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_fp8_breakdown.txt || exit $?
head -14 gpurun_out/prof_fp8_breakdown.txt
