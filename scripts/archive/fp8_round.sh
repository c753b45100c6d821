#!/bin/bash
# fp8 tile-path round: fp8 GPU tests, then bench.py --fp8 with the hand-written tile GEMMs on every
# projection (DLI_FP8_TILE=all) vs hipBLASLt on the K = 8192 ones (long), back to back, then a
# rocprofv3 kernel breakdown of the all-tile decode step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py -m gpu -x -q -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -2 gpurun_out/fp8_tests.log
[ $rc -ne 0 ] && exit $rc
for mode in all long all; do
  DLI_FP8_TILE=$mode timeout -k 10 600 python bench.py --fp8 --steps 10 --warmup 3 --json-out gpurun_out/fp8_$mode.json > gpurun_out/fp8_bench_$mode.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/fp8_$mode.json')); print('$mode', d['value'], d['ms_per_step'])"
done
rm -rf /tmp/prof_fp8all
DLI_FP8_TILE=all timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fp8all -o run -- python3 bench.py --fp8 --steps 5 --warmup 2 --json-out gpurun_out/prof_fp8all_bench.json > gpurun_out/prof_fp8all.log 2>&1 || exit $?
f=$(find /tmp/prof_fp8all -name "*kernel_trace.csv" | head -1)
s=$(find /tmp/prof_fp8all -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/prof_fp8all_kernel_stats.csv
python3 scripts/analyze_trace.py "$f" --steps 3 > gpurun_out/prof_fp8all_breakdown.txt || exit $?
head -16 gpurun_out/prof_fp8all_breakdown.txt
