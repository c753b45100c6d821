#!/bin/bash
# A/B of the LLM.int8 outlier weight gather: transposed copy (DLI_INT8_WT=1) vs row-major.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q -k "int8" --timeout 120 --timeout-method thread > gpurun_out/int8_tests.log 2>&1 || { tail -30 gpurun_out/int8_tests.log; exit 1; }
tail -1 gpurun_out/int8_tests.log
DLI_INT8_WT=1 timeout -k 10 400 python -u bench.py --int8 > gpurun_out/bench_int8_wt.log 2>&1 || { tail -20 gpurun_out/bench_int8_wt.log; exit 1; }
echo "WT=1: $(tail -1 gpurun_out/bench_int8_wt.log | cut -c 100-200)"
export TMPDIR=/tmp
DLI_INT8_WT=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_wt -o run -- python3 bench.py --int8 --steps 3 --warmup 1 > gpurun_out/prof_int8_wt.log 2>&1 || exit 1
f=$(find /tmp/prof_wt -name "*kernel_trace.csv" | head -1)
python3 scripts/analyze_trace.py "$f" --steps 2 > gpurun_out/prof_int8_wt_breakdown.txt || exit 1
grep -E "decode window|llm_int8" gpurun_out/prof_int8_wt_breakdown.txt
