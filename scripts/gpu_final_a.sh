#!/bin/bash
# Round-end validation A on one MI355X: every GPU test, smoke(), rocprofv3 decode breakdowns of
# the default and fp8 benches, PMC passes over the decode kernels.  Chained: a failure ends it.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_all.log 2>&1 || { tail -30 gpurun_out/gpu_tests_all.log; exit 1; }
tail -2 gpurun_out/gpu_tests_all.log
timeout -k 10 300 python3 -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/prof_default.sh > gpurun_out/prof_default.out 2>&1 || { tail -20 gpurun_out/prof_default.out; exit 1; }
head -16 gpurun_out/prof_bf16_breakdown.txt
bash scripts/pmc_decode.sh > gpurun_out/pmc.out 2>&1 || { tail -20 gpurun_out/pmc.out; exit 1; }
cat gpurun_out/pmc_decode_kernels.txt | head -30
