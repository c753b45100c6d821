#!/bin/bash
# batch-1 iteration: GEMV / norm numerics tests, GEMV stream rates, batch-1 benches, short-context
# decode attention split sweep.  Each GPU step has its own time limit; the steps are chained.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "skinny or gemv or norm or rope or 8bit" > gpurun_out/b1_tests.log 2>&1 || { tail -30 gpurun_out/b1_tests.log; exit 1; }
tail -2 gpurun_out/b1_tests.log
timeout -k 10 300 python3 -u scripts/gemv_bw.py > gpurun_out/gemv_bw.txt 2>&1 || { tail -5 gpurun_out/gemv_bw.txt; exit 1; }
grep stream gpurun_out/gemv_bw.txt
bash scripts/b1_sweep.sh || exit 1
timeout -k 10 300 python3 -u scripts/attn_bench.py --cases=1x600 --short > gpurun_out/attn_short.txt 2>&1 || { tail -5 gpurun_out/attn_short.txt; exit 1; }
cat gpurun_out/attn_short.txt
