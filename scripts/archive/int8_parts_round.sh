#!/bin/bash
# 8-bit bf16 split-K partials: int8 / fp8 / norm GPU tests, then bench.py --int8 with
# DLI_FP8_BF16_PARTS=1 (default) vs 0, alternating on one box
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "int8 or fp8 or splitk or partials or norm" --timeout 120 --timeout-method thread > gpurun_out/int8p_tests.log 2>&1
rc=$?; tail -2 gpurun_out/int8p_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  DLI_FP8_BF16_PARTS=$v timeout -k 10 600 python bench.py --int8 --steps 10 --warmup 3 --json-out gpurun_out/int8p_$v.json > gpurun_out/int8p_bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/int8p_$v.json')); print('int8 parts_bf16=$v', d['value'], d['ms_per_step'])"
done
