#!/bin/bash
# fp8 bf16 split-K partials: fp8 / quant / rope GPU tests, then bench.py --fp8 (--kv-fp8) with
# DLI_FP8_BF16_PARTS=1 (default) vs 0, alternating on one box
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or quant or rope or splitk" --timeout 120 --timeout-method thread > gpurun_out/parts_tests.log 2>&1
rc=$?; tail -2 gpurun_out/parts_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  DLI_FP8_BF16_PARTS=$v timeout -k 10 600 python bench.py --fp8 --kv-fp8 --steps 10 --warmup 3 --json-out gpurun_out/parts_$v.json > gpurun_out/parts_bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/parts_$v.json')); print('fp8kv parts_bf16=$v', d['value'], d['ms_per_step'])"
done
