#!/bin/bash
# fp8 MX round: MX GEMM / engine tests, then bench.py --fp8 with the MX down projection (default)
# vs the bf16 h + per-row quantiser path (DLI_FP8_MX=0), alternating on one box.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -m gpu -x -q -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/mx_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mx_tests.log
[ $rc -ne 0 ] && exit $rc
for mx in 1 0 1 0; do
  DLI_FP8_MX=$mx timeout -k 10 600 python bench.py --fp8 --steps 10 --warmup 3 --json-out gpurun_out/mx_$mx.json > gpurun_out/mx_bench_$mx.log 2>&1 || exit $?
  python -c "import json; d=json.load(open('gpurun_out/mx_$mx.json')); print('mx=$mx', d['value'], d['ms_per_step'])"
done
