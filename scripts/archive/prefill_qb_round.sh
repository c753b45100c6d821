#!/bin/bash
# prefill attention: QB = 2 query blocks per wave vs 1 (tests for both, then the microbench A/B)
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "prefill" --timeout 120 --timeout-method thread > gpurun_out/prefill_tests.log 2>&1
rc=$?; tail -2 gpurun_out/prefill_tests.log
[ $rc -ne 0 ] && exit $rc
for qb in 1 2 1 2; do
  DLI_PREFILL_QB=$qb timeout -k 10 200 python scripts/attn_prefill_bench.py > gpurun_out/prefill_bench_qb$qb.log 2>&1 || exit $?
  echo "qb=$qb"; grep -v amdgpu gpurun_out/prefill_bench_qb$qb.log
done
