#!/bin/bash
# attention kernels after a compute-path change: every attention GPU test, then the prefill and
# decode microbenches
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernel_canaries_gpu.py -m gpu -x -q -k "attn" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/attn_prefill_bench.py > gpurun_out/prefill_bench.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/prefill_bench.log
timeout -k 10 200 python scripts/attn_fp8kv_probe.py > gpurun_out/attn_probe.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/attn_probe.log
