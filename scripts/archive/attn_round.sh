#!/bin/bash
# attention round: attention / fp8 GPU tests, then the bf16-vs-fp8 KV decode probe
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernel_canaries_gpu.py tests/test_engine_gpu.py -m gpu -x -q -k "attn or fp8" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/attn_fp8kv_probe.py > gpurun_out/attn_probe.log 2>&1 || exit $?
python -c "
import json
for r in json.load(open('gpurun_out/attn_fp8kv_probe.json')): print(r)"
