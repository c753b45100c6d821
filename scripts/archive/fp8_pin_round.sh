#!/bin/bash
# fp8 tile GEMM with its MFMA segments pinned between the phase barriers: clock stamps of the
# previous (sunk-MFMA) build vs this one on the same box, the fp8 GPU tests, then bench.py --fp8.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools_bin/gemm_stamps_old > gpurun_out/stamps_fp8_old.txt 2>&1 || exit $?
timeout -k 10 120 tools_bin/gemm_stamps_new > gpurun_out/stamps_fp8_new.txt 2>&1 || exit $?
grep -h "fp8\|bf16_gate" gpurun_out/stamps_fp8_old.txt gpurun_out/stamps_fp8_new.txt
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py -m gpu -x -q -k "fp8" --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -2 gpurun_out/fp8_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --fp8 --steps 10 --warmup 3 --json-out gpurun_out/fp8_pinned.json > gpurun_out/fp8_bench_pinned.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --fp8 --kv-fp8 --steps 10 --warmup 3 --json-out gpurun_out/fp8kv_pinned.json > gpurun_out/fp8kv_bench_pinned.log 2>&1 || exit $?
python -c "import json; [print(f, json.load(open('gpurun_out/'+f))['value']) for f in ('fp8_pinned.json', 'fp8kv_pinned.json')]"
