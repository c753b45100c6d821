#!/bin/bash
# LLM.int8 kernel tests, then the --int8 bench line and its rocprofv3 breakdown.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -m gpu -x -v -k "int8" --timeout 120 --timeout-method thread > gpurun_out/int8_tests.log 2>&1 || { tail -30 gpurun_out/int8_tests.log; exit 1; }
tail -2 gpurun_out/int8_tests.log
bash scripts/archive/int8_round.sh
