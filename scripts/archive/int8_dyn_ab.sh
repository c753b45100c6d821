#!/bin/bash
# LLM.int8: GPU tests of the outlier path, then bench --int8 with dynamic outlier chunks (default)
# vs the static 64-column gathers (DLI_INT8_DYNAMIC=0), alternating on one box
set -o pipefail
mkdir -p gpurun_out/int8dyn
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -m gpu -k "int8" -x -v --timeout 120 --timeout-method thread > gpurun_out/int8dyn/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/int8dyn/tests.log; exit 1; }
tail -2 gpurun_out/int8dyn/tests.log
for i in 1 2; do
  for d in 1 0; do
    DLI_INT8_DYNAMIC=$d timeout -k 10 400 python -u bench.py --int8 --json-out gpurun_out/int8dyn/dyn${d}_$i.json > gpurun_out/int8dyn/dyn${d}_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/int8dyn/dyn${d}_$i.log; exit 1; }
    echo "dynamic=$d run $i: $(python -c "import json;d=json.load(open('gpurun_out/int8dyn/dyn${d}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
