#!/bin/bash
# MX attention output for the fp8 O projection: kernel + engine GPU tests, then bench --fp8 --kv-fp8
# and --fp8 with DLI_FP8_MX_ATTN=1 (default) vs 0, alternating on one box
set -o pipefail
mkdir -p gpurun_out/mxattn
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "mx_output or fp8 or attn_decode" -x -v --timeout 120 --timeout-method thread > gpurun_out/mxattn/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/mxattn/tests.log; exit 1; }
tail -1 gpurun_out/mxattn/tests.log
for i in 1 2; do
  for m in 1 0; do
    DLI_FP8_MX_ATTN=$m timeout -k 10 400 python -u bench.py --fp8 --kv-fp8 --json-out gpurun_out/mxattn/kv_m${m}_$i.json > gpurun_out/mxattn/kv_m${m}_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/mxattn/kv_m${m}_$i.log; exit 1; }
    echo "fp8+fp8kv mx_attn=$m run $i: $(python -c "import json;d=json.load(open('gpurun_out/mxattn/kv_m${m}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for m in 1 0; do
  DLI_FP8_MX_ATTN=$m timeout -k 10 400 python -u bench.py --fp8 --json-out gpurun_out/mxattn/w_m${m}.json > gpurun_out/mxattn/w_m${m}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/mxattn/w_m${m}.log; exit 1; }
  echo "fp8 mx_attn=$m: $(python -c "import json;d=json.load(open('gpurun_out/mxattn/w_m${m}.json'));print(d['value'], d['ms_per_step'])")"
done
