#!/bin/bash
# round-4 check B: engine tests (fused-norm GEMV path), headline + fp8 benches, PP=8 rehearsal
set -u
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/engine_tests.log 2>&1 || { tail -30 gpurun_out/r4b/engine_tests.log; exit 1; }
tail -2 gpurun_out/r4b/engine_tests.log
for cfg in "default:" "fp8:--fp8" "fp8kv:--fp8 --kv-fp8"; do
  name=${cfg%%:*}; flags=${cfg#*:}
  timeout -k 10 400 python3 -u bench.py $flags --json-out gpurun_out/r4b/bench_$name.json > gpurun_out/r4b/bench_$name.log 2>&1 || { tail -20 gpurun_out/r4b/bench_$name.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4b/bench_$name.json'));print('$name', d['value'], d['ms_per_step'])"
done
bash scripts/rehearsal_pp8_default.sh
