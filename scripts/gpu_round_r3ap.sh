# Round-3 GPU round AP: fp8-weight GEMV for 1-2 row decode - numerics, engine fp8 tests, batch-1 benches
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny" \
    > gpurun_out/ap_tests.log 2>&1 || { tail -40 gpurun_out/ap_tests.log; exit 1; }
tail -2 gpurun_out/ap_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "fp8" \
    > gpurun_out/ap_engine.log 2>&1 || { tail -40 gpurun_out/ap_engine.log; exit 1; }
tail -2 gpurun_out/ap_engine.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 900 python -u bench.py "$@" --json-out gpurun_out/results/$name.json > gpurun_out/results/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/results/$name.log; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/results/$name.json'));print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step p50', d['p50_token_latency_ms'])")"
}
run fp8_b1 --fp8 --batch-per-mb 1 --steps 20
run llama31_70b_fp8_fp8kv_b1_ctx127k --model llama-3.1-70b --fp8 --kv-fp8 --batch-per-mb 1 --prompt-len 130048 --steps 10 --warmup 3
