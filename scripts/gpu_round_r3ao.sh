# Round-3 GPU round AO: more long-context points on one GPU (Llama-3.1-70B)
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 900 python -u bench.py --model llama-3.1-70b "$@" --json-out gpurun_out/results/$name.json > gpurun_out/results/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/results/$name.log; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/results/$name.json'));print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step p50', d['p50_token_latency_ms'], 'prefill_s', d['prefill_s'])")"
}
run llama31_70b_fp8_fp8kv_b1_ctx127k --fp8 --kv-fp8 --batch-per-mb 1 --prompt-len 130048 --steps 10 --warmup 3
run llama31_70b_bf16_b8_ctx32k --batch-per-mb 8 --prompt-len 32768 --steps 10 --warmup 3
