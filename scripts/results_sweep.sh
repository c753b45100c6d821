# One-GPU results sweep behind README's table (each config its own process, back to back, one box)
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" --json-out gpurun_out/results/$name.json > gpurun_out/results/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/results/$name.log; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/results/$name.json'));print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step p50', d['p50_token_latency_ms'])")"
}
# $1: "b512" (the 512-sequence rows), "small" (batch 1 / 16 rows), or nothing (all)
part=${1:-all}
if [ "$part" != small ]; then
run bf16_b512
run fp8_b512 --fp8
run fp8_fp8kv_b512 --fp8 --kv-fp8
run bf16_fp8kv_b512 --kv-fp8
run llama3_8b_bf16_b512 --model llama-3-8b
run int8_b512 --int8
fi
if [ "$part" != b512 ]; then
run bf16_b1 --batch-per-mb 1 --steps 20
run fp8_b1 --fp8 --batch-per-mb 1 --steps 20
run int8_b1 --int8 --batch-per-mb 1 --steps 20
run bf16_b1_ctx8k --batch-per-mb 1 --prompt-len 8192 --steps 20
run bf16_b16_ctx8k --batch-per-mb 16 --prompt-len 8192 --steps 10
fi
