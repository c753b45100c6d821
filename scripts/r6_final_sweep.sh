# final-tree numbers: headline bench, long-context TTFTs (bf16 32k / 127k, fp8 + fp8 KV 127k,
# Mistral-7B 32k)
set -u
out=gpurun_out/r6fin
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" --json-out $out/$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  python -c "import json; d=json.load(open('$out/$name.json')); print('$name', 'prefill_s', d['prefill_s'], 'tok/s', d['value'], 'ms/step', d['ms_per_step'])"
}
run headline
run llama31_70b_32k --model llama-3.1-70b --batch-per-mb 1 --prompt-len 32768 --steps 5 --warmup 2
run llama31_70b_127k --model llama-3.1-70b --batch-per-mb 1 --prompt-len 130048 --steps 5 --warmup 2
run llama31_70b_fp8_fp8kv_127k --model llama-3.1-70b --fp8 --kv-fp8 --batch-per-mb 1 --prompt-len 130048 --steps 5 --warmup 2
run mistral_7b_32k --model mistral-7b --batch-per-mb 1 --prompt-len 32768 --steps 5 --warmup 2
