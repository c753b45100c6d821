# final-tree TTFT: Llama-3.1-70B bf16 at 32k / 127k, Mistral-7B (sliding window 4096) at 32k
set -u
out=gpurun_out/r6ttft2
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" --batch-per-mb 1 --steps 5 --warmup 2 --json-out $out/$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  python -c "import json; d=json.load(open('$out/$name.json')); print('$name', 'prefill_s', d['prefill_s'], 'tok/s', d['value'])"
}
run llama31_70b_32k --model llama-3.1-70b --prompt-len 32768
run llama31_70b_127k --model llama-3.1-70b --prompt-len 130048
run mistral_7b_32k --model mistral-7b --prompt-len 32768
