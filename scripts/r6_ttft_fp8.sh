# long-context TTFT with fp8 weights + fp8 KV (Llama-3.1-70B, batch 1, 127k-token prompt)
set -u
out=gpurun_out/r6ttft
mkdir -p $out
export TMPDIR=/tmp
L=130048
timeout -k 10 600 python -u bench.py --model llama-3.1-70b --fp8 --kv-fp8 --batch-per-mb 1 --prompt-len $L --steps 5 --warmup 2 --json-out $out/ttft_fp8_fp8kv_$L.json > $out/ttft_fp8_fp8kv_$L.log 2>&1 || { tail -20 $out/ttft_fp8_fp8kv_$L.log; exit 1; }
python -c "import json; d=json.load(open('$out/ttft_fp8_fp8kv_$L.json')); print($L, 'prefill_s', d['prefill_s'], 'tok/s', d['value'])"
