# Round-3 GPU round AN: long-context decode on one GPU - Llama-3.1-70B (llama3 rope scaling),
# batch 1 with a 127k-token prompt (chunked prefill, split-K decode attention over 127k keys)
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --model llama-3.1-70b --batch-per-mb 1 --prompt-len 130048 --steps 10 --warmup 3 \
    --json-out gpurun_out/results/llama31_70b_bf16_b1_ctx127k.json > gpurun_out/results/llama31_70b_bf16_b1_ctx127k.log 2>&1 \
    || { tail -30 gpurun_out/results/llama31_70b_bf16_b1_ctx127k.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/results/llama31_70b_bf16_b1_ctx127k.json'));print(d['value'], d['ms_per_step'], d['prefill_s'], d['kv_blocks'], d['kv_blocks_needed'])"
