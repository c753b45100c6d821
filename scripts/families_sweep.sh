# bench.py on the other Llama-family presets (one GPU, one micro-batch of 512, random init)
set -u
mkdir -p gpurun_out/results
export TMPDIR=/tmp
for m in mistral-7b qwen2-7b llama-3.1-8b; do
  timeout -k 10 600 python -u bench.py --model $m --json-out gpurun_out/results/${m}_bf16_b512.json > gpurun_out/results/${m}.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/results/${m}.log; exit 1; }
  echo "$m $(python -c "import json;d=json.load(open('gpurun_out/results/${m}_bf16_b512.json'));print(d['value'], 'tok/s', d['ms_per_step'], 'ms/step')")"
done
