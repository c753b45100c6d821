#!/bin/bash
# Throughput envelope on one GPU (70B bf16, PP=1): micro-batch 1024 / 768 at a 256-token prompt
# next to the default 512 x 512 (informational; the headline config stays 512 x 512)
set -o pipefail
mkdir -p gpurun_out/envelope
run() {
  local name=$1; shift
  timeout -k 10 500 python -u bench.py "$@" --json-out gpurun_out/envelope/$name.json > gpurun_out/envelope/$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/envelope/$name.log; exit 1; }
  echo "$name $(python -c "import json;d=json.load(open('gpurun_out/envelope/$name.json'));print(d['value'], d['ms_per_step'], d['kv_blocks'], d['kv_blocks_needed'])")"
}
run b512_p256 --batch-per-mb 512 --prompt-len 256
run b768_p256 --batch-per-mb 768 --prompt-len 256
run b1024_p256 --batch-per-mb 1024 --prompt-len 256
