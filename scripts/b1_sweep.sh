#!/bin/bash
# Llama-3-70B batch-1 decode on one GPU for bf16, fp8 and LLM.int8 weights (bench.py, no profiler)
set -u
mkdir -p gpurun_out/b1
for mode in bf16 fp8 int8; do
  flag=""
  [ "$mode" = fp8 ] && flag="--fp8"
  [ "$mode" = int8 ] && flag="--int8"
  timeout -k 10 300 python3 -u bench.py $flag --batch-per-mb 1 --steps 20 --warmup 3 --json-out gpurun_out/b1/${mode}_b1.json > gpurun_out/b1/${mode}_b1.log 2>&1 || { tail -20 gpurun_out/b1/${mode}_b1.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b1/${mode}_b1.json'));print('$mode b1', d['value'], 'tok/s', d['ms_per_step'], 'ms')"
done
