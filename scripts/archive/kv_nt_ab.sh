#!/bin/bash
# Interleaved same-box A/B: non-temporal K/V loads in bf16 single-split decode (DLI_KV_NT) after
# the decode-attention load-pipeline fix.
set -u
mkdir -p gpurun_out/kvnt
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --json-out gpurun_out/kvnt/$tag.json > gpurun_out/kvnt/$tag.log 2>&1 || { tail -20 gpurun_out/kvnt/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/kvnt/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run nt0_a DLI_KV_NT=0 && run nt1_a DLI_KV_NT=1 && run nt0_b DLI_KV_NT=0 && run nt1_b DLI_KV_NT=1 && run nt0_c DLI_KV_NT=0 && run nt1_c DLI_KV_NT=1
