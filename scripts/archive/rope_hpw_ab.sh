#!/bin/bash
# RoPE / KV-write kernel with 16 instead of 8 heads per workgroup (DLI_ROPE_HPW): bit-identity
# tests, then interleaved same-box bench.py A/B (default config).
set -u
mkdir -p gpurun_out/rope
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rope" > gpurun_out/rope/tests.log 2>&1 || { tail -30 gpurun_out/rope/tests.log; exit 1; }
tail -1 gpurun_out/rope/tests.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 -u bench.py --json-out gpurun_out/rope/$tag.json > gpurun_out/rope/$tag.log 2>&1 || { tail -20 gpurun_out/rope/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/rope/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run h8_a DLI_ROPE_HPW=8 && run h16_a DLI_ROPE_HPW=16 && run h8_b DLI_ROPE_HPW=8 && run h16_b DLI_ROPE_HPW=16 && run h8_c DLI_ROPE_HPW=8 && run h16_c DLI_ROPE_HPW=16
