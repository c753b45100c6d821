#!/bin/bash
# fp8 / int8 GEMV with 8 instead of 4 k-steps of weights in flight per wave (DLI_GEMV_UNROLL=8):
# numerics tests, GEMV stream rates, interleaved batch-1 benches.
set -u
mkdir -p gpurun_out/unroll
export TMPDIR=/tmp
DLI_GEMV_UNROLL=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "skinny or gemv or 8bit" > gpurun_out/unroll/tests.log 2>&1 || { tail -30 gpurun_out/unroll/tests.log; exit 1; }
tail -1 gpurun_out/unroll/tests.log
DLI_GEMV_UNROLL=4 timeout -k 10 300 python3 -u scripts/gemv_bw.py fp8 > gpurun_out/unroll/bw4.txt 2>&1 || { tail -5 gpurun_out/unroll/bw4.txt; exit 1; }
DLI_GEMV_UNROLL=8 timeout -k 10 300 python3 -u scripts/gemv_bw.py fp8 > gpurun_out/unroll/bw8.txt 2>&1 || { tail -5 gpurun_out/unroll/bw8.txt; exit 1; }
grep fp8 gpurun_out/unroll/bw4.txt gpurun_out/unroll/bw8.txt
run() {  # tag flag env...
  local tag=$1 flag=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $flag --batch-per-mb 1 --steps 20 --warmup 3 --json-out gpurun_out/unroll/$tag.json > gpurun_out/unroll/$tag.log 2>&1 || { tail -20 gpurun_out/unroll/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/unroll/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run fp8_u4a --fp8 DLI_GEMV_UNROLL=4 && run fp8_u8a --fp8 DLI_GEMV_UNROLL=8 && run fp8_u4b --fp8 DLI_GEMV_UNROLL=4 && run fp8_u8b --fp8 DLI_GEMV_UNROLL=8 && run int8_u4 --int8 DLI_GEMV_UNROLL=4 && run int8_u8 --int8 DLI_GEMV_UNROLL=8
