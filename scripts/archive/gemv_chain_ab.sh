#!/bin/bash
# Chained batch-1 GEMVs (gate|up -> down in one launch, DLI_GEMV_CHAIN): bit-identity tests, then
# interleaved same-box batch-1 benches (fp8, int8).
set -u
mkdir -p gpurun_out/chain
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemv_chain or skinny" > gpurun_out/chain/tests.log 2>&1 || { tail -30 gpurun_out/chain/tests.log; exit 1; }
tail -1 gpurun_out/chain/tests.log
run() {  # tag flag env...
  local tag=$1 flag=$2; shift 2
  env "$@" timeout -k 10 300 python3 -u bench.py $flag --batch-per-mb 1 --steps 20 --warmup 3 --json-out gpurun_out/chain/$tag.json > gpurun_out/chain/$tag.log 2>&1 || { tail -20 gpurun_out/chain/$tag.log; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/chain/$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
}
run fp8_c0a --fp8 DLI_GEMV_CHAIN=0 && run fp8_c1a --fp8 DLI_GEMV_CHAIN=1 && run fp8_c0b --fp8 DLI_GEMV_CHAIN=0 && run fp8_c1b --fp8 DLI_GEMV_CHAIN=1 && run int8_c0 --int8 DLI_GEMV_CHAIN=0 && run int8_c1 --int8 DLI_GEMV_CHAIN=1
