#!/bin/bash
# Prefill attention with scalar block-table loads: prefill tests, then the prefill-attention
# microbench old (ab_old/) vs new interleaved, then the decode-layer probe.
set -u
mkdir -p gpurun_out/pfab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "prefill or mask" > gpurun_out/pfab/tests.log 2>&1 || { tail -30 gpurun_out/pfab/tests.log; exit 1; }
tail -1 gpurun_out/pfab/tests.log
for i in 1 2; do
  (cd ab_old && timeout -k 10 300 python3 -u scripts/attn_prefill_bench.py > $GRAFT_REPO_ROOT/gpurun_out/pfab/old$i.txt 2>&1) || { tail -5 gpurun_out/pfab/old$i.txt; exit 1; }
  echo "old$i"; grep "{" gpurun_out/pfab/old$i.txt
  timeout -k 10 300 python3 -u scripts/attn_prefill_bench.py > gpurun_out/pfab/new$i.txt 2>&1 || { tail -5 gpurun_out/pfab/new$i.txt; exit 1; }
  echo "new$i"; grep "{" gpurun_out/pfab/new$i.txt
done
timeout -k 10 300 python3 -u scripts/decode_layer_probe.py fp8 > gpurun_out/pfab/dl_probe_fp8.txt 2>&1 || { tail -5 gpurun_out/pfab/dl_probe_fp8.txt; exit 1; }
cat gpurun_out/pfab/dl_probe_fp8.txt
