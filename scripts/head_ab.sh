#!/bin/bash
# LM head at M = 512 (N = 128256): hipBLASLt (default) vs the gemm4 tile path (DLI_GEMM_LIB=0),
# bench.py back to back, interleaved twice
set -u
mkdir -p gpurun_out/head_ab
for rep in 1 2; do
  for arm in lib tile; do
    if [ $arm = tile ]; then export DLI_GEMM_LIB=0; else export DLI_GEMM_LIB=1; fi
    timeout -k 10 400 python3 -u bench.py --json-out gpurun_out/head_ab/${arm}_$rep.json > gpurun_out/head_ab/${arm}_$rep.log 2>&1 || { tail -20 gpurun_out/head_ab/${arm}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/head_ab/${arm}_$rep.json'));print('$arm', $rep, d['value'], d['ms_per_step'])"
  done
done
